"""Checkpoint interoperability with the reference itself.

Runs only in the build container, where the reference is importable (SURVEY §8(c)
recipe, tests/golden/make_golden.import_reference); skipped elsewhere.

* reference -> pggan_amd: the reference's own ProgressiveGAN trains one step at stage 1
  and writes {save_root}/{run_id}/ckpt/{G,D}_{step,latest}.pt with its own
  save_checkpoint (pggan/model.py:50-67, lib/checkpoint.py:22-34); pggan_amd's
  load_checkpoint restores bit-identical parameters, Adam moments / step counts and the
  schedule scalars.
* pggan_amd -> reference: pggan_amd's save_checkpoint output is read back by the
  reference's own load_checkpoint (pggan/model.py:70-101) into a fresh reference model:
  bit-identical parameters and optimizer state.  (The reference hard-codes
  map_location='cuda' and .cuda() calls; on this CPU container they are redirected to
  the CPU for the duration of the call.)
"""
import os

import numpy as np
import pytest
import torch

from cpu_ops import CpuOps
from gen_inputs import TINY_DEPTHS, make_inputs, make_params
from pggan_amd import nets
from pggan_amd.model import ProgressiveGAN
from test_model_api import make_args

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "pggan")),
                                reason="the reference is importable only in the build container")


@pytest.fixture(autouse=True)
def _cpu_ops(monkeypatch):
    monkeypatch.setattr(ProgressiveGAN, "ops_factory", staticmethod(CpuOps))
    monkeypatch.setattr(nets, "OPS_FACTORY", CpuOps)


def _ref_model(R, tmp_path, run_id, s, ckpt_id=None):
    args = R["Config"].from_yaml(os.path.join(REF, "configs.yaml"))
    args.beta1 = float(args.beta1)
    args.isMaster = False
    args.depths = list(TINY_DEPTHS)
    args.batch_per_gpu = 4
    args.save_root = str(tmp_path)
    args.run_id = run_id
    args.ckpt_id = ckpt_id
    args.ckpt_step = None
    m = object.__new__(R["ProgressiveGAN"])
    m.args, m.gpu, m.scale_index = args, "cpu", s
    m.G = R["Generator"](args.latent_dim, TINY_DEPTHS[0], args.init_bias_to_zero, args.LReLU_slope,
                         args.apply_pixel_norm, args.generator_last_activation, args.output_dim,
                         args.equalized_lr)
    m.D = R["Discriminator"](TINY_DEPTHS[0], args.init_bias_to_zero, args.LReLU_slope,
                             args.decision_layer_size, args.apply_minibatch_norm, args.input_dim,
                             args.equalized_lr)
    for net in (m.G, m.D):     # the reference calls .cuda() after add_block (CPU here)
        net.cuda = (lambda n: (lambda *a, **k: n))(net)
    for i in range(1, s + 1):
        m.G.add_block(TINY_DEPTHS[i])
        m.D.add_block(TINY_DEPTHS[i])
    m.set_optimizers()
    m._loss_collector = R["WGANGPLoss"](args)
    m.alpha_index, m.alpha_jump_value = 1, 0.5
    m.next_alpha_jump_step, m.next_scale_jump_step = 9, 12
    return m


def test_checkpoints_interoperate_with_the_reference(tmp_path, monkeypatch):
    from make_golden import import_reference
    R = import_reference()
    import lib.checkpoint as ref_ckpt
    # ---- reference trains one step at stage 1 and saves
    torch.manual_seed(3)
    mr = _ref_model(R, tmp_path, "ref", 1)
    PG = make_params([(k, tuple(v.shape)) for k, v in mr.G.state_dict().items()], seed=41)
    PD = make_params([(k, tuple(v.shape)) for k, v in mr.D.state_dict().items()], seed=42)
    mr.G.load_state_dict({k: torch.from_numpy(v) for k, v in PG.items()})
    mr.D.load_state_dict({k: torch.from_numpy(v) for k, v in PD.items()})
    mr.G.alpha = mr.D.alpha = 0.5
    st = make_inputs(4, 8, seed=43)[0]
    mr.load_next_batch = lambda: torch.from_numpy(st["real"])
    mr.train_step()
    mr.save_checkpoint(7)
    assert sorted(os.listdir(tmp_path / "ref" / "ckpt")) == ["D_7.pt", "D_latest.pt", "G_7.pt",
                                                               "G_latest.pt"]
    # ---- pggan_amd resumes from it
    args = make_args(tmp_path, ckpt_id="ref", ckpt_step=None)
    ma = ProgressiveGAN(args, "cpu")
    ma.initialize_models()
    ma.set_optimizers()
    ma.set_dataset()
    ma.set_data_iterator()
    ma.set_loss_collector()
    ma.load_checkpoint()
    assert (ma.scale_index, ma.global_step, ma.alpha_index, ma.alpha_jump_value,
            ma.next_alpha_jump_step, ma.next_scale_jump_step) == (1, 7, 1, 0.5, 9, 12)
    assert ma.G.alpha == 0.5 and ma.D.alpha == 0.5
    for a, b in ((mr.G, ma.G), (mr.D, ma.D)):
        sa, sb = a.state_dict(), b.state_dict()
        assert list(sa) == list(sb)
        for k in sa:
            assert torch.equal(sa[k], sb[k]), k
    for opt_r, opt_a in ((mr.opt_G, ma.opt_G), (mr.opt_D, ma.opt_D)):
        ra, aa = opt_r.state_dict()["state"], opt_a.state_dict()["state"]
        assert set(ra) == set(aa)
        for i in ra:
            assert float(ra[i]["step"]) == float(aa[i]["step"])
            for k in ("exp_avg", "exp_avg_sq"):
                assert torch.equal(ra[i][k], aa[i][k]), (i, k)
    # ---- pggan_amd saves, the reference's own load_checkpoint reads it back
    ma.args.run_id = "ours"
    ma.save_checkpoint(11)
    mb = _ref_model(R, tmp_path, "reader", 0, ckpt_id="ours")
    mb.reset_solver = mb.set_optimizers          # its dataset half needs torchvision
    real_load = torch.load
    monkeypatch.setattr(ref_ckpt.torch, "load",
                        lambda p, map_location=None, **k: real_load(p, map_location="cpu", **k))
    mb.load_checkpoint()
    assert mb.scale_index == 1 and mb.global_step == 11
    for a, b in ((ma.G, mb.G), (ma.D, mb.D)):
        sa, sb = a.state_dict(), b.state_dict()
        assert list(sa) == list(sb)
        for k in sa:
            assert torch.equal(sa[k].cpu(), sb[k]), k
    for opt_a, opt_b in ((ma.opt_G, mb.opt_G), (ma.opt_D, mb.opt_D)):
        sa, sb = opt_a.state_dict()["state"], opt_b.state_dict()["state"]
        assert set(sa) == set(sb)
        for i in sa:
            for k in ("exp_avg", "exp_avg_sq"):
                assert torch.equal(sa[i][k].cpu(), sb[i][k]), (i, k)
    assert np.isclose(mb.opt_D.param_groups[0]["lr"], ma.opt_D.lr)
