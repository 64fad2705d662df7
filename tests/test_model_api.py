"""Host-side API of the drop-in (pggan_amd.nets / pggan_amd.model) on CPU.

The kernels are replaced by the CPU test double (tests/cpu_ops.py) through the
`ops_factory` / `OPS_FACTORY` seams, so this checks the reference interface
itself: module state_dict keys and shapes (pggan/nets.py), the progressive
schedule against the reference's own schedule run (tests/golden/schedule.npz,
made by tests/golden/make_golden.py from pggan/model.py:141-204), checkpoint
round trips in the reference file layout (lib/checkpoint.py), and that
ProgressiveGAN.train_step is the reference step (oracle, pggan/model.py:206-255).
"""
import ast
import os

import numpy as np
import pytest
import torch

from gen_inputs import TINY_DEPTHS
from golden_utils import GOLDEN, rel_l2

from cpu_ops import CpuOps
from oracle import pggan_oracle as O
from pggan_amd import engine as E
from pggan_amd import nets
from pggan_amd.config import Config
from pggan_amd.model import ProgressiveGAN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _cpu_ops(monkeypatch):
    monkeypatch.setattr(ProgressiveGAN, "ops_factory", staticmethod(CpuOps))
    monkeypatch.setattr(nets, "OPS_FACTORY", CpuOps)
    nets._ENGINES.clear()


def make_args(tmp_path, **over):
    a = Config.from_yaml(os.path.join(ROOT, "pggan_amd", "default_config.yaml"))
    a.update(depths=list(TINY_DEPTHS), batch_per_gpu=4, compute_dtype="f32",
             save_root=str(tmp_path), run_id="t", isMaster=False, dataset_root_list=[],
             synthetic_data=True)
    a.update(over)
    return a


def fresh_model(args):
    m = ProgressiveGAN(args, "cpu")
    m.initialize_models()
    m.set_optimizers()
    m.set_dataset()
    m.set_data_iterator()
    m.set_loss_collector()
    m.scale_index = 0
    m.alpha_index = 0
    m.alpha_jump_value = 0
    m.next_scale_jump_step = args.max_step_at_scale[0]
    m.next_alpha_jump_step = args.alpha_jump_start[0]
    return m


@pytest.mark.parametrize("s", [0, 1, 2, 3])
def test_state_dict_matches_reference_layout(s):
    """Key order and shapes == the reference state_dict (oracle shapes are cited against
    pggan/nets.py and pinned by the golden fixtures' gradient keys)."""
    G = nets.Generator(512, TINY_DEPTHS[0])
    D = nets.Discriminator(TINY_DEPTHS[0], apply_minibatch_norm=True)
    for i in range(1, s + 1):
        G.add_block(TINY_DEPTHS[i])
        D.add_block(TINY_DEPTHS[i])
    g = [(k, tuple(v.shape)) for k, v in G.state_dict().items()]
    d = [(k, tuple(v.shape)) for k, v in D.state_dict().items()]
    assert g == [(k, tuple(v)) for k, v in O.g_param_shapes(TINY_DEPTHS, s)]
    assert d == [(k, tuple(v)) for k, v in O.d_param_shapes(TINY_DEPTHS, s)]


def test_unsupported_switches_raise():
    with pytest.raises(NotImplementedError):
        nets.Generator(512, 8, equalized_lr=False)
    with pytest.raises(NotImplementedError):
        nets.Discriminator(8, apply_minibatch_norm=False)


def test_schedule_matches_reference(tmp_path):
    z = np.load(os.path.join(GOLDEN, "schedule.npz"), allow_pickle=False)
    sched = ast.literal_eval(bytes(z["meta"]).decode())
    ref = z["rows"]
    args = make_args(tmp_path, batch_per_gpu=2, **sched)
    m = fresh_model(args)
    rows = []
    for step in range(ref.shape[0]):
        m.check_jump(step)
        rows.append([m.scale_index, m.G.alpha, m.D.alpha, m.alpha_index, m.next_alpha_jump_step,
                     m.next_scale_jump_step])
        # the nets grow with the schedule
        assert len(m.G.blocks) == m.scale_index and len(m.D.blocks) == m.scale_index
    np.testing.assert_allclose(np.array(rows, np.float64), ref, rtol=0, atol=1e-12)


def test_train_step_is_reference_step(tmp_path):
    """One ProgressiveGAN.train_step at stage 1, alpha 0.5 == oracle train_step on the
    same parameters, reals and latents (latents read back from the model), replayed in
    float64 with the engine's leaky-ReLU region choices (tests/kink_parity.py)."""
    import kink_parity as K
    args = make_args(tmp_path)
    m = fresh_model(args)
    m.change_scale(0)
    m.G.alpha = m.D.alpha = 0.5
    PG0 = {k: v.detach().double().clone() for k, v in m.G.state_dict().items()}
    PD0 = {k: v.detach().double().clone() for k, v in m.D.state_dict().items()}
    rec = K.Recorder()
    m._engine(args.batch_per_gpu).trace = rec
    img_real, img_fake = m.train_step()
    real = m.synthetic.clone().double()
    z1, z2 = m._z[0].clone().double(), m._z[1].clone().double()
    ref = O.train_step(PG0, PD0, O.AdamState(args.lr_G), O.AdamState(args.lr_D), real, z1, z2,
                       1, 0.5, 0.5, kinks=rec.seq)
    L = m.loss_collector.loss_dict
    assert abs(L["L_D_real"] - round(ref.L_D_real, 4)) <= 2e-4
    assert abs(L["L_D_fake"] - round(ref.L_D_fake, 4)) <= 2e-4
    assert abs(L["L_G"] - round(ref.L_G, 4)) <= 2e-4
    assert rel_l2(img_real.numpy(), ref.img_real.numpy()) < 1e-6
    assert rel_l2(img_fake.numpy(), ref.img_fake_G.numpy()) < 1e-5
    for net, grads in ((m.D, ref.grads_D), (m.G, ref.grads_G)):
        for k, g in grads.items():
            if g is None:
                continue
            got = dict(net.named_parameters())[k].grad
            assert rel_l2(got.numpy(), g.numpy()) < 1e-3, k
    # parameters after both Adam steps: 1e-5 relative, or within 1e-3 of the Adam step
    # size lr (zero-initialised biases are O(lr) after one step, and beta1 = 0 makes the
    # step lr * g / (|g| + eps): last-bit differences of |g| ~ eps move it by ~1e-5 lr)
    for net, P0, lr in ((m.D, PD0, args.lr_D), (m.G, PG0, args.lr_G)):
        for k, p in P0.items():
            got = dict(net.named_parameters())[k].detach().numpy()
            assert rel_l2(got, p.numpy()) < 1e-5 or \
                float(np.abs(got - p.numpy()).max()) <= 1e-3 * lr, k


def test_checkpoint_round_trip(tmp_path):
    """save_checkpoint -> load_checkpoint (reference paths/keys, weights_only load) restores
    parameters, Adam moments and schedule scalars; the next step is then identical."""
    args = make_args(tmp_path, max_step_at_scale=[2, 5, 5], alpha_jump_start=[-1, 0, 0],
                     alpha_jump_interval=[0, 1, 1], alpha_jump_Ntimes=[0, 4, 4])
    m = fresh_model(args)
    for step in range(4):
        m.check_jump(step)
        m.train_step()
    m.save_checkpoint(3)
    ck = os.path.join(str(tmp_path), "t", "ckpt")
    assert sorted(os.listdir(ck)) == ["D_3.pt", "D_latest.pt", "G_3.pt", "G_latest.pt"]
    sd = torch.load(os.path.join(ck, "G_latest.pt"), weights_only=True)
    for k in ("args", "global_step", "alpha_G", "alpha_D", "alpha_index", "alpha_jump_value",
              "next_alpha_jump_step", "scale_index", "next_scale_jump_step", "model",
              "optimizer"):
        assert k in sd, k
    assert list(sd["model"].keys()) == list(m.G.state_dict().keys())

    args2 = make_args(tmp_path, ckpt_id="t", max_step_at_scale=[2, 5, 5],
                      alpha_jump_start=[-1, 0, 0], alpha_jump_interval=[0, 1, 1],
                      alpha_jump_Ntimes=[0, 4, 4])
    m2 = ProgressiveGAN(args2, "cpu")
    m2.initialize_models()
    m2.set_optimizers()
    m2.set_dataset()
    m2.set_data_iterator()
    m2.set_loss_collector()
    m2.load_checkpoint()
    assert (m2.scale_index, m2.G.alpha, m2.alpha_index, m2.next_alpha_jump_step,
            m2.next_scale_jump_step, m2.global_step) == \
        (m.scale_index, m.G.alpha, m.alpha_index, m.next_alpha_jump_step,
         m.next_scale_jump_step, 3)
    for a, b in ((m.G, m2.G), (m.D, m2.D)):
        for (k, p), (k2, p2) in zip(a.state_dict().items(), b.state_dict().items()):
            assert k == k2 and torch.equal(p, p2), k
    assert torch.equal(m.fpD.m, m2.fpD.m) and torch.equal(m.fpD.v, m2.fpD.v)
    assert m.fpD.step == m2.fpD.step and m.fpG.step == m2.fpG.step
    # one more step on both (same latents, same reals) gives the same parameters
    m2._rng_step = m._rng_step
    m.train_step()
    m2.train_step()
    for a, b in ((m.G, m2.G), (m.D, m2.D)):
        for (k, p), (_, p2) in zip(a.state_dict().items(), b.state_dict().items()):
            assert torch.allclose(p, p2, rtol=0, atol=0), k


def test_product_path_requires_hip_library(monkeypatch):
    """Without the seam the model binds the HIP library, which refuses CPU tensors: no
    silent CPU fallback."""
    monkeypatch.setattr(ProgressiveGAN, "ops_factory", None)
    from pggan_amd import _lib
    try:
        ops = _lib.HipOps(torch.float32)
    except (OSError, RuntimeError):
        return   # library absent: loading already fails loudly
    with pytest.raises((RuntimeError, ValueError, AssertionError)):
        ops.pixnorm(torch.zeros(4, 8), torch.zeros(4, 8), 8)


class _RefStyleConfig:
    """Behaves like the reference's lib/config.py Config: attribute reads of missing keys
    raise KeyError (lib/config.py:26-27), not AttributeError."""

    def __init__(self, d):
        self.__dict__.update(d)

    def __getattr__(self, k):
        return self.__dict__[k]

    def __setitem__(self, k, v):
        self.__dict__[k] = v


def test_accepts_reference_config_object(tmp_path):
    d = dict(make_args(tmp_path))
    for k in ("compute_dtype", "gp_mode", "W_gp"):   # keys the reference config lacks
        d.pop(k)
    m = fresh_model(_RefStyleConfig(d))
    assert m.dtype == torch.float32 and m.hyper.gp_mode == "r1"
    m.train_step()
    assert np.isfinite(m.loss_collector.loss_dict["L_D"])


def _forward_check(device="cpu", dtype=torch.float32, tol=1e-5, s=2, alpha=0.5, B=4):
    """Generator.forward / Discriminator.forward(get_feature=True) (pggan/nets.py:121-161,
    248-276) against the oracle on the same parameters and inputs."""
    from gen_inputs import make_inputs, make_params
    G = nets.Generator(512, TINY_DEPTHS[0]).to(device)
    D = nets.Discriminator(TINY_DEPTHS[0], apply_minibatch_norm=True).to(device)
    for i in range(1, s + 1):
        G.add_block(TINY_DEPTHS[i])
        D.add_block(TINY_DEPTHS[i])
    G.alpha = D.alpha = alpha
    G.compute_dtype = D.compute_dtype = dtype
    PG = {k: torch.from_numpy(v) for k, v in make_params(O.g_param_shapes(TINY_DEPTHS, s), 71).items()}
    PD = {k: torch.from_numpy(v) for k, v in make_params(O.d_param_shapes(TINY_DEPTHS, s), 72).items()}
    G.load_state_dict(PG)
    D.load_state_dict(PD)
    st = make_inputs(B, 4 * 2 ** s, seed=73)[0]
    z, x = torch.from_numpy(st["z1"]), torch.from_numpy(st["real"])
    with torch.no_grad():   # the sampling path (forward-only engine)
        img = G(z.to(device)).cpu()
    ref = O.generator_forward({k: v.double() for k, v in PG.items()}, z.double(), s, alpha)
    assert rel_l2(img.numpy(), ref.numpy()) <= tol
    with torch.no_grad():
        out, feat = D(x.to(device), get_feature=True)
    ro, rf = O.discriminator_forward({k: v.double() for k, v in PD.items()}, x.double(), s, alpha,
                                     get_feature=True)
    assert rel_l2(out.cpu().numpy(), ro.numpy()) <= tol
    assert rel_l2(feat.cpu().numpy(), rf.numpy()) <= tol
    return G, D


def test_module_forward_is_reference():
    G, D = _forward_check()
    # one forward-only engine per net, evicted when the net grows
    assert set(nets._ENGINES) == {"G", "D"}
    assert nets._ENGINES["G"][1].forward_only == "G" and "gy0" not in nets._ENGINES["G"][1].g
    G.add_block(TINY_DEPTHS[3])
    assert "G" not in nets._ENGINES


def test_bias_init_follows_reference():
    """init_bias_to_zero=False keeps nn.Conv2d / nn.Linear's default uniform bias
    (lib/layers.py:51-52 skips the zero fill)."""
    torch.manual_seed(0)
    G = nets.Generator(512, 32, init_bias_to_zero=False)
    b = G.first_block.block[0].module.bias if hasattr(G.first_block.block, "__getitem__") else \
        getattr(G.first_block.block, "0").module.bias
    bound = 1.0 / (32 * 9) ** 0.5
    assert float(b.abs().max()) <= bound and float(b.abs().max()) > 0.0
    G0 = nets.Generator(512, 32)
    assert float(G0.latent_format_layer.module.bias.abs().max()) == 0.0


def _autograd_check(device="cpu", dtype=torch.float32, tol=1e-4, s=2, alpha=0.5, B=4):
    """The modules are differentiable once, like the reference's (pggan/nets.py:121-161,
    248-276 under autograd): L = BCE(D(G(z)), 1) backpropagated through both nets gives
    the oracle's gradients for every G and D parameter (compared kink-tolerantly at tiny
    widths: a relative L2 bound, float64 oracle)."""
    from gen_inputs import make_inputs, make_params
    G = nets.Generator(512, TINY_DEPTHS[0]).to(device)
    D = nets.Discriminator(TINY_DEPTHS[0], apply_minibatch_norm=True).to(device)
    for i in range(1, s + 1):
        G.add_block(TINY_DEPTHS[i])
        D.add_block(TINY_DEPTHS[i])
    G.alpha = D.alpha = alpha
    G.compute_dtype = D.compute_dtype = dtype
    PG = {k: torch.from_numpy(v) for k, v in make_params(O.g_param_shapes(TINY_DEPTHS, s), 81).items()}
    PD = {k: torch.from_numpy(v) for k, v in make_params(O.d_param_shapes(TINY_DEPTHS, s), 82).items()}
    G.load_state_dict(PG)
    D.load_state_dict(PD)
    z = torch.from_numpy(make_inputs(B, 4 * 2 ** s, seed=83)[0]["z1"])
    import kink_parity as K
    img = G(z.to(device))
    out, _ = D(img, get_feature=True)
    assert img.requires_grad and out.requires_grad, (torch.is_grad_enabled(), img.requires_grad)
    # the forwards' leaky-ReLU region choices, injected into the oracle (kink_parity)
    kG = O.Kinks(K.g_masks(nets._ENGINES["Gtrain"][1]))
    kD = O.Kinks(K.d_masks(nets._ENGINES["Dtrain"][1]))
    L = torch.nn.functional.binary_cross_entropy_with_logits(out, torch.ones_like(out))
    L.backward()
    P64 = lambda P: {k: v.double().requires_grad_() for k, v in P.items()}
    RG, RD = P64(PG), P64(PD)
    ri = O.generator_forward(RG, z.double(), s, alpha, kinks=kG)
    # D sees our image (its value), the gradient flows into the oracle's G
    ri_ours = ri + (img.detach().cpu().double() - ri).detach()
    Lr = O.bce_logits(O.discriminator_forward(RD, ri_ours, s, alpha, kinks=kD), 1)
    Lr.backward()
    assert abs(float(L) - float(Lr)) <= tol * abs(float(Lr)) + 1e-6
    errs = {}
    for net, R in ((G, RG), (D, RD)):
        for k, p in net.named_parameters():
            if R[k].grad is None:
                assert p.grad is None, k
                continue
            errs[k] = rel_l2(p.grad.cpu().numpy(), R[k].grad.numpy())
    worst = max(errs.values())
    assert worst <= tol, sorted(errs.items(), key=lambda kv: -kv[1])[:4]
    # the double backward of the R1 penalty is not available through autograd
    x = img.detach().clone().requires_grad_()
    o = D(x)
    with pytest.raises(NotImplementedError):
        torch.autograd.grad(o.sum(), x, create_graph=True)
    return worst


def test_modules_are_differentiable():
    _autograd_check()
