"""The reference's Python surface on the HIP kernels:

* f4  Generator.forward / Discriminator.forward (pggan/nets.py:121-161, 248-276) against
      the oracle (fp32 mode to 1e-4, bf16 storage to 3e-2).
* f2  ProgressiveGAN.check_jump driving two change_scale transitions and alpha ramps
      (pggan/model.py:141-204) with a fresh Adam per stage, every train_step checked
      against the oracle replayed (float64, the step's own leaky-ReLU region choices)
      from the model's state before the step: every D and G gradient within 1e-3,
      parameters after both Adam steps within 1e-5.
"""
import pytest
import torch

import kink_parity as K
from gen_inputs import TINY_DEPTHS
from oracle import pggan_oracle as O
from test_model_api import _forward_check, make_args

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2)],
                         ids=["f32", "bf16"])
def test_module_forward_on_hip(dtype, tol):
    from pggan_amd import nets
    nets.OPS_FACTORY = None
    nets._ENGINES.clear()
    _forward_check(device="cuda", dtype=dtype, tol=tol)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-3), (torch.bfloat16, 5e-2)],
                         ids=["f32", "bf16"])
def test_modules_differentiable_on_hip(dtype, tol):
    """The autograd path of the modules (first-order backward on the HIP kernels) against
    the oracle's autograd, with the forwards' region choices injected."""
    from pggan_amd import nets
    from test_model_api import _autograd_check
    nets.OPS_FACTORY = None
    nets._ENGINES.clear()
    _autograd_check(device="cuda", dtype=dtype, tol=tol)


def test_progressive_transitions_on_hip(tmp_path):
    from pggan_amd import nets
    from pggan_amd.model import ProgressiveGAN
    nets.OPS_FACTORY = None
    ProgressiveGAN.ops_factory = None
    args = make_args(tmp_path, max_step_at_scale=[2, 2, 3, 3], alpha_jump_start=[-1, 0, 1, 1],
                     alpha_jump_interval=[0, 1, 1, 1], alpha_jump_Ntimes=[0, 2, 2, 2],
                     depths=list(TINY_DEPTHS))
    torch.manual_seed(5)
    m = ProgressiveGAN(args, 0)
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
    seen = []
    for step in range(6):
        m.check_jump(step)
        s, aG, aD = m.scale_index, float(m.G.alpha), float(m.D.alpha)
        seen.append((s, aG))
        B = args.batch_per_gpu
        eng = m._engine(B)
        PG0 = {k: v.detach().cpu().double().clone() for k, v in m.G.state_dict().items()}
        PD0 = {k: v.detach().cpu().double().clone() for k, v in m.D.state_dict().items()}
        optG = K._adam_state(m.fpG, m.hyper.lr_G, m.hyper, torch.float64)
        optD = K._adam_state(m.fpD, m.hyper.lr_D, m.hyper, torch.float64)
        rec = K.Recorder()
        eng.trace = rec
        m.train_step()
        m.flush()
        eng.trace = None
        real = m.synthetic.detach().cpu().double()
        z1, z2 = m._z[0].detach().cpu().double(), m._z[1].detach().cpu().double()
        ref = O.train_step(PG0, PD0, optG, optD, real, z1, z2, s, aG, aD, kinks=rec.seq)
        rep = K.flip_report(rec.seq)
        assert max(v[2] for v in rep.values()) <= K.FLIP_BOUND[torch.float32], rep
        for net, grads, P in (("D", ref.grads_D, m.D), ("G", ref.grads_G, m.G)):
            named = dict(P.named_parameters())
            for k, g in grads.items():
                if g is None:
                    continue
                e = K.rel_l2(named[k].grad.detach().cpu(), g)
                assert e <= 1e-3 or float(g.norm()) == 0.0, (step, net, k, e)
        # parameters after both Adam steps: 1e-5 relative or within 1e-3 of the step size
        # (zero-initialised biases are O(lr); see test_model_api.test_train_step_is_reference_step)
        for P, R, lr in ((m.D, PD0, m.hyper.lr_D), (m.G, PG0, m.hyper.lr_G)):
            for k, v in P.state_dict().items():
                a = v.detach().cpu().double()
                assert K.rel_l2(a, R[k]) <= 1e-5 or float((a - R[k]).abs().max()) <= 1e-3 * lr, \
                    (step, k)
    # two stage transitions and an alpha ramp happened
    assert [x[0] for x in seen] == [0, 0, 1, 1, 2, 2]
    assert any(0.0 < x[1] < 1.0 for x in seen)
