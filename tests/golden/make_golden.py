"""Generate golden vectors by running the REFERENCE training step on CPU.

Runs only in the build container, where the read-only reference is mounted at
/root/reference (it never travels to the GPU box).  Recipe = SURVEY.md §8(c):
empty stub modules for the unused top-level imports (torchvision, cv2, wandb),
``args.beta1 = float(args.beta1)``, G/D built without ``.cuda``, weights set
with ``load_state_dict`` from tests/golden/gen_inputs.py, ``load_next_batch``
and ``torch.randn`` fed the same synthetic inputs, then the reference's own
``ProgressiveGAN.train_step`` (pggan/model.py:206-255) is called.

Output: tests/golden/<config>.npz  (inputs are NOT stored: they are regenerated
from the seeds; outputs, losses, gradients and post-Adam parameters are).

Usage:  python tests/golden/make_golden.py [config-name ...]
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
from gen_inputs import GOLDEN_CONFIGS, make_inputs, make_params  # noqa: E402
from oracle.pggan_oracle import PAPER_DEPTHS, d_param_shapes, g_param_shapes  # noqa: E402

REF = "/root/reference"
N_SAMPLES = 96  # sampled elements per tensor for the non-full configs
FULL_MAX = 65536  # larger tensors are stored as samples + L2 norm


def import_reference():
    for n in ["torchvision", "torchvision.utils", "torchvision.transforms",
              "torchvision.models", "cv2", "wandb"]:
        sys.modules.setdefault(n, types.ModuleType(n))
    tv = sys.modules["torchvision"]
    tv.utils = sys.modules["torchvision.utils"]
    tv.transforms = sys.modules["torchvision.transforms"]
    tv.models = sys.modules["torchvision.models"]
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import lib.loss as ref_loss
    import lib.utils as ref_utils
    from lib.config import Config
    from pggan.loss import WGANGPLoss
    from pggan.model import ProgressiveGAN
    from pggan.nets import Discriminator, Generator
    return dict(Config=Config, ProgressiveGAN=ProgressiveGAN, Generator=Generator,
                Discriminator=Discriminator, WGANGPLoss=WGANGPLoss, loss=ref_loss,
                utils=ref_utils)


def sample_idx(n, seed):
    rng = np.random.default_rng(seed)
    k = min(n, N_SAMPLES)
    return np.sort(rng.choice(n, size=k, replace=False)).astype(np.int64)


def run_config(R, name, depths, s, B, alpha, n_steps, full):
    depths = list(depths or PAPER_DEPTHS)
    torch.manual_seed(0)
    args = R["Config"].from_yaml(os.path.join(REF, "configs.yaml"))
    args.beta1 = float(args.beta1)
    args.isMaster = False
    args.depths = depths
    args.batch_per_gpu = B

    m = object.__new__(R["ProgressiveGAN"])
    m.args = args
    m.gpu = "cpu"
    m.scale_index = s
    G = R["Generator"](args.latent_dim, depths[0], args.init_bias_to_zero, args.LReLU_slope,
                       args.apply_pixel_norm, args.generator_last_activation, args.output_dim,
                       args.equalized_lr)
    D = R["Discriminator"](depths[0], args.init_bias_to_zero, args.LReLU_slope,
                           args.decision_layer_size, args.apply_minibatch_norm, args.input_dim,
                           args.equalized_lr)
    for i in range(1, s + 1):
        G.add_block(depths[i])
        D.add_block(depths[i])
    gsh, dsh = g_param_shapes(depths, s), d_param_shapes(depths, s)
    # pin the oracle's parameter naming / shapes to the reference's state_dict
    assert [(k, tuple(v.shape)) for k, v in G.state_dict().items()] == gsh, "G mismatch"
    assert [(k, tuple(v.shape)) for k, v in D.state_dict().items()] == dsh, "D mismatch"
    PG = make_params(gsh, seed=1000 + 10 * s + B)
    PD = make_params(dsh, seed=2000 + 10 * s + B)
    G.load_state_dict({k: torch.from_numpy(v) for k, v in PG.items()})
    D.load_state_dict({k: torch.from_numpy(v) for k, v in PD.items()})
    G.alpha = alpha
    D.alpha = alpha
    m.G, m.D = G, D
    m.set_optimizers()
    m._loss_collector = R["WGANGPLoss"](args)

    res = 4 * 2 ** s
    steps = make_inputs(B, res, seed=3000 + 10 * s + B, n_steps=n_steps)
    rec = {}
    batch_q, randn_q = [], []
    m.load_next_batch = lambda: batch_q.pop(0)

    real_randn = torch.randn

    def fake_randn(*a, **k):
        if randn_q and tuple(a) == tuple(randn_q[0].shape):
            return randn_q.pop(0).clone()
        return real_randn(*a, **k)

    orig_r1 = R["loss"].Loss.get_r1_reg

    def r1_rec(d_out, x_in):
        v = orig_r1(d_out, x_in)
        rec["R1"] = float(v)
        return v

    orig_update = R["utils"].update_net

    def update_rec(opt, loss):
        opt.zero_grad()
        loss.backward()
        which = "D" if opt is m.opt_D else "G"
        net = m.D if which == "D" else m.G
        rec["grads_" + which] = {k: (None if p.grad is None else p.grad.detach().clone())
                                 for k, p in net.named_parameters()}
        opt.step()

    lc = m._loss_collector
    orig_lD, orig_lG = lc.get_loss_D, lc.get_loss_G

    def lD(D_dict):
        rec["pred_real"] = D_dict["pred_real"].detach().clone()
        rec["pred_fake"] = D_dict["pred_fake"].detach().clone()
        rec["img_real"] = D_dict["img_real"].detach().clone()
        rec["img_fake_D"] = D_dict["img_fake"].detach().clone()
        return orig_lD(D_dict)

    def lG(G_dict):
        rec["pred_fake_G"] = G_dict["pred_fake"].detach().clone()
        return orig_lG(G_dict)

    lc.get_loss_D, lc.get_loss_G = lD, lG
    R["loss"].Loss.get_r1_reg = staticmethod(r1_rec)
    R["utils"].update_net = update_rec
    torch.randn = fake_randn
    out = {}
    try:
        for t, st in enumerate(steps):
            batch_q.append(torch.from_numpy(st["real"]))
            randn_q.extend([torch.from_numpy(st["z1"]), torch.from_numpy(st["z2"])])
            rec.clear()
            img_real, img_fake = m.train_step()
            assert not batch_q and not randn_q
            pre = f"s{t}/"
            ld = lc.loss_dict
            out[pre + "losses"] = np.array([ld["L_D_real"], ld["L_D_fake"], rec["R1"], ld["L_D"],
                                            ld["L_G"]], np.float64)
            tensors = {"img_real": rec["img_real"], "img_fake_D": rec["img_fake_D"],
                       "img_fake_G": img_fake.detach(), "pred_real": rec["pred_real"],
                       "pred_fake": rec["pred_fake"], "pred_fake_G": rec["pred_fake_G"]}
            for k, v in tensors.items():
                out[pre + k] = v.numpy().astype(np.float32)
            for net, P in (("G", m.G), ("D", m.D)):
                for k, g in rec["grads_" + net].items():
                    key = f"{pre}grad_{net}/{k}"
                    if g is None:
                        out[key + "#none"] = np.zeros(0, np.float32)
                        continue
                    _store(out, key, g, full)
                for k, p in P.named_parameters():
                    _store(out, f"{pre}param_{net}/{k}", p.detach(), False)
    finally:
        torch.randn = real_randn
        R["loss"].Loss.get_r1_reg = staticmethod(orig_r1)
        R["utils"].update_net = orig_update
    meta = dict(name=name, depths=depths, s=s, B=B, alpha=alpha, n_steps=n_steps, full=full)
    out["meta"] = np.frombuffer(repr(meta).encode(), dtype=np.uint8)
    return out


def _store(out, key, t, full):
    a = t.numpy().astype(np.float32)
    if full and a.size <= FULL_MAX:
        out[key] = a
    else:
        flat = a.reshape(-1)
        idx = sample_idx(flat.size, seed=flat.size)
        out[key + "#idx"] = idx
        out[key + "#val"] = flat[idx]
        out[key + "#norm"] = np.array([np.linalg.norm(flat.astype(np.float64))])


# WGAN-GP optional mode (dead code in the reference): fixtures from the reference's own
# get_gradient_penalty / get_drift_loss (pggan/loss.py:54-100), SURVEY §8(c) recipe incl.
# the Tensor.get_device patch (pggan/loss.py:73 calls .get_device(), -1 on CPU)
GP_CONFIGS = [  # (name, depths, s, B, alpha)
    ("gp_tiny_s2_b8_a03", "tiny", 2, 8, 0.3),
    ("gp_tiny_s1_b4_a05", "tiny", 1, 4, 0.5),
]


def run_gp(R, name, depths, s, B, alpha):
    from gen_inputs import TINY_DEPTHS
    depths = list(TINY_DEPTHS if depths == "tiny" else depths)
    torch.manual_seed(0)
    args = R["Config"].from_yaml(os.path.join(REF, "configs.yaml"))
    args.beta1 = float(args.beta1)
    args.isMaster = False
    args.depths = depths
    G = R["Generator"](args.latent_dim, depths[0], args.init_bias_to_zero, args.LReLU_slope,
                       args.apply_pixel_norm, args.generator_last_activation, args.output_dim,
                       args.equalized_lr)
    D = R["Discriminator"](depths[0], args.init_bias_to_zero, args.LReLU_slope,
                           args.decision_layer_size, args.apply_minibatch_norm, args.input_dim,
                           args.equalized_lr)
    for i in range(1, s + 1):
        G.add_block(depths[i])
        D.add_block(depths[i])
    gsh, dsh = g_param_shapes(depths, s), d_param_shapes(depths, s)
    PG = make_params(gsh, seed=1000 + 10 * s + B)
    PD = make_params(dsh, seed=2000 + 10 * s + B)
    G.load_state_dict({k: torch.from_numpy(v) for k, v in PG.items()})
    D.load_state_dict({k: torch.from_numpy(v) for k, v in PD.items()})
    G.alpha = D.alpha = alpha
    lc = R["WGANGPLoss"](args)
    st = make_inputs(B, 4 * 2 ** s, seed=3000 + 10 * s + B)[0]
    real = torch.from_numpy(st["real"])
    if s:   # the real-image fade of train_step (pggan/model.py:217-221)
        low = torch.nn.functional.interpolate(torch.nn.functional.avg_pool2d(real, (2, 2)),
                                              scale_factor=2, mode="nearest")
        real = (1 - alpha) * low + alpha * real
    img_real = real.detach().clone().requires_grad_()
    pred_real = D(img_real)
    with torch.no_grad():
        img_fake = G(torch.from_numpy(st["z1"]))
    D_dict = {"img_real": img_real, "img_fake": img_fake.detach(), "pred_real": pred_real}
    eps = torch.from_numpy(st["gp_eps"])
    real_rand, real_gd = torch.rand, torch.Tensor.get_device
    torch.rand = lambda *a, **k: eps.clone()
    torch.Tensor.get_device = lambda self: "cpu"
    try:
        D.zero_grad()
        gp = lc.get_gradient_penalty(D_dict, D, backward=True)
        grads = {k: (None if p.grad is None else p.grad.detach().clone())
                 for k, p in D.named_parameters()}
        drift = lc.get_drift_loss(D_dict)
    finally:
        torch.rand, torch.Tensor.get_device = real_rand, real_gd
    out = {"gp": np.array([gp], np.float64), "drift": np.array([drift], np.float64),
           "W_gp": np.array([float(args.W_gp)]), "W_drift_D": np.array([float(args.W_drift_D)]),
           "img_real": img_real.detach().numpy().astype(np.float32),
           "img_fake": img_fake.numpy().astype(np.float32),
           "pred_real": pred_real.detach().numpy().astype(np.float32)}
    for k, g in grads.items():
        if g is None:
            out[f"grad_D/{k}#none"] = np.zeros(0, np.float32)
        else:
            out[f"grad_D/{k}"] = g.numpy().astype(np.float32)
    meta = dict(name=name, depths=depths, s=s, B=B, alpha=alpha)
    out["meta"] = np.frombuffer(repr(meta).encode(), dtype=np.uint8)
    return out


SCHEDULE_ARGS = dict(max_step_at_scale=[5, 7, 9, 9], alpha_jump_start=[-1, 2, 3, 1],
                     alpha_jump_interval=[0, 1, 2, 1], alpha_jump_Ntimes=[0, 3, 2, 4],
                     depths=[8, 8, 8, 8])


def run_schedule(R, n_steps=30):
    """The reference's progressive schedule (pggan/model.py:141-204 driven as in
    train.py:27-45) with G/D/solver stubbed: per step (scale_index, alpha_G, alpha_D,
    alpha_index, next_alpha_jump_step, next_scale_jump_step)."""
    args = R["Config"].from_yaml(os.path.join(REF, "configs.yaml"))
    args.isMaster = False
    for k, v in SCHEDULE_ARGS.items():
        setattr(args, k, v)

    class Net:
        alpha = 0

        def add_block(self, d):
            pass

        def cuda(self):
            return self

    m = object.__new__(R["ProgressiveGAN"])
    m.args, m.gpu, m.G, m.D = args, "cpu", Net(), Net()
    m.reset_solver = lambda: None
    m.alpha, m.alpha_index, m.scale_index, m.alpha_jump_value = 0, 0, 0, 0
    m.next_scale_jump_step = args.max_step_at_scale[0]
    m.next_alpha_jump_step = args.alpha_jump_start[0]
    rows = []
    for step in range(n_steps):
        m.check_jump(step)
        rows.append([m.scale_index, m.G.alpha, m.D.alpha, m.alpha_index, m.next_alpha_jump_step,
                     m.next_scale_jump_step])
    return np.array(rows, np.float64)


def main(names):
    R = import_reference()
    if not names or "schedule" in names:
        np.savez_compressed(os.path.join(HERE, "schedule.npz"), rows=run_schedule(R),
                            meta=np.frombuffer(repr(SCHEDULE_ARGS).encode(), dtype=np.uint8))
        print("schedule: written")
    for (name, depths, s, B, alpha) in GP_CONFIGS:
        if names and name not in names:
            continue
        out = run_gp(R, name, depths, s, B, alpha)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **out)
        print(f"{name}: GP {float(out['gp'][0]):.6e} drift {float(out['drift'][0]):.6e}, "
              f"{os.path.getsize(path) / 1e6:.2f} MB")
    for (name, depths, s, B, alpha, n_steps, full) in GOLDEN_CONFIGS:
        if names and name not in names:
            continue
        out = run_config(R, name, depths, s, B, alpha, n_steps, full)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **out)
        print(f"{name}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main(sys.argv[1:])
