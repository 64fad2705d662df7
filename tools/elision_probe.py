"""Run-to-run spread of the alpha = 1 elision check (test_engine_cpu.elision_bitwise) on HIP:
prints the relative L2 difference per step and tensor (images, loss, D/G grads, D/G params)
between the elided and computed fade-in branches.  python tools/elision_probe.py [dtype] [s]"""
import sys
sys.path[:0] = ["tests", "tests/golden", "."]
import torch
from pggan_amd import _lib, engine as E
from gen_inputs import make_inputs, make_params
from oracle import pggan_oracle as O

dt = torch.bfloat16 if (sys.argv[1:2] or ["bf16"])[0] == "bf16" else torch.float32
s = int((sys.argv[2:3] or ["6"])[0])
depths, B = O.PAPER_DEPTHS, 4
out = []
for elide in (False, True):
    gsh, dsh = E.g_param_shapes(depths, s), E.d_param_shapes(depths, s)
    PG = {k: torch.from_numpy(v) for k, v in make_params(gsh, seed=61).items()}
    PD = {k: torch.from_numpy(v) for k, v in make_params(dsh, seed=62).items()}
    fpG = E.FlatParams(gsh, E.dead_params("G", s), "cuda", PG)
    fpD = E.FlatParams(dsh, E.dead_params("D", s), "cuda", PD)
    eng = E.StepEngine(_lib.HipOps(dt), depths, s, B, "cuda")
    eng.elide_zero_blend = elide
    eng.bind(fpG, fpD, E.Hyper())
    eng.keep_fake_D = True
    res = []
    for t, st in enumerate(make_inputs(B, 4 * 2 ** s, seed=63, n_steps=2)):
        r, z1, z2 = (torch.from_numpy(st[k]).to("cuda") for k in ("real", "z1", "z2"))
        ims = eng.train_step(r, z1, z2, 1.0, 1.0)
        eng.flush()
        res.append([x.detach().cpu().clone() for x in ims] +
                   [eng.loss.cpu().clone(), fpD.grad.cpu().clone(), fpG.grad.cpu().clone(),
                    fpD.flat.cpu().clone(), fpG.flat.cpu().clone()])
    out.append(res)
names = ["img_real", "img_fake_D", "img_fake_G", "loss", "gD", "gG", "pD", "pG"]
for t, (a, b) in enumerate(zip(*out)):
    print(t, " ".join(f"{n}={float((x.double() - y.double()).norm() / max(float(y.double().norm()), 1e-30)):.1e}"
                      for n, x, y in zip(names, a, b)), flush=True)
