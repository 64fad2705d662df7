"""Debug: run the same D passes with HipOps (GPU, fp32) and the CPU test double on
identical inputs at a full-width stage and print the relative error of every engine
buffer after each pass."""
import sys
sys.path[:0] = ['.', 'tests', 'tests/golden']
import torch
from cpu_ops import CpuOps
from gen_inputs import make_inputs
from golden_utils import rel_l2
from test_engine_cpu import build
from oracle import pggan_oracle as O
from pggan_amd import _lib
torch.set_num_threads(16)
s, B, a = int(sys.argv[1]), 4, float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
meta = dict(depths=O.PAPER_DEPTHS, s=s, B=B, alpha=a, n_steps=1)
st = make_inputs(B, 4 * 2 ** s, seed=3000 + 10 * s + B)[0]
runs = {}
for name, ops, dev in (("gpu", _lib.HipOps(torch.float32), "cuda"), ("cpu", CpuOps(), "cpu")):
    eng, fpG, fpD = build(meta, ops, device=dev)
    eng.pack("G", fpG.views); eng.pack("D", fpD.views)
    real = torch.from_numpy(st["real"]).to(dev)
    snaps = {}
    eng.d_forward(fpD.views, real, a)
    snaps["F"] = {k: v.detach().float().cpu().clone() for k, v in eng.dd.items()}
    ops.bce(eng.dd["logit"], True, 1.0, eng.loss[0:1], eng.dd["u"], eng.dd["hl"])
    eng.dd["gimg"].zero_()
    eng.d_backward(fpD.views, None, eng.dd["u"], a, gimg=eng.dd["gimg"])
    snaps["B1"] = {k: v.detach().float().cpu().clone() for k, v in eng.dd.items()}
    ops.r1_penalty(eng.dd["gimg"], B, eng.loss[2:3], eng.dd["gbar"])
    fpD.grad.zero_()
    tout, inj = eng.d_tangent(fpD.views, fpD.gviews, eng.dd["gbar"], eng.dd["u"], a)
    snaps["T"] = {k: v.detach().float().cpu().clone() for k, v in eng.dd.items()}
    snaps["Tgrad"] = {k: v.detach().float().cpu().clone() for k, v in fpD.gviews.items()}
    runs[name] = snaps
for ph in ("F", "B1", "T", "Tgrad"):
    errs = {k: rel_l2(runs["gpu"][ph][k].numpy(), runs["cpu"][ph][k].numpy())
            for k in runs["cpu"][ph]}
    print(ph, {k: f"{v:.1e}" for k, v in errs.items() if v > 1e-5})
