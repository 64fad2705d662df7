"""Run-to-run reproducibility of the HIP training step: the same configuration run twice in
one process from the same parameters and inputs, every engine buffer and the flat
parameters / gradients compared BITWISE after each step; prints, per step, the buffers that
differ in schedule order (the first one is where the two runs diverge).
python tools/repro_probe.py [dtype=bf16] [s=6] [B=4] [steps=2] [runs=2] [elide=1]"""
import sys
sys.path[:0] = ["tests", "tests/golden", "."]
import torch
from pggan_amd import _lib, engine as E
from gen_inputs import make_inputs, make_params
from oracle import pggan_oracle as O

a = sys.argv[1:]
dt = torch.bfloat16 if (a[0:1] or ["bf16"])[0] == "bf16" else torch.float32
s = int((a[1:2] or ["6"])[0])
B = int((a[2:3] or ["4"])[0])
n_steps = int((a[3:4] or ["2"])[0])
n_runs = int((a[4:5] or ["2"])[0])
elide = (a[5:6] or ["1"])[0] != "0"
depths = O.PAPER_DEPTHS


def snapshot(eng, fpG, fpD):
    out = {}
    sets = [("g", eng.g2 if eng.g2 is not None else eng.g),
            ("d", eng.dd2 if eng.dd2 is not None else eng.dd)]
    for pre, dct in sets:
        for k, v in dct.items():
            if torch.is_tensor(v):
                out[f"{pre}.{k}"] = v.detach().clone().cpu()
    out["loss"] = eng.loss.cpu().clone()
    for n, fp in (("G", fpG), ("D", fpD)):
        out[f"grad{n}"] = fp.grad.cpu().clone()
        out[f"param{n}"] = fp.flat.cpu().clone()
    return out


def poison(byte):
    """Fill the caching allocator's free blocks with `byte` (a read of never-written
    torch.empty memory then shows up as that pattern), small and large pools."""
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    keep = [torch.full((1 << 30,), byte, dtype=torch.uint8, device="cuda") for _ in range(24)]
    keep += [torch.full((1 << 19,), byte, dtype=torch.uint8, device="cuda") for _ in range(512)]
    torch.cuda.synchronize()
    del keep


POISON = [int(x, 0) for x in __import__("os").environ.get("POISON", "").split(",") if x]

runs = []
for r in range(n_runs):
    if POISON:
        poison(POISON[r % len(POISON)])
    gsh, dsh = E.g_param_shapes(depths, s), E.d_param_shapes(depths, s)
    PG = {k: torch.from_numpy(v) for k, v in make_params(gsh, seed=61).items()}
    PD = {k: torch.from_numpy(v) for k, v in make_params(dsh, seed=62).items()}
    fpG = E.FlatParams(gsh, E.dead_params("G", s), "cuda", PG)
    fpD = E.FlatParams(dsh, E.dead_params("D", s), "cuda", PD)
    eng = E.StepEngine(_lib.HipOps(dt), depths, s, B, "cuda")
    eng.elide_zero_blend = elide
    eng.bind(fpG, fpD, E.Hyper())
    snaps = []
    for t, st in enumerate(make_inputs(B, 4 * 2 ** s, seed=63, n_steps=n_steps)):
        real, z1, z2 = (torch.from_numpy(st[k]).to("cuda") for k in ("real", "z1", "z2"))
        eng.train_step(real, z1, z2, 1.0, 1.0)
        eng.flush()
        torch.cuda.synchronize()
        snaps.append(snapshot(eng, fpG, fpD))
    runs.append(snaps)
    del eng
    torch.cuda.synchronize()

def by_param(fp, x, y):
    """Names of the parameters whose slice of a flat buffer differs (element counts)."""
    out = []
    for n in fp.names:
        o = fp.offsets[n]
        k = int(torch.tensor(fp.shapes[n]).prod())
        m = int((x[o:o + k] != y[o:o + k]).sum())
        if m:
            out.append(f"{n}[{m}]")
    return out


bad = 0
for r in range(1, n_runs):
    for t in range(n_steps):
        A, Bs = runs[0][t], runs[r][t]
        diffs = []
        for k in A:
            x, y = A[k], Bs[k]
            if not torch.equal(x.view(torch.uint8) if x.dtype != torch.uint8 else x,
                               y.view(torch.uint8) if y.dtype != torch.uint8 else y):
                xd, yd = x.double(), y.double()
                n = int((x != y).sum())
                rel = float((xd - yd).norm() / max(float(yd.norm()), 1e-30))
                diffs.append(f"{k}:{n}el,rel={rel:.1e}")
                if k[:4] in ("grad", "para") and n < 10 ** 6:
                    diffs.append("(" + " ".join(by_param(fpG if k[-1] == "G" else fpD, x, y)) + ")")
        bad += len(diffs)
        print(f"run0 vs run{r} step{t}: {'BITWISE EQUAL' if not diffs else ' '.join(diffs)}",
              flush=True)
print("REPRO", "OK" if bad == 0 else f"DIFF({bad})")
