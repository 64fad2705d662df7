"""Data-parallel contract on the GPU: two ranks on the one GPU of the box,
gloo process group, HipOps kernels, the product path's bucketed asynchronous exchange
(pggan_amd.dp.GradExchange hooked into the engine exactly as ProgressiveGAN does).

Contract (tests/test_dp_gloo.py states it on the CPU double): the DP D gradient equals the
mean over ranks of the single-process reference D gradient on each rank's shard (NOT one
global-batch step: R1 scales as 1/B^2), and parameters and G gradients are bit-identical
across ranks after both Adam steps.  The per-shard reference is the float64 oracle replayed
with that rank's leaky-ReLU region choices (tests/kink_parity.py), so every D tensor is
held to 1e-3.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gen_inputs import TINY_DEPTHS, make_inputs, make_params

pytestmark = pytest.mark.gpu

S, B, ALPHA = 2, 4, 0.5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, reduce_bf16=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), here, os.path.join(here, "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import kink_parity as K
    from oracle import pggan_oracle as O
    from pggan_amd import _lib
    from pggan_amd import engine as E
    from pggan_amd.dp import GradExchange
    torch.cuda.set_device(0)
    gsh, dsh = E.g_param_shapes(TINY_DEPTHS, S), E.d_param_shapes(TINY_DEPTHS, S)
    PG = {k: torch.from_numpy(v) for k, v in make_params(gsh, seed=801).items()}
    PD = {k: torch.from_numpy(v) for k, v in make_params(dsh, seed=802).items()}
    fpG = E.FlatParams(gsh, E.dead_params("G", S), "cuda", PG)
    fpD = E.FlatParams(dsh, E.dead_params("D", S), "cuda", PD)
    eng = E.StepEngine(_lib.HipOps(torch.float32), TINY_DEPTHS, S, B, "cuda")
    eng.bind(fpG, fpD, E.Hyper())
    ex = GradExchange(world, bucket_bytes=64 << 10,   # small buckets: several per net
                      reduce_dtype=torch.bfloat16 if reduce_bf16 else torch.float32)
    ex.bind("G", fpG)
    ex.bind("D", fpD)
    eng.grad_ready = ex.ready
    rec = K.Recorder()
    eng.trace = rec
    st = make_inputs(B, 4 * 2 ** S, seed=900 + rank)[0]
    real, z1, z2 = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2"))
    eng.train_step(real.cuda(), z1.cuda(), z2.cuda(), ALPHA, ALPHA, grad_hook=ex.hook)
    eng.flush()
    torch.cuda.synchronize()
    eng.trace = None
    # this shard's single-process reference D gradient (float64, this rank's kinks)
    P64 = lambda P: {k: v.double() for k, v in P.items()}
    ref = O.train_step(P64(PG), P64(PD), O.AdamState(1e-4), O.AdamState(1e-5), real.double(),
                       z1.double(), z2.double(), S, ALPHA, ALPHA, kinks=rec.seq)
    gD_ref = np.zeros(fpD.numel, np.float64)
    for k, g in ref.grads_D.items():
        if g is not None:
            o = fpD.offsets[k]
            gD_ref[o:o + g.numel()] = g.numpy().ravel()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), gD=fpD.grad.cpu().numpy(),
             gG=fpG.grad.cpu().numpy(), pD=fpD.flat.cpu().numpy(), pG=fpG.flat.cpu().numpy(),
             gD_ref=gD_ref, n_live=fpD.n_live)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("reduce", ["f32", "bf16"])
def test_dp_two_ranks_on_hip_kernels(tmp_path, reduce):
    """reduce = bf16 (dp_reduce_dtype): each rank's gradient is rounded to bf16 before the
    sum, so the mean is held to 1e-2 of the addends' L2 norm (2^-8 rounding per addend)
    instead of 1e-3 of the result's."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), reduce == "bf16"), nprocs=world,
             join=True)
    r = [np.load(tmp_path / f"rank{i}.npz") for i in range(world)]
    for k in ("gD", "gG", "pD", "pG"):
        assert np.array_equal(r[0][k], r[1][k]), f"{k} differs across ranks"
    from pggan_amd import engine as E
    dsh = E.d_param_shapes(TINY_DEPTHS, S)
    fpD = E.FlatParams(dsh, E.dead_params("D", S), "cpu")
    ref = sum(x["gD_ref"] for x in r) / world
    for n in fpD.names:
        if n in fpD.dead:
            continue
        lo, hi = fpD.offsets[n], fpD.offsets[n] + int(np.prod(fpD.shapes[n]))
        a, b = r[0]["gD"][lo:hi].astype(np.float64), ref[lo:hi]
        if reduce == "bf16":
            # the rounding is of each rank's addend (and of the bf16 sum): measured against the
            # addends' magnitude, since a mean of opposite-signed terms (a bias gradient) can
            # cancel to far below them
            scale = sum(np.abs(x["gD_ref"][lo:hi]) for x in r) / world
            err = np.linalg.norm(a - b) / max(np.linalg.norm(scale), 1e-30)
        else:
            err = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
        assert err <= (1e-2 if reduce == "bf16" else 1e-3), (n, err)
