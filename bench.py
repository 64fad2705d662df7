"""Benchmark: images/sec of the full PGGAN G+D+R1 training step (BASELINE.json metric).

Workload (BASELINE configs[4] / SURVEY §8(d) C5): 1024x1024 stage (s=8), paper
depths [512,512,512,512,256,128,64,32,16], batch 4 per GPU, alpha = 1, R1
penalty, both Adam steps, bf16 storage with fp32 accumulation.  Synthetic data:
reals U[-1,1) resident in HBM, latents drawn on the GPU by the pg_randn kernel,
random-init weights (reference init: W ~ N(0,1), b = 0).

Launch:  python bench.py [--gpus N --steps K --warmup W]
         (N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
One process per GPU; gradients all-reduced (mean) over RCCL before each Adam step, the
exchange overlapped with the work that does not depend on it (engine.train_step).
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (G+D+GP step) at 1024×1024 bs=4/GPU, 1/2/4/8 MI355X"
PAPER_DEPTHS = [512, 512, 512, 512, 256, 128, 64, 32, 16]
# dense peaks, /opt/skills/guides/MI355X_MICROARCH.md (chip-level parameters)
PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}
PEAK_HBM_GBS = 8000.0
# minimal algorithmic GFLOP per image of the step (counted over the reference's
# own train_step incl. the double backward, without the discarded D wgrad of the G half)
STEP_GFLOP_PER_IMG = {5: 626.63, 6: 844.33, 7: 1062.29, 8: 1280.78}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--stage", type=int, default=8)
    p.add_argument("--batch", type=int, default=4)
    p.add_argument("--alpha", type=float, default=1.0)
    p.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    p.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-kernel-events", action="store_true")
    return p.parse_args()


def conv_bytes(x, wpk, y, kw):
    """Algorithmic HBM bytes of one conv3x3 launch: input (at its stored resolution), output
    (read too when accumulating), the mask operand, the second output, the input sign bits,
    packed weights -- each at its own element size (bf16 activations, uint8 sign bits)."""
    B, H, W, fl = kw["B"], kw["H"], kw["W"], kw["flags"]
    hin = H // 2 if fl & 1 else H
    ho = H // 2 if fl & 16 else H
    wo = W // 2 if fl & 16 else W
    n = B * hin * (W // 2 if fl & 1 else W) * x.shape[-1] * x.element_size()
    n += B * ho * wo * y.shape[-1] * y.element_size() * (2 if fl & 32 else 1)
    aux = kw.get("aux")
    if aux is not None:
        n += B * H * W * aux.shape[-1] * aux.element_size()
    y2 = kw.get("y2")
    if y2 is not None:
        n += B * H * W * y2.shape[-1] * y2.element_size() if y2.dim() == 4 and y2.shape[1] == H \
            else y2.numel() * y2.element_size()
    xb = kw.get("xbits")
    if xb is not None:
        n += B * H * W * xb.shape[-1] * xb.element_size()
    return n + wpk.numel() * wpk.element_size()


class KernelTimer:
    """HIP events around every conv launch (fwd/dgrad/tangent kernel and wgrad kernel),
    recorded on the stream the kernels run on; FLOPs are the algorithmic MAC count x2
    of the logical channels."""

    def __init__(self, ops, dtype):
        self.dtype = dtype
        self.rec = {"conv3x3": [], "wgrad3x3": []}
        self.shapes = []
        self.on = False
        f_conv, f_wg = ops.conv3x3, ops.conv_wgrad

        def conv3x3(x, wpk, y, **kw):
            if not self.on:
                return f_conv(x, wpk, y, **kw)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f_conv(x, wpk, y, **kw)
            b.record()
            fl = 2.0 * kw["B"] * kw["H"] * kw["W"] * 9 * kw["cin"] * kw["cout"]
            by = conv_bytes(x, wpk, y, kw)
            self.rec["conv3x3"].append((a, b, fl, by))
            self.shapes.append(("conv3x3", kw["H"], kw["cin"], kw["cout"], kw["flags"], a, b, fl,
                                by))

        def conv_wgrad(x, gz, dw, **kw):
            if not self.on:
                return f_wg(x, gz, dw, **kw)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f_wg(x, gz, dw, **kw)
            b.record()
            fl = 2.0 * kw["B"] * kw["H"] * kw["W"] * 9 * kw["cin"] * kw["cout"]
            hin = kw["H"] // 2 if kw["ups"] else kw["H"]
            by = (kw["B"] * hin * hin * x.shape[-1] + kw["B"] * kw["H"] * kw["W"] * gz.shape[-1]) \
                * x.element_size() + 2 * dw.numel() * 4
            self.rec["wgrad3x3"].append((a, b, fl, by))
            self.shapes.append(("wgrad3x3", kw["H"], kw["cin"], kw["cout"], int(kw["ups"]), a, b,
                                fl, by))

        ops.conv3x3, ops.conv_wgrad = conv3x3, conv_wgrad

    def per_shape(self, steps=1):
        agg = {}
        for k, H, ci, co, fl, a, b, f, by in self.shapes:
            key = (k, H, ci, co, fl)
            t = agg.setdefault(key, [0.0, 0.0, 0, 0.0])
            t[0] += a.elapsed_time(b)
            t[1] += f
            t[2] += 1
            t[3] += by
        rows = sorted(agg.items(), key=lambda kv: -kv[1][0])
        return [dict(kernel=k[0], H=k[1], cin=k[2], cout=k[3], flags=k[4],
                     ms_per_step=round(v[0] / steps, 3), tflops=round(v[1] / (v[0] * 1e-3) / 1e12, 1),
                     gbps=round(v[3] / (v[0] * 1e-3) / 1e9, 1),
                     calls_per_step=v[2] // steps) for k, v in rows]

    def peak_key(self, fam):
        # the f32 path and the f32-MFMA wgrad kernel run at the f32 MFMA rate
        return "f32" if self.dtype == "f32" else "bf16"

    def summary(self):
        out = {}
        for k, lst in self.rec.items():
            if not lst:
                continue
            pf = PEAK_TFLOPS[self.peak_key(k)] * 1e12
            ms = sum(a.elapsed_time(b) for a, b, _, _ in lst)
            fl = sum(f for _, _, f, _ in lst)
            by = sum(v for _, _, _, v in lst)
            # per-launch roofline time: max(flops / MFMA peak, bytes / HBM peak)
            roof_s = sum(max(f / pf, v / (PEAK_HBM_GBS * 1e9)) for _, _, f, v in lst)
            out[k] = dict(launches=len(lst), total_ms=ms, avg_us=1e3 * ms / len(lst),
                          flops=fl, bytes=by, tflops=fl / (ms * 1e-3) / 1e12,
                          gbps=by / (ms * 1e-3) / 1e9, roofline_time_frac=roof_s / (ms * 1e-3),
                          t_mfma_s=fl / pf, t_hbm_s=by / (PEAK_HBM_GBS * 1e9))
        return out


def init_params(E, depths, s, device, rank_seed):
    gsh, dsh = E.g_param_shapes(depths, s), E.d_param_shapes(depths, s)
    gen = torch.Generator().manual_seed(1234)   # same init on every rank (then broadcast)
    init = lambda sh: {k: (torch.randn(v, generator=gen) if k.endswith("weight")
                           else torch.zeros(v)) for k, v in sh}
    fpG = E.FlatParams(gsh, E.dead_params("G", s), device, init(gsh))
    fpD = E.FlatParams(dsh, E.dead_params("D", s), device, init(dsh))
    return fpG, fpD


def pmc_traffic(args, fam):
    """HBM bytes per launch of `fam` from the newest committed rocprofv3 PMC summary of this
    same workload (profiles/*_prof_summary.json, written by tools/prof_summary.py from
    separate --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py, gfx950 FETCH x2 correction).
    PMC counters cannot be read inside the timed run, so this is the profiled twin's value."""
    import glob
    import re
    key = f"stage{args.stage}_b{args.batch}_{args.dtype}"

    def version(path):   # r<round>_v<n>: numeric order (r1_v10 is newer than r1_v9)
        return tuple(int(t) for t in re.findall(r"\d+", os.path.basename(path)))

    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_prof_summary.json")), key=version,
                    reverse=True):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        f = d.get("families", {}).get(fam, {})
        if d.get("config") == key and f.get("hbm_bytes_per_call"):
            return round(f["hbm_bytes_per_call"]), os.path.relpath(p, ROOT)
    return None, None


def cpu_baseline(args, steps=1):
    """The CPU oracle (fp32 restatement of the reference step, pinned to the reference's
    golden vectors) on the host cores: one train_step at the same workload."""
    from oracle import pggan_oracle as O
    torch.set_num_threads(args.cpu_threads)
    s, B = args.stage, args.batch
    depths = PAPER_DEPTHS
    gen = torch.Generator().manual_seed(7)
    PG = {k: (torch.randn(v, generator=gen) if k.endswith("weight") else torch.zeros(v))
          for k, v in O.g_param_shapes(depths, s)}
    PD = {k: (torch.randn(v, generator=gen) if k.endswith("weight") else torch.zeros(v))
          for k, v in O.d_param_shapes(depths, s)}
    R = 4 * 2 ** s
    real = torch.rand(B, 3, R, R, generator=gen) * 2 - 1
    optG, optD = O.AdamState(1e-4), O.AdamState(1e-5)
    t0 = time.perf_counter()
    for _ in range(steps):
        z1 = torch.randn(B, 512, generator=gen)
        z2 = torch.randn(B, 512, generator=gen)
        O.train_step(PG, PD, optG, optD, real, z1, z2, s, args.alpha, args.alpha)
    dt = time.perf_counter() - t0
    return dict(value=B * steps / dt, unit="images/sec", cores=args.cpu_threads, kind="port",
                sample=f"{steps} oracle train_step at {R}x{R}, batch {B}, alpha {args.alpha} "
                       f"(fp32, torch CPU, {args.cpu_threads} threads): {dt:.1f} s")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    # PG_DIST_BACKEND=gloo + ranks sharing a GPU: a rehearsal of the N>1 path on a 1-GPU box
    backend = os.environ.get("PG_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % ndev if backend != "nccl" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from pggan_amd import _lib
    from pggan_amd import engine as E

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    ops = _lib.HipOps(dtype)
    timer = None if args.no_kernel_events else KernelTimer(ops, args.dtype)
    s, B = args.stage, args.batch
    depths = PAPER_DEPTHS
    R = 4 * 2 ** s
    fpG, fpD = init_params(E, depths, s, dev, rank)
    if world > 1:   # replaces DDP's constructor-time broadcast (lib/model.py:78-79)
        dist.broadcast(fpG.flat, 0)
        dist.broadcast(fpD.flat, 0)
    eng = E.StepEngine(ops, depths, s, B, dev)
    eng.bind(fpG, fpD, E.Hyper())
    gen = torch.Generator(device=dev).manual_seed(1000 * rank)
    real = torch.rand(B, 3, R, R, device=dev, generator=gen) * 2 - 1
    z = torch.empty(2, B, 512, device=dev)

    class Pending:
        """Async RCCL all-reduce of a net's flat live gradient; the engine waits (and the
        mean is applied) right before that net's Adam step, so the exchange overlaps the
        work that does not depend on it (engine.train_step)."""

        def __init__(self, g):
            self.g, self.work = g, dist.all_reduce(g, async_op=True)

        def wait(self):
            self.work.wait()
            self.g.mul_(1.0 / world)

    def hook(net, g):
        return Pending(g) if world > 1 else None

    step_no = [0]

    def step():
        ops.randn(z, 1000 * rank + 17, step_no[0] * z.numel())
        step_no[0] += 1
        eng.train_step(real, z[0], z[1], args.alpha, args.alpha, grad_hook=hook)

    for _ in range(args.warmup):
        step()
    eng.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        # per-launch HIP events on the conv kernels during the last timed step only: each
        # event pair costs ~7 us of GPU time, so instrumenting every step would cost ~10 %
        # of the throughput being measured
        if timer:
            timer.on = i == args.steps - 1
        step()
    eng.flush()          # the last step's (deferred) generator update is part of the step
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if timer:
        timer.on = False
    # host-side cost of enqueueing one step (kernels are not waited for): if this is close
    # to ms_per_step the step is launch-bound, not GPU-bound
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    for _ in range(2):
        step()
    eng.flush()
    host_ms = (time.perf_counter() - h0) * 1e3 / 2
    torch.cuda.synchronize()
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    assert torch.isfinite(eng.loss).all(), "non-finite loss"
    ksum = timer.summary() if timer else {}
    if timer and os.environ.get("PG_BENCH_SHAPES"):
        with open(os.environ["PG_BENCH_SHAPES"], "w") as f:
            json.dump(timer.per_shape(1), f, indent=1)

    if rank == 0:
        roof = None
        if ksum:
            dom = max(ksum, key=lambda k: ksum[k]["total_ms"])
            kd = ksum[dom]
            hbm = kd["t_hbm_s"] > kd["t_mfma_s"]
            if hbm:
                ach, peak, unit = kd["gbps"], PEAK_HBM_GBS, "GB/s"
            else:
                ach, peak, unit = kd["tflops"], PEAK_TFLOPS[timer.peak_key(dom)], "TFLOP/s"
            traffic, tsrc = pmc_traffic(args, dom)
            roof = dict(bound="hbm" if hbm else "mfma", kernel=dom, achieved=round(ach, 2),
                        peak=peak, unit=unit, frac=round(ach / peak, 4), traffic=traffic,
                        traffic_source=tsrc,
                        algorithmic_bytes_per_launch=round(kd["bytes"] / kd["launches"]),
                        flops_per_launch=round(kd["flops"] / kd["launches"]),
                        launches_per_step=kd["launches"],
                        avg_launch_us=round(kd["avg_us"], 2),
                        roofline_time_frac=round(kd["roofline_time_frac"], 4),
                        # whole-step MFMA fraction at the minimal algorithmic
                        # 1280.78 GFLOP per image (C5), all kernels, wall clock
                        step_mfma_frac=round(STEP_GFLOP_PER_IMG.get(args.stage, 0.0) * 1e9 *
                                             B * args.steps / dt /
                                             (PEAK_TFLOPS[args.dtype] * 1e12), 4),
                        kernels={k: dict(total_ms_per_step=round(v["total_ms"], 3),
                                         tflops=round(v["tflops"], 2), gbps=round(v["gbps"], 1),
                                         roofline_time_frac=round(v["roofline_time_frac"], 4),
                                         launches_per_step=v["launches"])
                                 for k, v in ksum.items()})
        cpu = None
        if args.cpu_baseline == "auto" and world == 1:
            cpu = cpu_baseline(args)
        line = {
            "metric": METRIC,
            "value": round(B * world * args.steps / dt, 3),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (U[-1,1) reals resident in HBM, N(0,1) latents on GPU, "
                    "random-init weights)",
            "config": {"workload": f"C5 G+D+R1 train_step, stage {s} ({R}x{R}), batch {B}/GPU, "
                                   f"alpha {args.alpha}, depths {depths}",
                       "global_batch": B * world, "resolution": R,
                       "parallelism": f"dp{world}"},
            "host_enqueue_ms_per_step": round(host_ms, 3),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
