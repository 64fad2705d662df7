"""Benchmark: images/sec of the full PGGAN G+D+R1 training step (BASELINE.json metric).

Workload (BASELINE configs[4] / SURVEY §8(d) C5): 1024x1024 stage (s=8), paper
depths [512,512,512,512,256,128,64,32,16], batch 4 per GPU, alpha = 1, R1
penalty, both Adam steps, bf16 storage with fp32 accumulation.  Synthetic data:
reals U[-1,1) resident in HBM, latents drawn on the GPU by the pg_randn kernel,
random-init weights (reference init: W ~ N(0,1), b = 0).

Launch:  python bench.py [--gpus N --steps K --warmup W]
         (N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
The timed step is ProgressiveGAN.train_step (the path train.py runs).  One process per
GPU; gradients all-reduced (mean) over RCCL in per-layer buckets as the backward
finishes them (pggan_amd.dp), overlapped with the work that does not depend on them
(engine.train_step).  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

# One process per GPU with the DP gradient exchange: RCCL's stream and the engine's two
# streams must not share a hardware queue (HIP's default is 4 per process): a collective's
# wait-on-event barrier in a shared queue stalls the compute kernels queued behind it
# (bench.py --dp-exchange at one rank: -16 % of the step with 4 queues, -4 % with 8 or 16,
# profiles/r3_dp_queues.txt; round 6: -2.0 % with 8, -2.2 % with 16, the plain step itself
# -0.75 % at 16, profiles/r6_dp_lines.txt).  Must be set before the HIP runtime starts.
if int(os.environ.get("WORLD_SIZE", "1")) > 1 or "--dp-exchange" in sys.argv:
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

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
CONFIG_NAME = {(5, 16): "C2", (6, 8): "C3", (7, 8): "C4", (8, 4): "C5"}


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
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="0: the process's CPU share (OMP_NUM_THREADS, else os.cpu_count())")
    p.add_argument("--gp-mode", choices=["r1", "wgan-gp"], default="r1")
    p.add_argument("--no-kernel-events", action="store_true")
    p.add_argument("--graph", action="store_true",
                   help="replay the step as a hipGraph from the second step on (one process)")
    p.add_argument("--eager", action="store_true",
                   help="enqueue every step from Python (default: the library's C++ replay of "
                        "the recorded step from the third step on, one process)")
    p.add_argument("--dp-exchange", action="store_true",
                   help="at one process: run the DP gradient exchange anyway (a one-rank RCCL "
                        "group), to measure the bookkeeping's cost against the plain step")
    p.add_argument("--dp-bucket-mb", type=float, default=64.0,
                   help="DP all-reduce bucket size (config dp_bucket_mb)")
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
        # timing events without the system-scope fence (pg_event_create(timing=1)): a torch
        # timing event writes back and invalidates every XCD's L2 at each record, so the
        # launch it brackets would start cold and ~6.5 us late
        # created here, before any timed step: ~0.5k events per instrumented step, and
        # creating them inside the step made the host the bottleneck of that step
        pool = [ops.event(timing=True) for _ in range(2048)]
        self.ev = lambda: pool.pop() if pool else ops.event(timing=True)

        def conv3x3(x, wpk, y, **kw):
            if not self.on:
                return f_conv(x, wpk, y, **kw)
            a, b = self.ev(), self.ev()
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
            a, b = self.ev(), self.ev()
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

        def rgb_conv(f):
            """conv3x3_rgbw / conv3x3_rgbd: the input-gradient conv with the fromRGB backward
            in its epilogue (no conv output stored; the image read or its gradient written)."""
            def g(x, wpk, **kw):
                if not self.on:
                    return f(x, wpk, **kw)
                a, b = self.ev(), self.ev()
                a.record()
                f(x, wpk, **kw)
                b.record()
                fl = 2.0 * kw["B"] * kw["H"] * kw["W"] * 9 * kw["cin"] * kw["cout"]
                img = kw.get("img") if kw.get("img") is not None else kw.get("gimg")
                by = (x.numel() * x.element_size() + wpk.numel() * wpk.element_size() +
                      kw["aux"].numel() * kw["aux"].element_size() +
                      (img.numel() * img.element_size() if isinstance(img, torch.Tensor) else 0))
                self.rec["conv3x3"].append((a, b, fl, by))
                self.shapes.append(("conv3x3", kw["H"], kw["cin"], kw["cout"], kw["flags"], a, b,
                                    fl, by))
            return g

        ops.conv3x3, ops.conv_wgrad = conv3x3, conv_wgrad
        if hasattr(ops, "conv3x3_rgbw"):
            ops.conv3x3_rgbw = rgb_conv(ops.conv3x3_rgbw)
            ops.conv3x3_rgbd = rgb_conv(ops.conv3x3_rgbd)

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

    def _launches(self):
        """(family, H, flops, bytes, ms, bound) per recorded launch; bound = the roofline
        that limits THIS launch: mfma if flops/peak >= bytes/HBM peak, else hbm."""
        pf = PEAK_TFLOPS[self.peak_key("")] * 1e12
        out = []
        for fam, H, ci, co, fl, a, b, f, by in self.shapes:
            bound = "mfma" if f / pf >= by / (PEAK_HBM_GBS * 1e9) else "hbm"
            out.append((fam, H, f, by, a.elapsed_time(b), bound))
        return out

    def summary(self):
        """Per (family, bound) group: launches, time, FLOPs, bytes, achieved rates, and the
        per-launch roofline fraction sum(max(t_mfma, t_hbm)) / sum(t)."""
        pf = PEAK_TFLOPS[self.peak_key("")] * 1e12
        groups = {}
        for fam, H, f, by, ms, bound in self._launches():
            g = groups.setdefault(f"{fam}/{bound}", dict(launches=0, total_ms=0.0, flops=0.0,
                                                         bytes=0.0, roof_s=0.0, bound=bound))
            g["launches"] += 1
            g["total_ms"] += ms
            g["flops"] += f
            g["bytes"] += by
            g["roof_s"] += max(f / pf, by / (PEAK_HBM_GBS * 1e9))
        for g in groups.values():
            t = g["total_ms"] * 1e-3
            g.update(avg_us=1e3 * g["total_ms"] / g["launches"], tflops=g["flops"] / t / 1e12,
                     gbps=g["bytes"] / t / 1e9, roofline_time_frac=g["roof_s"] / t)
        return groups

    def per_resolution(self):
        """The north star's view: per resolution of the conv / weight-gradient launches,
        achieved TFLOP/s and MFMA fraction, achieved GB/s and HBM fraction, and which
        roofline bounds the majority of that resolution's launch time."""
        pf = PEAK_TFLOPS[self.peak_key("")] * 1e12
        rows = {}
        for fam, H, f, by, ms, bound in self._launches():
            r = rows.setdefault(H, dict(ms=0.0, flops=0.0, bytes=0.0, ms_mfma=0.0, launches=0))
            r["ms"] += ms
            r["flops"] += f
            r["bytes"] += by
            r["launches"] += 1
            if bound == "mfma":
                r["ms_mfma"] += ms
        out = []
        for H in sorted(rows):
            r = rows[H]
            t = r["ms"] * 1e-3
            tf, gb = r["flops"] / t / 1e12, r["bytes"] / t / 1e9
            out.append(dict(res=H, launches=r["launches"], ms_per_step=round(r["ms"], 3),
                            bound="mfma" if r["ms_mfma"] >= 0.5 * r["ms"] else "hbm",
                            tflops=round(tf, 1), mfma_frac=round(tf * 1e12 / pf, 4),
                            gbps=round(gb, 1), hbm_frac=round(gb / PEAK_HBM_GBS, 4)))
        return out


def pmc_traffic(args, fam, launches):
    """HBM bytes per launch of `fam` from the newest committed rocprofv3 PMC summary of this
    same workload AND schedule (profiles/*_prof_summary.json, written by tools/prof_summary.py
    from separate --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py, gfx950 FETCH x2
    correction): the summary's call count of the group must equal this run's `launches` per
    step, so a profile of another schedule (other merges, other tiles) is never paired with
    the line.  PMC counters cannot be read inside the timed run, so this is the profiled
    twin's value."""
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
        f = d.get("groups", {}).get(fam, {})
        if d.get("config") == key and f.get("hbm_bytes_per_call") and f.get("calls") == launches:
            return round(f["hbm_bytes_per_call"]), os.path.relpath(p, ROOT)
    return None, None


def host_threads():
    """CPU threads this process may use: the pool sets OMP_NUM_THREADS to the box's CPU
    share (16 per GPU) while os.cpu_count() reports every logical CPU of the machine (256);
    oversubscribing that share made the baseline step run for minutes."""
    share = os.environ.get("OMP_NUM_THREADS")
    n = os.cpu_count() or 1
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return n


def cpu_baseline(args, steps=1):
    """The CPU oracle (fp32 restatement of the reference step, pinned to the reference's
    golden vectors) on the host cores: one train_step at the same workload, with
    torch.set_num_threads(<the process's CPU share>) (CPU-baseline plan)."""
    from oracle import pggan_oracle as O
    threads = args.cpu_threads or host_threads()
    torch.set_num_threads(threads)
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
    return dict(value=B * steps / dt, unit="images/sec", cores=threads, kind="port",
                host_cpu_count=os.cpu_count(), omp_num_threads=os.environ.get("OMP_NUM_THREADS"),
                sample=f"{steps} oracle train_step at {R}x{R}, batch {B}, alpha {args.alpha} "
                       f"(fp32, torch CPU, torch.set_num_threads({threads})): {dt:.1f} s")


def build_model(args, rank, local, world, ops_factory):
    """The product path train.py runs: ProgressiveGAN (pggan/model.py:11-265 interface)
    grown to the benchmark stage, reference init (W ~ N(0,1), b = 0), the resident
    synthetic batch (`synthetic_data`), RCCL gradient exchange when world > 1."""
    from pggan_amd.config import Config
    from pggan_amd.model import ProgressiveGAN
    cfg = Config.from_yaml(os.path.join(ROOT, "pggan_amd", "default_config.yaml"))
    cfg.update(depths=list(PAPER_DEPTHS), batch_per_gpu=args.batch, compute_dtype=args.dtype,
               synthetic_data=True, isMaster=False, use_mGPU=world > 1, gpu_num=world,
               run_id="bench", gp_mode=args.gp_mode,
               dp_exchange_world1=bool(args.dp_exchange and world == 1),
               dp_bucket_mb=args.dp_bucket_mb)
    ProgressiveGAN.ops_factory = ops_factory
    torch.manual_seed(1234)                      # same init on every rank (then broadcast)
    m = ProgressiveGAN(cfg, local)
    m.initialize_models()
    for i in range(1, args.stage + 1):           # pggan/model.py:158-169 add_block per stage
        m.G.add_block(PAPER_DEPTHS[i])
        m.D.add_block(PAPER_DEPTHS[i])
    m.scale_index = args.stage
    m.G.alpha = m.D.alpha = args.alpha
    if world > 1 or args.dp_exchange:
        m.set_multi_GPU()                        # RCCL, parameter broadcast, GradExchange
    m.set_optimizers()
    m.set_dataset()
    m.set_data_iterator()
    m.set_loss_collector()
    return m


def _engine_opts():
    from pggan_amd import engine
    return engine.engine_options()


class _host_breakdown:
    """PG_BENCH_HOSTLOG: host seconds of a replayed step split into the C++ launch segments
    and each kind of Python host action between them (the DP exchange's collectives, seals,
    waits), and the time outside the replay."""

    def __init__(self):
        from pggan_amd import model as M
        self.M, self.orig, self.t = M, M._Segments.replay, {}
        me = self

        def replay(seg):
            for x in seg.segs:
                t0 = time.perf_counter()
                if hasattr(x, "replay"):
                    x.replay()
                    k = "cpp segments"
                else:
                    x()
                    f = getattr(x, "func", x)
                    k = getattr(f, "__name__", "host action")
                d = me.t.setdefault(k, [0.0, 0])
                d[0] += time.perf_counter() - t0
                d[1] += 1
        M._Segments.replay = replay

    def restore(self):
        self.M._Segments.replay = self.orig


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
    elif args.dp_exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)

    from pggan_amd import _lib

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    ops = _lib.HipOps(dtype)
    timer = None if args.no_kernel_events else KernelTimer(ops, args.dtype)
    s, B = args.stage, args.batch
    depths = PAPER_DEPTHS
    R = 4 * 2 ** s
    model = build_model(args, rank, local, world, lambda dt: ops)

    def step():
        model.train_step()

    log = lambda m: print(f"[bench] {m}", file=sys.stderr, flush=True)
    log(f"stage {s} batch {B} world {world}: {args.warmup} warm-up steps")
    # --graph (one process): from the second step on, train_step replays the step captured
    # as a hipGraph (ProgressiveGAN.use_graph); off by default (slower on the GPU)
    model.use_graph = bool(args.graph)
    # the product default: the step recorded by the library and re-issued from C++ (pg_replay)
    # on the engine's own streams, under DP with the exchange's collectives and waits recorded
    # between the launch segments; --eager enqueues every step from Python
    model.use_replay = not args.eager and not args.graph
    for _ in range(args.warmup):
        step()
    model.flush()
    torch.cuda.synchronize()
    # host-side cost of enqueueing one step (kernels are not waited for): if this is close
    # to ms_per_step the step is launch-bound, not GPU-bound.  Measured on the steps the
    # timed loop runs (graph replays in one process), before it.
    # the first step after a flush starts without a deferred generator update (under DP a
    # different replay key, whose second occurrence records): one step first, so the two
    # measured below are the replays the timed loop runs
    step()
    hostparts = _host_breakdown() if os.environ.get("PG_BENCH_HOSTLOG") else None
    h0 = time.perf_counter()
    for _ in range(2):
        step()
    model.flush()
    host_ms = (time.perf_counter() - h0) * 1e3 / 2
    if hostparts is not None:
        hostparts.restore()
        log("host enqueue per step (ms): " + ", ".join(
            f"{k} {v[0] * 1e3 / 2:.3f} ({v[1] / 2:.1f}x)" for k, v in sorted(
                hostparts.t.items(), key=lambda kv: -kv[1][0])))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    replays0 = model.graph_replays
    t0 = time.perf_counter()
    hostlog = [] if os.environ.get("PG_BENCH_HOSTLOG") else None
    for i in range(args.steps):
        # per-launch HIP events on the conv kernels during the last timed step only: each
        # event pair costs ~7 us of GPU time, so instrumenting every step would cost ~10 %
        # of the throughput being measured.  That step runs eagerly (events around each
        # launch), the others are graph replays.
        if timer and i == args.steps - 1:
            timer.on = True
            model.use_graph = model.use_replay = False
        if hostlog is not None:
            hostlog.append(time.perf_counter())
        step()
    if hostlog is not None:   # when each step's host work started (ms from the first)
        log("host step starts (ms): " + " ".join(f"{1e3 * (t - hostlog[0]):.2f}" for t in hostlog))
    model.flush()        # the last step's (deferred) generator update is part of the step
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if timer:
        timer.on = False
    graph_steps = model.graph_replays - replays0
    # one more instrumented step (untimed) with every launch on one stream: the timed
    # region overlaps weight gradients (side stream) with the input-gradient chain, so its
    # per-launch durations include the other stream's contention; this gives each kernel
    # family's rate in isolation (roofline.isolated)
    ksum_iso, iso_launches = {}, []
    if timer:
        from pggan_amd import engine as _E
        saved = (timer.rec, timer.shapes)
        timer.rec, timer.shapes = {k: [] for k in timer.rec}, []
        _E.FORCE_SERIAL = True
        timer.on = True
        step()
        model.flush()
        torch.cuda.synchronize()
        timer.on = False
        _E.FORCE_SERIAL = False
        ksum_iso = timer.summary()
        iso_launches = timer._launches()
        if os.environ.get("PG_BENCH_SHAPES"):
            with open(os.environ["PG_BENCH_SHAPES"] + ".iso.json", "w") as f:
                json.dump(timer.per_shape(1), f, indent=1)
        timer.rec, timer.shapes = saved
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ld = model.loss_collector.loss_dict
    assert all(v == v and abs(v) != float("inf") for v in ld.values()), f"non-finite loss {ld}"
    ksum = timer.summary() if timer else {}
    if timer and os.environ.get("PG_BENCH_SHAPES"):
        with open(os.environ["PG_BENCH_SHAPES"], "w") as f:
            json.dump(timer.per_shape(1), f, indent=1)
    if timer and os.environ.get("PG_BENCH_LAUNCHES"):
        # the instrumented step's conv / wgrad calls in launch order, with the roofline group
        # of each: tools/prof_summary.py aligns them with a --pmc pass's dispatches to give
        # each group its measured HBM bytes per call (roofline.traffic)
        # (".iso": the one-stream step's calls in ITS order -- the last dispatches of a --pmc
        # pass; the final pass's tail weight gradients sit elsewhere in the two-stream order)
        for path, ls in ((os.environ["PG_BENCH_LAUNCHES"], timer._launches()),
                         (os.environ["PG_BENCH_LAUNCHES"] + ".iso", iso_launches)):
            with open(path, "w") as f:
                json.dump([dict(group=f"{fam}/{bound}", H=H, flops=fl, bytes=by)
                           for fam, H, fl, by, ms, bound in ls], f)

    if rank == 0:
        roof = None
        if ksum:
            # dominant = the (kernel family, bound) group with the most time: every launch
            # is classified against its own roofline, so a group's achieved rate and peak
            # are in the same unit
            dom = max(ksum, key=lambda k: ksum[k]["total_ms"])
            kd = ksum[dom]
            fam = dom.split("/")[0]
            if kd["bound"] == "hbm":
                ach, peak, unit = kd["gbps"], PEAK_HBM_GBS, "GB/s"
            else:
                ach, peak, unit = kd["tflops"], PEAK_TFLOPS[timer.peak_key(fam)], "TFLOP/s"
            traffic, tsrc = pmc_traffic(args, dom, kd["launches"])
            roof = dict(bound=kd["bound"], kernel=dom, achieved=round(ach, 2),
                        peak=peak, unit=unit, frac=round(ach / peak, 4), traffic=traffic,
                        traffic_source=tsrc,
                        algorithmic_bytes_per_launch=round(kd["bytes"] / kd["launches"]),
                        flops_per_launch=round(kd["flops"] / kd["launches"]),
                        launches_per_step=kd["launches"],
                        avg_launch_us=round(kd["avg_us"], 2),
                        roofline_time_frac=round(kd["roofline_time_frac"], 4),
                        # whole-step MFMA fraction at the minimal algorithmic
                        # GFLOP per image (1280.78 at C5), all kernels, wall clock
                        step_mfma_frac=round(STEP_GFLOP_PER_IMG.get(args.stage, 0.0) * 1e9 *
                                             B * args.steps / dt /
                                             (PEAK_TFLOPS[args.dtype] * 1e12), 4),
                        groups={k: dict(total_ms_per_step=round(v["total_ms"], 3),
                                        tflops=round(v["tflops"], 2), gbps=round(v["gbps"], 1),
                                        roofline_time_frac=round(v["roofline_time_frac"], 4),
                                        launches_per_step=v["launches"])
                                for k, v in sorted(ksum.items())},
                        per_resolution=timer.per_resolution())
            if ksum_iso:
                # the same groups from the isolated step (no overlap): achieved / frac per
                # group against its own peak
                def _iso(k, v):
                    hbm = v["bound"] == "hbm"
                    a = v["gbps"] if hbm else v["tflops"]
                    pk = PEAK_HBM_GBS if hbm else PEAK_TFLOPS[timer.peak_key(k.split("/")[0])]
                    return dict(achieved=round(a, 2), unit="GB/s" if hbm else "TFLOP/s",
                                frac=round(a / pk, 4), avg_launch_us=round(v["avg_us"], 2),
                                total_ms_per_step=round(v["total_ms"], 3))
                roof["isolated"] = dict(
                    note="one extra untimed step with every launch on one stream (per-launch "
                         "durations without the side stream's overlap)",
                    groups={k: _iso(k, v) for k, v in sorted(ksum_iso.items())})
        cpu = None
        log(f"timed: {1e3 * dt / args.steps:.3f} ms/step")
        if args.cpu_baseline == "auto" and world == 1:
            log(f"CPU baseline: one oracle step on {args.cpu_threads or host_threads()} threads")
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
            "config": {"workload": f"{CONFIG_NAME.get((s, B), 'custom')} G+D+"
                                   f"{'R1' if args.gp_mode == 'r1' else 'WGAN-GP'} train_step "
                                   f"via ProgressiveGAN.train_step, stage {s} ({R}x{R}), "
                                   f"batch {B}/GPU, alpha {args.alpha}, depths {depths}" +
                                   (" (alpha = 1: the fade-in's zero-weight low-resolution "
                                    "branches elided, results bit-identical on the CPU double, "
                                    "PG_ENGINE=elide_zero_blend=0 computes them)"
                                    if args.alpha == 1.0 and
                                    _engine_opts()["elide_zero_blend"] else ""),
                       "global_batch": B * world, "resolution": R,
                       "parallelism": f"dp{world}"},
            "host_enqueue_ms_per_step": round(host_ms, 3),
            # timed steps re-issued by the library's C++ replay (or a hipGraph with --graph);
            # the last timed step runs eagerly with the per-launch timers
            "replayed_steps": graph_steps,
            "launch_path": ("hipgraph" if args.graph else "eager" if args.eager else
                            "cpp-replay"),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        ex = getattr(model, "_exchange", None)
        if ex is not None:
            line["dp_exchange"] = dict(
                note="world-1 RCCL group: grad_ready buckets + side-stream joins on"
                if world == 1 else "RCCL", bucket_mb=ex.bucket_bytes / (1 << 20),
                collectives_per_step=round(ex.calls / (args.warmup + args.steps + 3), 1),
                host_ms_per_collective=round(1e3 * ex.host_s / max(ex.calls, 1), 3))
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
