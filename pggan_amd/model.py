"""ProgressiveGAN with the reference plugin interface (lib/model.py:8-138,
pggan/model.py:11-265) running the MI355X step engine.

Same method names, return values and schedule semantics as the reference:
`initialize_models`, `set_multi_GPU`, `set_optimizers`, `set_dataset`,
`set_data_iterator`, `set_loss_collector`, `load_next_batch`, `train_step` ->
`[img_real, img_fake]`, `check_jump` / `change_scale` / `change_alpha` /
`reset_alpha` / `reset_solver`, `save_checkpoint` / `load_checkpoint`
(reference checkpoint file layout and dict keys), `save_image`, `validation`,
`loss_collector`.  `G` and `D` are pggan_amd.nets modules whose parameters are
views of the engine's flat fp32 buffers.

Differences (deliberate):
  * set_multi_GPU really all-reduces G and D gradients (mean over ranks) before
    each Adam step; the reference discards its DDP wrapper (lib/model.py:78-79).
  * latents are drawn on the GPU per rank (pg_randn) instead of the CPU RNG.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.distributed as dist

from . import dp as DP
from . import engine as E
from .config import cfg_get
from .data import BatchLoader, ImageFolderDataset
from .loss import WGANGPLoss
from .nets import Discriminator, Generator


class FlatAdam:
    """torch.optim.Adam semantics (lib/model.py:95-97) over a net's flat buffers; the
    state_dict() has torch.optim.Adam's layout so reference checkpoints interoperate."""

    def __init__(self, fp: E.FlatParams, names, lr, betas, eps=1e-8):
        self.fp, self.names = fp, list(names)
        self.lr, self.betas, self.eps = lr, tuple(betas), eps
        self.param_groups = [dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=0,
                                  amsgrad=False, maximize=False, foreach=None,
                                  capturable=False, differentiable=False, fused=None,
                                  decoupled_weight_decay=False)]

    def zero_grad(self, set_to_none=True):
        self.fp.grad.zero_()

    def state_dict(self):
        st = {}
        if self.fp.step > 0:
            for i, n in enumerate(self.names):
                if n in self.fp.dead:
                    continue
                st[i] = {"step": torch.tensor(float(self.fp.step)),
                         "exp_avg": self.fp._view(self.fp.m, n).clone(),
                         "exp_avg_sq": self.fp._view(self.fp.v, n).clone()}
        pg = dict(self.param_groups[0])
        pg["params"] = list(range(len(self.names)))
        return {"state": st, "param_groups": [pg]}

    def load_state_dict(self, sd):
        steps = set()
        for i, s in sd.get("state", {}).items():
            n = self.names[int(i)]
            self.fp._view(self.fp.m, n).copy_(s["exp_avg"])
            self.fp._view(self.fp.v, n).copy_(s["exp_avg_sq"])
            steps.add(int(float(s["step"])))
        if steps:
            self.fp.step = max(steps)
        if sd.get("param_groups"):
            g = sd["param_groups"][0]
            self.lr, self.betas, self.eps = g["lr"], tuple(g["betas"]), g["eps"]


class _Segments:
    """A recorded step: the library's launch recordings (`_lib.Recording`) and, under DP, the
    exchange's host actions between them, re-issued in order."""

    def __init__(self, segs):
        self.segs = [x for x in segs if callable(x) or len(x) > 0]

    def replay(self):
        for x in self.segs:
            if hasattr(x, "replay"):
                x.replay()
            else:
                x()

    def __len__(self):
        return sum(len(x) for x in self.segs if hasattr(x, "replay"))


class ProgressiveGAN:
    """pggan/model.py:11-265.

    `ops_factory(dtype)` builds the kernel op set; the default is the HIP library
    (`pggan_amd._lib.HipOps`).  Tests substitute a CPU double to exercise the host
    logic (schedule, checkpoints, DP bookkeeping) without a GPU."""

    ops_factory = None

    def __init__(self, args, gpu):
        self.args = args
        self.gpu = gpu
        self.device = torch.device("cuda", gpu) if isinstance(gpu, int) else torch.device(gpu)
        self.G = self.D = None
        self.scale_index = 0
        self.world, self.rank = 1, 0
        self.dtype = torch.bfloat16 if cfg_get(args, "compute_dtype", "f32") == "bf16" \
            else torch.float32
        self.hyper = E.Hyper(lr_G=args.lr_G, lr_D=args.lr_D, beta1=float(args.beta1),
                             beta2=float(args.beta2), W_adv=float(cfg_get(args, "W_adv", 1) or 0),
                             slope_cfg=float(cfg_get(args, "LReLU_slope", 0.2)),
                             gp_mode=cfg_get(args, "gp_mode", "r1"),
                             W_gp=float(cfg_get(args, "W_gp", 10)),
                             W_drift=float(cfg_get(args, "W_drift_D", 0) or 0))
        self._engines = {}
        self._rng_step = 0
        self.global_step = 0
        self.alpha_index = 0
        self.alpha_jump_value = 0
        self.next_alpha_jump_step = 0
        self.next_scale_jump_step = 0
        self.train_dataset = None
        self.synthetic = None
        self._exchange = None

    # ------------------------------------------------------------------ models
    def initialize_models(self):
        a = self.args
        self.G = Generator(a.latent_dim, a.depths[0], a.init_bias_to_zero, a.LReLU_slope,
                           a.apply_pixel_norm, a.generator_last_activation, a.output_dim,
                           a.equalized_lr).to(self.device)
        self.D = Discriminator(a.depths[0], a.init_bias_to_zero, a.LReLU_slope,
                               a.decision_layer_size, a.apply_minibatch_norm, a.input_dim,
                               a.equalized_lr).to(self.device)
        self.G.compute_dtype = self.dtype
        self.D.compute_dtype = self.dtype
        self.G.train()
        self.D.train()

    def set_multi_GPU(self):
        """lib/model.py:74-79 + lib/utils.py:78-83, but with a working gradient all-reduce:
        one process per GPU, RCCL, initial parameter broadcast from rank 0."""
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "3456")
            dist.init_process_group("nccl", rank=int(os.environ.get("RANK", self.gpu)),
                                    world_size=int(os.environ.get("WORLD_SIZE",
                                                                  self.args.gpu_num)))
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self._broadcast_params()
        # dp_exchange_world1: the exchange also at one rank (an RCCL all-reduce over one
        # rank), to measure what the DP bookkeeping costs the step (bench.py --dp-exchange)
        if self.world > 1 or cfg_get(self.args, "dp_exchange_world1", False):
            from .dp import GradExchange
            rd = torch.bfloat16 if cfg_get(self.args, "dp_reduce_dtype", "f32") == "bf16" \
                else torch.float32
            # bucket size: config dp_bucket_mb (64 MiB).  Each collective costs ~50-100 us of
            # host time (torch + RCCL enqueue) and ~0.15 % of the step at one rank (32 -> 64 MiB:
            # 10 -> 5 collectives per step, -3.2 -> -2.5 %, profiles/r5_dp_ab.txt); the tail the
            # last backward leaves for finish() is the last 512-channel layers either way
            mb = float(cfg_get(self.args, "dp_bucket_mb", 64))
            self._exchange = GradExchange(self.world, bucket_bytes=int(mb * (1 << 20)),
                                          reduce_dtype=rd)

    def _broadcast_params(self):
        if self.world > 1:
            self.flush()
            for net in (self.G, self.D):
                for p in net.parameters():
                    dist.broadcast(p.data, 0)
            self._params_changed()

    def _params_changed(self):
        for eng in self._engines.values():
            eng.params_changed()

    def _flat(self, net, which):
        shapes = [(n, tuple(p.shape)) for n, p in net.named_parameters()]
        init = {n: p.detach() for n, p in net.named_parameters()}
        fp = E.FlatParams(shapes, E.dead_params(which, self.scale_index), self.device, init)
        for n, p in net.named_parameters():
            p.data = fp.views[n]
            p.grad = fp.gviews[n]
        return fp

    def set_optimizers(self):
        """lib/model.py:95-97: fresh Adam(lr, betas) for G and D (moments reset)."""
        a = self.args
        self.fpG, self.fpD = self._flat(self.G, "G"), self._flat(self.D, "D")
        self.opt_G = FlatAdam(self.fpG, [n for n, _ in self.G.named_parameters()], a.lr_G,
                              (float(a.beta1), float(a.beta2)))
        self.opt_D = FlatAdam(self.fpD, [n for n, _ in self.D.named_parameters()], a.lr_D,
                              (float(a.beta1), float(a.beta2)))

    # ------------------------------------------------------------------ data
    def set_dataset(self):
        """pggan/model.py:118-126: the images under `dataset_root_list`, 70% train split.

        A configured root that does not exist, or roots holding no image, raise (the
        reference's DataLoader fails on an empty dataset too).  The resident synthetic
        batch (U[-1,1) reals in HBM, the benchmark setting) is used only when the config
        asks for it with `synthetic_data: True`."""
        R = 4 * 2 ** self.scale_index
        if cfg_get(self.args, "synthetic_data", False):
            self.train_dataset = None
            g = torch.Generator(device=self.device).manual_seed(1000 * self.rank)
            self.synthetic = torch.rand(self.args.batch_per_gpu, 3, R, R, device=self.device,
                                        generator=g) * 2 - 1
            return
        roots = list(cfg_get(self.args, "dataset_root_list", None) or [])
        missing = [r for r in roots if not os.path.isdir(r)]
        if missing:
            raise FileNotFoundError(f"dataset_root_list: no such directory: {missing}")
        ds = ImageFolderDataset(roots, self.scale_index)
        if len(ds) == 0:
            raise RuntimeError(f"no images found under dataset_root_list {roots} (set "
                               f"synthetic_data: True to train on a synthetic batch)")
        n_train = round(len(ds) * 0.7)
        perm = np.random.default_rng(0).permutation(len(ds))
        ds.paths = [ds.paths[i] for i in perm[:n_train]]
        self.train_dataset = ds

    def set_data_iterator(self):
        """lib/model.py:44-52: without use_mGPU the dataset is read in order (DataLoader without
        a sampler, no shuffle); with use_mGPU (any world size, one included) each rank reads its
        DistributedSampler shard (seed 0, set_epoch never called, so every epoch repeats the
        same order: SURVEY Appendix A.4)."""
        self._order, self._pos = None, 0
        if self.train_dataset is not None:
            self._order = sampler_order(len(self.train_dataset), self.rank, self.world,
                                        distributed=bool(cfg_get(self.args, "use_mGPU", False)))

    def load_next_batch(self):
        """pggan/model.py:104-115."""
        if self.train_dataset is None:
            return self.synthetic
        B = self.args.batch_per_gpu
        if self._pos + B > len(self._order):
            self._pos = 0
        idx = self._order[self._pos:self._pos + B]
        self._pos += B
        nxt = self._pos if self._pos + B <= len(self._order) else 0
        if getattr(self, "_loader", None) is None or self._loader.ds is not self.train_dataset:
            # decode + resize on host threads, flip + ColorJitter + normalize on the GPU
            # (pggan_amd.data; lib/dataset.py:106-117).  A new stage's loader replaces the
            # previous one (its threads and pending decodes are cancelled) and keeps drawing
            # augmentation parameters from the same generator, so stages do not replay one
            # parameter sequence.
            from . import _lib
            if getattr(self, "_loader", None) is not None:
                self._loader.close()
            if getattr(self, "_aug_gen", None) is None:
                self._aug_gen = torch.Generator().manual_seed(1000 + self.rank)
            # decoded images stay in HBM (pggan_amd.data.HbmImageCache): config
            # hbm_image_cache_gb, default 40 % of the free device memory
            gb = cfg_get(self.args, "hbm_image_cache_gb", None)
            self._loader = BatchLoader(self.train_dataset, self.device, _lib.HipOps(torch.float32),
                                       gen=self._aug_gen,
                                       cache_bytes=None if gb is None else int(float(gb) * (1 << 30)))
        return self._loader.next(idx, prefetch=self._order[nxt:nxt + B])

    def set_loss_collector(self):
        self._loss_collector = WGANGPLoss(self.args)

    @property
    def loss_collector(self):
        return self._loss_collector

    def set_validation(self):
        pass

    def validation(self, *args):
        pass

    # ------------------------------------------------------------------ step
    def _engine(self, B):
        key = (self.scale_index, B)
        if key not in self._engines:
            from . import _lib
            self.flush()
            self._engines = {}   # one stage at a time: free the previous stage's buffers
            factory = type(self).ops_factory or _lib.HipOps
            eng = E.StepEngine(factory(self.dtype), self.args.depths, self.scale_index, B,
                               self.device, self.args.latent_dim)
            self._engines[key] = eng
        eng = self._engines[key]
        eng.bind(self.fpG, self.fpD, self.hyper)      # no-op unless the buffers changed
        if self._exchange is not None:
            eng.grad_ready = self._exchange.ready
            if self._exchange._fp.get("G") is not self.fpG or \
                    self._exchange._fp.get("D") is not self.fpD:
                self._exchange.bind("G", self.fpG)
                self._exchange.bind("D", self.fpD)
        return eng

    def _grad_hook(self, net, g):
        """Before each Adam step: the asynchronous bucketed RCCL all-reduce (mean) of the
        net's live gradient (pggan_amd.dp); the engine waits on it right before Adam and
        overlaps it with the work that does not depend on it."""
        if self._exchange is None:
            return None
        return self._exchange.hook(net, g)

    def flush(self):
        """Complete a deferred G update (overlapped DP mode): call before reading G's
        parameters outside train_step (save_checkpoint does)."""
        for eng in self._engines.values():
            eng.flush()

    # one training step captured once per (stage, schedule scalars) and replayed as a
    # hipGraph (world == 1, use_graph = True): the host enqueue of ~600 launches (6.3 ms) becomes
    # one graph launch (1.5-1.7 ms).  Off by default: on ROCm 7.2 the replay of this
    # two-stream step runs 6-7 % slower on the GPU than the eager streams (13.5 vs 12.55
    # ms/step, interleaved A/B in one call, profiles/r3_graph_ab.txt), and the step is
    # GPU-bound (12.5 ms of kernels vs 6.3 ms of host enqueue).
    use_graph = False
    # the same step recorded once by the library's launch recorder and re-issued from C++
    # (pg_record_* / pg_replay, world == 1, R1 mode): the host enqueue without the Python layer
    # (1.5 vs 4.6 ms per C5 step), on the engine's own two streams (a hipGraph re-levels them
    # onto other hardware queues).  Bitwise the eager step (tests/test_gpu_graph.py).  The
    # first step of a (stage, batch, alpha, hyper-parameter) key runs eagerly, the second is
    # recorded while it runs, later ones replay; anything the key does not see -- a parameter
    # edited through .data, a buffer reallocated -- needs _params_changed() or use_replay off.
    use_replay = True
    graph_replays = 0

    def _graph_key(self, eng, B):
        """The key of a replayable step, or None when this step must run eagerly: the HIP op
        set (device-side step counters), no trace hook, packed weights.  The hipGraph form:
        one process, no deferred generator update.  The C++ replay also under DP: the
        exchange's collectives and waits are host actions recorded between launch segments
        (dp.GradExchange._act), and a deferred generator update is the exchange's own state."""
        dp = self._exchange is not None
        if not ((self.use_graph or self.use_replay) and
                self.device.type == "cuda" and self.hyper.gp_mode == "r1" and
                hasattr(eng.ops, "randn_dev") and hasattr(eng.ops, "adam_dev") and
                eng.trace is None and not E.FORCE_SERIAL and all(eng._packed.values())):
            return None
        if dp:
            if not self.use_replay or eng.grad_ready != self._exchange.ready or \
                    not (eng._pending_G is None or isinstance(eng._pending_G, DP.Handle)):
                return None
        elif eng.grad_ready is not None or eng._pending_G is not None:
            return None
        h = self.hyper
        return ("replay" if self.use_replay else "graph",
                id(eng), id(self.fpG), id(self.fpD), B, float(self.G.alpha), float(self.D.alpha),
                h.lr_G, h.lr_D, h.beta1, h.beta2, h.eps, h.W_adv, h.slope_cfg, h.gp_mode, h.W_gp,
                h.W_drift, id(self._exchange), isinstance(eng._pending_G, DP.Handle))

    def _step_body(self, eng, real, B):
        """The work of one step after the batch is resident: latents, then the engine step."""
        z = self._z
        if hasattr(eng.ops, "randn_dev"):
            off = getattr(self, "_rng_off", None)
            if off is None or off.device != self.device:
                off = self._rng_off = torch.zeros(1, dtype=torch.int64, device=self.device)
                self._rng_off_host = None
            if self._rng_off_host != self._rng_step * z.numel():   # keep host and device in step
                off.fill_(self._rng_step * z.numel())
            eng.ops.randn_dev(z, 1000 * self.rank + 17, off)
            self._rng_off_host = (self._rng_step + 1) * z.numel()
        else:
            eng.ops.randn(z, 1000 * self.rank + 17, self._rng_step * z.numel())
        self._rng_step += 1
        gp_eps = None
        if self.hyper.gp_mode != "r1":
            gp_eps = torch.rand(B, 1, device=self.device)
        return eng.train_step(real, z[0], z[1], float(self.G.alpha), float(self.D.alpha),
                              grad_hook=self._grad_hook, gp_eps=gp_eps)

    def _replay(self, eng, key, img_real, B):
        """Run the step from the captured graph (capturing it on the second step with the
        same key); returns the engine's outputs or None to run eagerly."""
        # one state per key (a DP run alternates two: with and without a deferred generator
        # update, e.g. around flush()); the first step of a key runs eagerly (warms every lazy
        # buffer), the second records, later ones replay
        states = self.__dict__.setdefault("_gstates", {})
        gs = states.get(key)
        if gs is None:
            if len(states) >= 4:
                states.clear()
            states[key] = gs = {"key": key}
            self._gstate = gs
            return None
        self._gstate = gs
        # the graph's kernels read the device-side Adam step counts and RNG offset and advance
        # them, and a capture would record the host's re-sync of them (a fill) into the graph:
        # capture or replay only while the host's counts are the ones the device holds.  An
        # optimizer load_state_dict or a schedule reset changes a host count alone; that step
        # runs eagerly (which rewrites the device copies) and the next one captures again.
        if (any(fp._step_dev_host != fp.step for fp in (self.fpG, self.fpD)) or
                getattr(self, "_rng_off_host", None) != self._rng_step * self._z.numel()):
            states.clear()
            states[key] = self._gstate = {"key": key}
            return None
        if key[0] == "replay":
            if "rec" not in gs:
                # record the second step while it runs; the recording holds the buffer
                # pointers of this batch, so later batches are copied into the same buffer.
                # Under DP the exchange's host actions split it into segments: C++ launch
                # recordings and the Python collectives / waits between them.
                gs["real"] = img_real if img_real is self.synthetic else img_real.clone()
                segs = []

                def hook(fn):
                    segs.append(eng.ops.record_end())
                    segs.append(fn)
                    eng.ops.record_begin()

                if self._exchange is not None:
                    self._exchange.record_hook = hook
                eng.ops.record_begin()
                steps0 = (self.fpG.step, self.fpD.step)
                ok = False
                try:
                    gs["out"] = self._step_body(eng, gs["real"], B)
                    ok = True
                finally:
                    segs.append(eng.ops.record_end())
                    if self._exchange is not None:
                        self._exchange.record_hook = None
                    if ok:
                        gs["rec"] = _Segments(segs)
                        # the engine's host state after the step (a deferred generator update
                        # under DP, the merged-forward flags): a replay runs no Python, so it
                        # restores what the recorded step left behind.  The Adam steps the
                        # recording runs: one per net, except under DP where a step that starts
                        # with no deferred G update (after a flush) runs no Adam_G
                        gs["post"] = eng.host_state()
                        gs["adam"] = (self.fpG.step - steps0[0], self.fpD.step - steps0[1])
                    else:       # a truncated recording is never replayed: the key starts over
                        states.pop(key, None)
                        self.__dict__.pop("_gstate", None)
                return gs["out"]
            if img_real is not gs["real"]:
                gs["real"].copy_(img_real)
            self._rng_step += 1
            self._rng_off_host = self._rng_step * self._z.numel()
            for fp, n in zip((self.fpG, self.fpD), gs["adam"]):
                fp.step += n
                fp._step_dev_host = fp.step
            gs["rec"].replay()
            eng.set_host_state(gs["post"])
            self.graph_replays += 1
            return gs["out"]
        if "graph" not in gs:
            gs["real"] = img_real if img_real is self.synthetic else img_real.clone()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                gs["out"] = self._step_body(eng, gs["real"], B)
            gs["graph"] = g
            # capture ran the host bookkeeping of one step (step counts, RNG offset) without
            # the kernels; the replay below executes them
        else:
            if img_real is not gs["real"]:
                gs["real"].copy_(img_real)
            self._rng_step += 1
            self._rng_off_host = self._rng_step * self._z.numel()
            for fp in (self.fpG, self.fpD):
                fp.step += 1
                fp._step_dev_host = fp.step
        gs["graph"].replay()
        self.graph_replays += 1
        return gs["out"]

    def train_step(self):
        """pggan/model.py:206-255; returns [img_real, img_fake]."""
        img_real = self.load_next_batch()
        B = img_real.shape[0]
        eng = self._engine(B)
        # in-place edits of G / D parameters outside the engine (load_state_dict, p.copy_,
        # EMA copies) bump the parameters' version counters: repack the weights before the
        # step uses them.  Edits through `p.data` bypass the counters; call _params_changed()
        # after those.
        ver = (sum(p._version for p in self.G.parameters()),
               sum(p._version for p in self.D.parameters()))
        if ver != getattr(self, "_param_ver", ver):
            self._params_changed()
        self._param_ver = ver
        self.hyper.lr_G, self.hyper.lr_D = self.opt_G.lr, self.opt_D.lr
        z = getattr(self, "_z", None)
        if z is None or z.shape[1] != B:
            self._z = z = torch.empty(2, B, self.args.latent_dim, device=self.device)
        key = self._graph_key(eng, B)
        out = self._replay(eng, key, img_real, B) if key is not None else None
        if out is None:
            if key is None:        # an eager step may change what a captured graph assumed
                self.__dict__.pop("_gstates", None)
                self.__dict__.pop("_gstate", None)
            out = self._step_body(eng, img_real, B)
        img_real, _, img_fake = out
        self.loss_collector.attach(eng.loss, self.hyper.gp_mode)
        return [img_real, img_fake]

    # ------------------------------------------------------------------ schedule
    def reset_solver(self):
        """pggan/model.py:131-139."""
        self.flush()
        self.set_dataset()
        self.set_data_iterator()
        self.set_optimizers()

    def reset_alpha(self, global_step):
        """pggan/model.py:141-156."""
        self.G.alpha = 0
        self.D.alpha = 0
        self.alpha_index = 0
        self.next_alpha_jump_step = global_step + self.args.alpha_jump_start[self.scale_index]
        self.alpha_jump_value = 1 / self.args.alpha_jump_Ntimes[self.scale_index]
        if cfg_get(self.args, "isMaster", False):
            print("alpha and alpha_index are initialized to 0")
            print(f"next_alpha_jump_step is set to {self.next_alpha_jump_step}")
            print(f"alpha_jump_value is set to {self.alpha_jump_value}")

    def change_scale(self, global_step):
        """pggan/model.py:158-174: add a block to G and D, fresh solver, reset alpha."""
        self.flush()
        self.scale_index += 1
        self.next_scale_jump_step += self.args.max_step_at_scale[self.scale_index]
        self.G.add_block(self.args.depths[self.scale_index])
        self.D.add_block(self.args.depths[self.scale_index])
        self._broadcast_params()
        self.reset_solver()
        self.reset_alpha(global_step)
        if cfg_get(self.args, "isMaster", False):
            print(f"\nNOW global_step is {global_step}")
            print(f"scale_index is updated to {self.scale_index}")
            print(f"next_scale_jump_step is {self.next_scale_jump_step}")

    def change_alpha(self, global_step):
        """pggan/model.py:176-194 (alpha rounded to 4 d.p.)."""
        self.alpha_index += 1
        self.G.alpha += self.alpha_jump_value
        self.D.alpha += self.alpha_jump_value
        self.G.alpha = round(self.G.alpha, 4)
        self.D.alpha = round(self.D.alpha, 4)
        if self.alpha_index == self.args.alpha_jump_Ntimes[self.scale_index]:
            self.next_alpha_jump_step = 0
        else:
            self.next_alpha_jump_step = global_step + self.args.alpha_jump_interval[self.scale_index]
        if cfg_get(self.args, "isMaster", False):
            print(f"\nNOW global_step is {global_step}")
            print(f"alpha_index is updated to {self.alpha_index}")
            print(f"next_alpha_jump_step is {self.next_alpha_jump_step}")
            print(f"alpha is now {self.G.alpha}")

    def check_jump(self, global_step):
        """pggan/model.py:196-204."""
        if self.next_scale_jump_step == global_step:
            self.change_scale(global_step)
        if self.next_alpha_jump_step == global_step:
            self.change_alpha(global_step)

    # ------------------------------------------------------------------ persistence
    def _ckpt_dict(self, global_step):
        return {"args": dict(self.args.__dict__), "global_step": global_step,
                "alpha_G": self.G.alpha, "alpha_D": self.D.alpha,
                "alpha_index": self.alpha_index, "alpha_jump_value": self.alpha_jump_value,
                "next_alpha_jump_step": self.next_alpha_jump_step,
                "scale_index": self.scale_index,
                "next_scale_jump_step": self.next_scale_jump_step}

    def save_checkpoint(self, global_step):
        """pggan/model.py:50-67 + lib/checkpoint.py:22-34 (same paths and keys)."""
        from . import checkpoint
        self.flush()
        base = self._ckpt_dict(global_step)
        checkpoint.save_checkpoint(self.G, self.opt_G, "G", dict(base))
        checkpoint.save_checkpoint(self.D, self.opt_D, "D", dict(base))

    def load_checkpoint(self):
        """pggan/model.py:70-101: restore schedule scalars, re-add blocks, fresh solver, then
        load model (strict=False) and optimizer state."""
        from . import checkpoint
        Gd = checkpoint.load_checkpoint(self.args, "G", self.device)
        Dd = checkpoint.load_checkpoint(self.args, "D", self.device)
        if not Gd or not Dd:
            raise RuntimeError("checkpoint not found")
        for k, v in Gd["args"].items():
            setattr(self.args, k, v) if not hasattr(self.args, "__setitem__") else \
                self.args.__setitem__(k, v)
        self.global_step = Gd["global_step"]
        self.alpha_index = Gd["alpha_index"]
        self.alpha_jump_value = Gd["alpha_jump_value"]
        self.next_alpha_jump_step = Gd["next_alpha_jump_step"]
        self.next_scale_jump_step = Gd["next_scale_jump_step"]
        target = Gd["scale_index"]
        # the reference re-adds blocks with depths[index] for index in range(scale_index)
        # (pggan/model.py:89-93); it builds a model whose depth list is depths[0..s]
        while self.scale_index < target:
            self.scale_index += 1
            self.G.add_block(self.args.depths[self.scale_index])
            self.D.add_block(self.args.depths[self.scale_index])
        self.reset_solver()
        self.G.alpha = Gd["alpha_G"]
        self.D.alpha = Gd["alpha_D"]
        self.G.load_state_dict(Gd["model"], strict=False)
        self.D.load_state_dict(Dd["model"], strict=False)
        self.opt_G.load_state_dict(Gd["optimizer"])
        self.opt_D.load_state_dict(Dd["optimizer"])
        self._params_changed()

    def save_image(self, images, step):
        """lib/utils.py:86-91: make_grid_image(images) * 255 written to
        {save_root}/{run_id}/imgs/e{step}.jpg (cv2.imwrite saturates and rounds to uint8)."""
        from PIL import Image
        grid = make_grid_image(images).permute(1, 2, 0).numpy().astype(np.float64) * 255
        d = f"{self.args.save_root}/{self.args.run_id}/imgs"
        os.makedirs(d, exist_ok=True)
        Image.fromarray(np.clip(np.rint(grid), 0, 255).astype(np.uint8)).save(f"{d}/e{step}.jpg")


def sampler_order(n, rank, world, distributed=None):
    """The sample order rank `rank` of `world` reads (lib/model.py:50-51).  The reference picks
    the sampler from args.use_mGPU (`distributed`; None: world > 1).  Without it the DataLoader
    has no sampler, i.e. in order.  With it: torch.utils.data.DistributedSampler(dataset) with
    its defaults (shuffle, seed 0, drop_last False) at epoch 0 -- torch.randperm(n) from a
    generator seeded with 0, padded by wrapping to a multiple of world, then every world-th
    index from rank (world may be 1: the whole permutation)."""
    if distributed is None:
        distributed = world > 1
    if not distributed:
        return np.arange(n)
    g = torch.Generator().manual_seed(0)
    idx = torch.randperm(n, generator=g).tolist()
    total = math.ceil(n / world) * world
    pad = total - n
    if pad <= n:
        idx += idx[:pad]
    else:
        idx += (idx * math.ceil(pad / n))[:pad]
    return np.asarray(idx[rank:total:world], dtype=np.int64)


def make_grid_image(list_of_tensors):
    """lib/utils.py:94-103: one torchvision.utils.make_grid row per tensor (its first 8
    images, nrow = their count, padding 2, pad value 0), each row * 0.5 + 0.5, rows stacked
    along the height.  Returns a CPU fp32 [C, H, W] tensor (the padding ends up 0.5, values
    are not clamped, as in the reference)."""
    rows = []
    for t in list_of_tensors:
        t = t[:8].detach().float().cpu()
        rows.append(_make_grid(t, nrow=t.shape[0]) * 0.5 + 0.5)
    return torch.cat(rows, dim=1)


def _make_grid(t, nrow, padding=2, pad_value=0.0):
    """torchvision.utils.make_grid's layout for a [N, C, H, W] batch (normalize=False)."""
    if t.dim() == 4 and t.shape[1] == 1:
        t = torch.cat((t, t, t), 1)
    if t.shape[0] == 1:
        return t.squeeze(0)
    n = t.shape[0]
    xmaps = min(nrow, n)
    ymaps = int(math.ceil(float(n) / xmaps))
    h, w = t.shape[2] + padding, t.shape[3] + padding
    grid = t.new_full((t.shape[1], h * ymaps + padding, w * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= n:
                break
            grid[:, y * h + padding:(y + 1) * h, x * w + padding:(x + 1) * w] = t[k]
            k += 1
    return grid
