"""Data-parallel gradient exchange: one process per GPU, RCCL over xGMI.

The reference wraps its nets in DistributedDataParallel and immediately discards the
wrapper (lib/model.py:74-79), so its ranks never exchange gradients.  Here the mean
over ranks of each net's flat live gradient is all-reduced before that net's Adam
step, in buckets launched as the final backward pass finishes each layer:

* the engine calls `ready(net, names)` right after the last kernel that writes those
  parameters' gradients (StepEngine.grad_ready), in backward order -- the 512-channel
  layers near the logit finish first, so their buckets (the bulk of the 92 MB per net
  at 1024^2) travel while the high-resolution layers are still being differentiated;
* `finish(net)` launches what is left and returns a Pending whose wait() completes the
  exchange and applies the 1/world mean; the engine waits right before that net's Adam
  step, which it schedules after independent work (the G forward for D, the next
  step's real-image D part for G; engine.train_step).

A collective enqueued on the RCCL stream waits for the compute stream at the time of
the call, so every bucket sees its finished gradient.

Every host action of the exchange (a bucket's all-reduce, sealing a net's exchange into its
Pending, the wait before Adam) goes through `_act`: while `ProgressiveGAN` records a step for
the C++ replay (`record_hook` set), the action is also appended to the recording between the
library's launch segments, so a replayed step issues the same collectives and waits at the
same points of the launch sequence, on the same streams.  `reduce_dtype=torch.bfloat16`
halves the bytes on the links (gradients rounded to bf16 before the sum: an opt-in
trade, the default fp32 keeps the DP contract exact to fp32 rounding).
"""
from __future__ import annotations

import functools
import time

import torch
import torch.distributed as dist


def _stream_of(t):
    """The current stream of a CUDA tensor's device (None for CPU tensors)."""
    return torch.cuda.current_stream(t.device) if t.is_cuda else None


class Handle:
    """What `finish` returns to the engine (its grad_hook result): wait() completes the
    net's exchange.  The exchange itself lives in GradExchange._pending, so a replayed step's
    sealed exchange is the one the next wait finds."""

    def __init__(self, ex, net):
        self.ex, self.net = ex, net

    def wait(self):
        self.ex._act(functools.partial(self.ex._wait_now, self.net,
                                       _stream_of(self.ex._fp[self.net].grad)))


class Pending:
    """The in-flight exchange of one net's gradient; wait() finishes it."""

    def __init__(self, works, grad, world, casts):
        self.works, self.grad, self.world, self.casts = works, grad, world, casts

    def wait(self):
        for w in self.works:
            w.wait()
        for lo, hi, buf in self.casts:
            # buf was allocated on the stream that launched the collective (the weight-gradient
            # stream): tell the caching allocator this stream reads it too, or the block could be
            # handed out again there before this copy has run
            if buf.is_cuda:
                buf.record_stream(torch.cuda.current_stream(buf.device))
            self.grad[lo:hi].copy_(buf)
        if self.world > 1:
            self.grad.mul_(1.0 / self.world)


class GradExchange:
    """Bucketed asynchronous all-reduce (mean) of flat gradients, one instance per
    process; `bucket_bytes` is the smallest bucket launched on its own (smaller ready
    ranges are merged and sent with the next one or at finish)."""

    def __init__(self, world=None, bucket_bytes=4 << 20, reduce_dtype=torch.float32, group=None):
        self.world = world if world is not None else dist.get_world_size(group)
        self.bucket_bytes = bucket_bytes
        self.reduce_dtype = reduce_dtype
        self.group = group
        self._fp = {}
        self._state = {}
        self._pending = {}     # net -> the sealed, in-flight exchange (Pending)
        # set while a step is recorded for replay: called with each host action
        self.record_hook = None
        self.calls = 0          # collectives launched, and the host seconds spent in them
        self.host_s = 0.0

    def bind(self, net, fp):
        """fp: the net's engine.FlatParams (live parameters first)."""
        self._fp[net] = fp
        self._state[net] = dict(works=[], casts=[], pend=[], pend_elems=0, sent=[])

    def _act(self, fn):
        """Run one host action now (and append it to a step being recorded)."""
        if self.record_hook is not None:
            self.record_hook(fn)
        fn()

    def _launch(self, net, lo, hi):
        self._state[net]["sent"].append((lo, hi))
        self._act(functools.partial(self._launch_now, net, lo, hi, _stream_of(self._fp[net].grad)))

    def _launch_now(self, net, lo, hi, stream):
        t0 = time.perf_counter()
        st, g = self._state[net], self._fp[net].grad
        if stream is not None:
            with torch.cuda.stream(stream):
                self._all_reduce(st, g, lo, hi)
        else:
            self._all_reduce(st, g, lo, hi)
        self.calls += 1
        self.host_s += time.perf_counter() - t0

    def _all_reduce(self, st, g, lo, hi):
        if self.reduce_dtype == torch.float32:
            st["works"].append(dist.all_reduce(g[lo:hi], group=self.group, async_op=True))
        else:
            buf = g[lo:hi].to(self.reduce_dtype)
            st["works"].append(dist.all_reduce(buf, group=self.group, async_op=True))
            st["casts"].append((lo, hi, buf))

    def _seal(self, net):
        """The collectives launched for `net` since the last seal become its Pending."""
        st = self._state[net]
        self._pending[net] = Pending(st["works"], self._fp[net].grad, self.world, st["casts"])
        st["works"], st["casts"] = [], []

    def _wait_now(self, net, stream):
        p = self._pending.pop(net)
        if stream is not None:
            with torch.cuda.stream(stream):
                p.wait()
        else:
            p.wait()

    def _launch_merged(self, net, ranges):
        """One collective per maximal contiguous span of `ranges`."""
        run = None
        for lo, hi in sorted(ranges):
            if run is not None and lo <= run[1]:
                run = (run[0], max(run[1], hi))
                continue
            if run is not None:
                self._launch(net, *run)
            run = (lo, hi)
        if run is not None:
            self._launch(net, *run)

    def ready(self, net, names):
        """Gradients of `names` (a layer's weight and bias) are final."""
        if net not in self._fp:
            return
        fp, st = self._fp[net], self._state[net]
        for n in names:
            if n in fp.dead:
                continue
            lo, hi = fp.spans[n]
            st["pend"].append((lo, hi))
            st["pend_elems"] += hi - lo
        if st["pend_elems"] * 4 >= self.bucket_bytes:
            self._launch_merged(net, st["pend"])
            st["pend"], st["pend_elems"] = [], 0

    def finish(self, net):
        """Launch the rest of `net`'s live gradient (pending buckets, and any live range the
        engine never reported) and return its Pending."""
        fp, st = self._fp[net], self._state[net]
        done = sorted(st["sent"] + st["pend"])
        rest, pos = list(st["pend"]), 0
        for lo, hi in done:
            if lo > pos:
                rest.append((pos, lo))
            pos = max(pos, hi)
        if pos < fp.n_live:
            rest.append((pos, fp.n_live))
        self._launch_merged(net, rest)
        self._act(functools.partial(self._seal, net))
        st["pend"], st["pend_elems"], st["sent"] = [], 0, []
        return Handle(self, net)

    def hook(self, net, g):
        """engine.train_step grad_hook."""
        return self.finish(net)
