"""ctypes binding of libpggan_hip.so (the C ABI declared in include/pggan_hip.h).

`HipOps` is the tensor-level op set the step engine is written against: every
method takes torch tensors resident on the GPU, passes raw device pointers and
the current HIP stream to one C-ABI entry point, and raises RuntimeError on a
non-zero status.  There is no fallback: if the shared library is missing or a
tensor is not on the GPU the call fails loudly.
"""
from __future__ import annotations

import ctypes
import os

import torch

PG_F32, PG_BF16 = 0, 1

CONV_UPS_IN, CONV_BIAS, CONV_LRELU, CONV_MASK, CONV_POOL, CONV_ACCUM = 1, 2, 4, 8, 16, 32
CONV_PIXNORM = 64
CONV_PNBWD = 2048
CONV_RGBW = 4096
CONV_RGBD = 8192
CONV_RGBO = 16384
CONV_Y2_BITS, CONV_AUX_BITS, CONV_X_BITS, CONV_GZ_BITS = 128, 256, 512, 1024
PACK_FWD, PACK_DGRAD = 0, 1
LIN_BIAS, LIN_LRELU, LIN_MASK, LIN_IN_CHW, LIN_OUT_CHW, LIN_F32_IN, LIN_F32_OUT = (
    1, 2, 4, 8, 16, 32, 64)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpggan_hip.so")


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("B", "H", "W", "cin", "cout", "x_cs", "y_cs", "aux_cs", "y2_cs", "flags")] + \
               [("slope", ctypes.c_float), ("out_scale", ctypes.c_float), ("xb_cs", ctypes.c_int)]


class PackItem(ctypes.Structure):
    """pg_pack_item (include/pggan_hip.h)."""
    _fields_ = [("w", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("fwd", ctypes.c_void_p),
                ("dgrad", ctypes.c_void_p), ("bias_scaled", ctypes.c_void_p),
                ("scale", ctypes.c_float), ("cout", ctypes.c_int), ("cin", ctypes.c_int),
                ("pad_", ctypes.c_int)]


def _cinp(c):
    return (c + 7) // 8 * 8 if c <= 16 else (c + 31) // 32 * 32


class ImgMix:
    """An image operand given as a per-sample mix (pg_img_src): img[b] = a[b] * x0[b] +
    c[b] * x1[b] (x1 / c optional; a None means x0 itself).  The penalty passes feed the
    fromRGB layers the interpolated image and the weighted input gradient this way."""

    def __init__(self, x0, x1=None, a=None, c=None):
        self.x0, self.x1, self.a, self.c = x0, x1, a, c

    @property
    def shape(self):
        return self.x0.shape

    @property
    def device(self):
        return self.x0.device

    def materialize(self):
        """The mixed image as a tensor (the CPU test double; never the HIP path)."""
        if self.a is None:
            return self.x0
        v = self.a.view(-1, 1, 1, 1) * self.x0
        if self.x1 is not None:
            v = v + self.c.view(-1, 1, 1, 1) * self.x1
        return v


class ImgSrcDesc(ctypes.Structure):
    """pg_img_src (include/pggan_hip.h)."""
    _fields_ = [("x0", ctypes.c_void_p), ("x1", ctypes.c_void_p), ("a", ctypes.c_void_p),
                ("c", ctypes.c_void_p)]


class LinearDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("B", "K", "N", "in_cs", "out_cs", "flags")] + \
               [("scale", ctypes.c_float), ("slope", ctypes.c_float)]


_lib = None
_SIDE_STREAMS = {}   # device index -> the least-priority side stream (pg_stream_create)

_VP, _I, _F, _SZ, _U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_uint64
_SIGS = {
    "pg_version": ([], _I),
    "pg_scratch_bytes": ([], _SZ),
    "pg_conv3x3_packed_elems": ([_I, _I, _I], _SZ),
    "pg_conv3x3_pack": ([_I, _I, _I, _I, _VP, _F, _VP, _VP], _I),
    "pg_conv3x3_pack_batch": ([_I, _I, _VP, _I, _VP], _I),
    "pg_conv3x3_workspace_size": ([ctypes.POINTER(ConvDesc)], _SZ),
    "pg_conv3x3_fwd": ([_I, ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _VP, _VP, _SZ, _VP],
                       _I),
    "pg_conv3x3_supported": ([_I, ctypes.POINTER(ConvDesc), _SZ], _I),
    "pg_conv3x3_rgbw": ([_I, ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _F, _VP, _VP, _VP, _VP],
                        _I),
    "pg_conv3x3_rgbd": ([_I, ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _F, _VP, _VP, _VP, _F,
                         _VP, _VP], _I),
    "pg_conv3x3_rgbo": ([_I, ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _VP, _VP, _F, _VP,
                         _VP], _I),
    "pg_conv3x3_fwd_ex": ([_I, ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP,
                           _SZ, _VP], _I),
    "pg_conv3x3_wgrad_ex": ([_I, ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _F, _VP, _VP, _VP, _SZ,
                             _VP], _I),
    "pg_conv3x3_wgrad_workspace_size": ([_I, ctypes.POINTER(ConvDesc)], _SZ),
    "pg_conv3x3_wgrad": ([_I, ctypes.POINTER(ConvDesc), _VP, _VP, _F, _VP, _VP, _VP, _SZ, _VP],
                         _I),
    "pg_bias_grad": ([_I, _I, _I, _I, _VP, _F, _VP, _VP, _VP], _I),
    "pg_pixnorm_fwd": ([_I, _I, _I, _I, _VP, _VP, _VP], _I),
    "pg_pixnorm_lrelu_bwd": ([_I, _I, _I, _I, _VP, _VP, _F, _I, _VP, _VP], _I),
    "pg_pixnorm_lrelu_bwd_y": ([_I, _I, _I, _I, _VP, _VP, _VP, _F, _VP, _VP], _I),
    "pg_unpool_mask": ([_I, _I, _I, _I, _I, _I, _VP, _I, _VP, _F, _F, _I, _I, _VP, _VP], _I),
    "pg_unpool_mask_bits": ([_I, _I, _I, _I, _I, _I, _VP, _VP, _F, _F, _I, _I, _VP, _VP], _I),
    "pg_avgpool2": ([_I, _I, _I, _I, _I, _I, _VP, _I, _VP, _VP], _I),
    "pg_blend": ([_I, _SZ, _F, _VP, _F, _VP, _VP, _VP], _I),
    "pg_rgb_out": ([_I, _I, _I, _I, _I, _VP, _VP, _VP, _F, _I, _I, _VP, _VP, _VP, _F, _F, _VP,
                    _VP], _I),
    "pg_rgb_out_bwd": ([_I, _I, _I, _I, _I, _VP, _VP, _F, _I, _I, _VP, _VP, _F, _F, _VP, _VP,
                        _VP, _VP, _VP, _VP, _VP, _VP, _VP], _I),
    "pg_from_rgb": ([_I, _I, _I, _I, _VP, _I, _VP, _VP, _F, _F, _VP, _I, _VP, _VP], _I),
    "pg_from_rgb_bwd": ([_I, _I, _I, _I, _VP, _I, _VP, _F, _I, _VP, _VP, _VP, _VP, _VP, _VP], _I),
    "pg_img_fade": ([_I, _I, _I, _VP, _F, _VP, _VP], _I),
    "pg_from_rgb_src": ([_I, _I, _I, _I, ctypes.POINTER(ImgSrcDesc), _I, _VP, _VP, _F, _F, _VP, _I,
                         _VP, _VP], _I),
    "pg_rgb_out_bwd_pn": ([_I, _I, _I, _I, _I, _VP, _VP, _VP, _F, _VP, _F, _I, _VP, _VP], _I),
    "pg_rgb_out_bwd_pn_wg": ([_I, _I, _I, _I, _I, _VP, _VP, _VP, _F, _VP, _F, _I, _VP, _VP, _VP,
                              _VP, _VP], _I),
    "pg_from_rgb_bits": ([_I, _I, _I, _I, ctypes.POINTER(ImgSrcDesc), _I, _VP, _VP, _F, _F, _VP,
                          _I, _VP, _VP, _VP], _I),
    "pg_from_rgb_bwd_src": ([_I, _I, _I, _I, ctypes.POINTER(ImgSrcDesc), _I, _VP, _F, _I, _VP, _VP,
                             _I, _VP, _VP, _VP, _VP, _VP], _I),
    "pg_penalty_scale": ([_I, _I, _VP, _F, _VP, _VP, _VP], _I),
    "pg_linear_fwd": ([_I, ctypes.POINTER(LinearDesc), _VP, _VP, _VP, _VP, _VP, _VP], _I),
    "pg_linear_dgrad": ([_I, ctypes.POINTER(LinearDesc), _VP, _VP, _VP, _VP, _VP], _I),
    "pg_linear_wgrad": ([_I, ctypes.POINTER(LinearDesc), _VP, _VP, _VP, _VP, _VP], _I),
    "pg_linear_workspace_size": ([_I, ctypes.POINTER(LinearDesc), _I], _SZ),
    "pg_linear_fwd_ws": ([_I, ctypes.POINTER(LinearDesc), _VP, _VP, _VP, _VP, _VP, _VP, _SZ, _VP],
                         _I),
    "pg_linear_dgrad_ws": ([_I, ctypes.POINTER(LinearDesc), _VP, _VP, _VP, _VP, _VP, _SZ, _VP],
                           _I),
    "pg_mbstd_fwd": ([_I, _I, _I, _I, _I, _VP, _I, _VP, _VP], _I),
    "pg_mbstd_bwd": ([_I, _I, _I, _I, _I, _VP, _I, _VP, _VP, _VP], _I),
    "pg_mbstd_r1": ([_I, _I, _I, _I, _I, _VP, _VP, _I, _VP, _VP, _VP, _VP], _I),
    "pg_bce_loss": ([_I, _VP, _I, _F, _VP, _VP, _VP, _VP], _I),
    "pg_r1_penalty": ([_I, _SZ, _VP, _VP, _VP, _VP, _VP], _I),
    "pg_drift_loss": ([_I, _VP, _F, _VP, _VP, _VP], _I),
    "pg_gp_interp": ([_I, _SZ, _VP, _VP, _VP, _VP, _VP], _I),
    "pg_gp_penalty": ([_I, _SZ, _VP, _F, _VP, _VP, _VP, _VP, _VP], _I),
    "pg_mul_add": ([_SZ, _VP, _VP, _VP, _VP, _VP], _I),
    "pg_adam": ([_SZ, _VP, _VP, _VP, _VP, _F, _F, _F, _F, _I, _VP], _I),
    "pg_randn": ([_SZ, _U64, _U64, _VP, _VP], _I),
    "pg_randn_dev": ([_SZ, _U64, _VP, _VP, _VP], _I),
    "pg_adam_table_len": ([_F, _F, _F], _I),
    "pg_adam_table": ([_F, _F, _F, _I, _VP], _I),
    "pg_adam_dev": ([_SZ, _VP, _VP, _VP, _VP, _F, _F, _F, _VP, _I, _VP, _VP], _I),
    "pg_cast": ([_I, _I, _SZ, _VP, _VP, _VP], _I),
    "pg_augment_workspace_bytes": ([_I, _I, _I], _SZ),
    "pg_augment_u8": ([_I, _I, _I, _VP, _VP, _VP, _SZ, _VP, _VP], _I),
    "pg_step_plan_create": ([_I, _I, ctypes.POINTER(ctypes.c_int), _I, _I,
                             ctypes.POINTER(ctypes.c_void_p)], _I),
    "pg_step_plan_workspace_size": ([_VP], _SZ),
    "pg_step_plan_describe": ([_VP, ctypes.c_char_p, _SZ], _I),
    "pg_step_plan_destroy": ([_VP], None),
    "pg_event_create": ([_I, ctypes.POINTER(ctypes.c_void_p)], _I),
    "pg_event_record": ([_VP, _VP], _I),
    "pg_stream_wait_event": ([_VP, _VP], _I),
    "pg_event_elapsed_ms": ([_VP, _VP, ctypes.POINTER(ctypes.c_float)], _I),
    "pg_event_destroy": ([_VP], _I),
    "pg_fill_zero": ([_VP, _SZ, _VP], _I),
    "pg_copy": ([_VP, _VP, _SZ, _VP], _I),
    "pg_record_begin": ([], _I),
    "pg_record_end": ([ctypes.POINTER(ctypes.c_void_p)], _I),
    "pg_record_count": ([_VP], _I),
    "pg_replay": ([_VP], _I),
    "pg_record_destroy": ([_VP], None),
    "pg_stream_create": ([_I, ctypes.POINTER(ctypes.c_void_p)], _I),
    "pg_stream_destroy": ([_VP], _I),
}
SYMBOLS = ["pg_last_error"] + list(_SIGS)


def load_library(path: str = LIB_PATH):
    """Load libpggan_hip.so and declare every signature.  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"pggan_amd: HIP library not built: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    lib.pg_last_error.argtypes = []
    lib.pg_last_error.restype = ctypes.c_char_p
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def _p(t):
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


class HipEvent:
    """A HIP event from pg_event_create: record on / wait from torch streams.  Unlike
    torch.cuda.Event its record releases to device scope only (no L2 writeback / invalidate
    of every XCD per record), which is all that ordering two streams of one device needs."""

    def __init__(self, ops, timing=False):
        self.lib = ops.lib
        h = ctypes.c_void_p()
        ops._chk(self.lib.pg_event_create(int(bool(timing)), ctypes.byref(h)), "event_create")
        self.h = h

    def record(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        rc = self.lib.pg_event_record(self.h, ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"event_record failed ({rc}): {self.lib.pg_last_error().decode()}")

    def wait(self, stream=None):
        """Make `stream` (default: current) wait for this event's last record."""
        s = stream if stream is not None else torch.cuda.current_stream()
        rc = self.lib.pg_stream_wait_event(ctypes.c_void_p(s.cuda_stream), self.h)
        if rc != 0:
            raise RuntimeError(f"stream_wait_event failed ({rc}): {self.lib.pg_last_error().decode()}")

    def elapsed_time(self, end):
        ms = ctypes.c_float()
        rc = self.lib.pg_event_elapsed_ms(self.h, end.h, ctypes.byref(ms))
        if rc != 0:
            raise RuntimeError(f"event_elapsed_ms failed ({rc}): {self.lib.pg_last_error().decode()}")
        return ms.value

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h is not None and h.value:
            try:
                self.lib.pg_event_destroy(h)
            except Exception:
                pass


class Recording:
    """A pg_record_* recording: replay() issues the recorded launches again (pg_replay)."""

    def __init__(self, ops, h):
        self.lib, self.h = ops.lib, h
        self.ops = ops

    def __len__(self):
        return int(self.lib.pg_record_count(self.h))

    def replay(self):
        self.ops._chk(self.lib.pg_replay(self.h), "replay")

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h is not None and h.value:
            try:
                self.lib.pg_record_destroy(h)
            except Exception:
                pass


class HipOps:
    """Tensor-level wrappers of the C ABI.  `dtype` = storage dtype of activations."""

    def __init__(self, dtype: torch.dtype = torch.float32):
        self.lib = load_library()
        assert dtype in (torch.float32, torch.bfloat16)
        self.tdtype = dtype
        self.dt = PG_F32 if dtype == torch.float32 else PG_BF16
        self._scratch = {}   # stream handle -> reduction scratch (pg_scratch_bytes)

    # -- plumbing --------------------------------------------------------
    def _s(self):
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def _scr(self):
        """The current stream's reduction scratch (include/pggan_hip.h: PG_SCRATCH_BYTES,
        zero-filled once, one per stream; every call leaves it zeroed): the deterministic
        fixed-order sums over workgroups of the RGB weight gradients, norms and biases."""
        s = torch.cuda.current_stream()
        t = self._scratch.get(s.cuda_stream)
        if t is None:
            n = int(self.lib.pg_scratch_bytes()) // 4
            t = self._scratch[s.cuda_stream] = torch.zeros(n, dtype=torch.float32, device=s.device)
        return _p(t)

    def _chk(self, rc, what):
        if rc != 0:
            msg = self.lib.pg_last_error().decode(errors="replace")
            raise RuntimeError(f"{what} failed ({rc}): {msg}")

    def _cuda(self, *ts):
        for t in ts:
            if t is not None and not t.is_cuda:
                raise RuntimeError("pggan_amd: HIP op called with a CPU tensor (no CPU fallback)")

    def _dt(self, t):
        return PG_F32 if t.dtype == torch.float32 else PG_BF16

    # -- stream ordering -----------------------------------------------------
    def side_stream(self):
        """The current device's least-priority stream (pg_stream_create): created once per
        process and device and shared by every engine (engines rebuilt per stage / batch
        size reuse it instead of leaking a stream and its hardware queue each time)."""
        dev = torch.cuda.current_device()
        st = _SIDE_STREAMS.get(dev)
        if st is None:
            h = ctypes.c_void_p()
            self._chk(self.lib.pg_stream_create(1, ctypes.byref(h)), "stream_create")
            st = _SIDE_STREAMS[dev] = torch.cuda.ExternalStream(h.value)
        return st

    def event(self, timing=False):
        """A HipEvent (device-scope release; see pg_event_create)."""
        return HipEvent(self, timing)

    # -- device memory (recordable) ------------------------------------------
    def zero_(self, t):
        """t.zero_() through the library (pg_fill_zero: part of a recording)."""
        self._cuda(t)
        assert t.is_contiguous()
        self._chk(self.lib.pg_fill_zero(_p(t), t.numel() * t.element_size(), self._s()), "fill_zero")

    def copy_(self, dst, src):
        """dst.copy_(src) for same-dtype contiguous device tensors (pg_copy: recordable)."""
        self._cuda(dst, src)
        assert dst.is_contiguous() and src.is_contiguous() and dst.dtype == src.dtype
        assert dst.numel() == src.numel()
        self._chk(self.lib.pg_copy(_p(dst), _p(src), dst.numel() * dst.element_size(), self._s()),
                  "copy")

    # -- launch recorder (include/pggan_hip.h: pg_record_*) ------------------
    def record_begin(self):
        self._chk(self.lib.pg_record_begin(), "record_begin")

    def record_end(self):
        """The launches since record_begin as a Recording (replay() re-issues them)."""
        h = ctypes.c_void_p()
        self._chk(self.lib.pg_record_end(ctypes.byref(h)), "record_end")
        return Recording(self, h)

    # -- step plan ---------------------------------------------------------
    def step_plan(self, depths, stage, batch):
        """(workspace bytes, description) of pg_step_plan_create for one training step."""
        arr = (ctypes.c_int * len(depths))(*depths)
        h = ctypes.c_void_p()
        self._chk(self.lib.pg_step_plan_create(self.dt, len(depths), arr, stage, batch,
                                               ctypes.byref(h)), "step_plan_create")
        try:
            ws = int(self.lib.pg_step_plan_workspace_size(h))
            buf = ctypes.create_string_buffer(16384)
            self._chk(self.lib.pg_step_plan_describe(h, buf, len(buf)), "step_plan_describe")
            return ws, buf.value.decode()
        finally:
            self.lib.pg_step_plan_destroy(h)

    # -- conv ------------------------------------------------------------
    def packed_elems(self, mode, cout, cin):
        return int(self.lib.pg_conv3x3_packed_elems(mode, cout, cin))

    def conv_pack(self, mode, w, scale, out):
        self._cuda(w, out)
        cout, cin = w.shape[0], w.shape[1]
        self._chk(self.lib.pg_conv3x3_pack(self._dt(out), mode, cout, cin, _p(w), scale, _p(out),
                                           self._s()), "conv3x3_pack")

    def pack_table(self, entries):
        """entries: [(w, bias|None, fwd, dgrad, bias_scaled, scale)] -> (device table, n,
        max_tiles) for conv_pack_batch.  The table holds raw pointers: rebuild it if any of
        the tensors is reallocated."""
        n = len(entries)
        arr = (PackItem * n)()
        mt = 1
        for i, (w, b, pf, pd, bs, sc) in enumerate(entries):
            self._cuda(w, b, pf, pd, bs)
            cout, cin = w.shape[0], w.shape[1]
            arr[i] = PackItem(_p(w), _p(b), _p(pf), _p(pd), _p(bs), float(sc), cout, cin, 0)
            O = max((cout + 15) // 16 * 16, _cinp(cout))
            C = max(_cinp(cin), (cin + 15) // 16 * 16)
            mt = max(mt, ((O + 31) // 32) * ((C + 31) // 32))
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        return raw.to(entries[0][0].device), n, mt

    def conv_pack_batch(self, table):
        dev, n, mt = table
        self._cuda(dev)
        self._chk(self.lib.pg_conv3x3_pack_batch(self.dt, n, _p(dev), mt, self._s()),
                  "conv3x3_pack_batch")

    def conv3x3(self, x, wpk, y, *, B, H, W, cin, cout, flags, slope=0.2, out_scale=1.0,
                bias=None, aux=None, y2=None, ws=None, xbits=None):
        """ws: optional fp32 workspace tensor enabling split-K (see conv_workspace_bytes).
        Bit tensors (aux with CONV_AUX_BITS, y2 with CONV_Y2_BITS, xbits with CONV_X_BITS)
        are uint8 [B, H, W, bytes per pixel]."""
        self._cuda(x, wpk, y, bias, aux, y2, ws, xbits)
        d = ConvDesc(B, H, W, cin, cout, x.shape[-1], y.shape[-1],
                     aux.shape[-1] if aux is not None else 0,
                     y2.shape[-1] if y2 is not None else 0, flags, slope, out_scale,
                     xbits.shape[-1] if xbits is not None else 0)
        wsb = ws.numel() * ws.element_size() if ws is not None else 0
        self._chk(self.lib.pg_conv3x3_fwd_ex(self._dt(y), ctypes.byref(d), _p(x), _p(xbits),
                                             _p(wpk), _p(bias), _p(aux), _p(y), _p(y2), _p(ws),
                                             wsb, self._s()),
                  "conv3x3_fwd")

    def conv3x3_rgbw(self, x, wpk, *, B, H, W, cin, cout, flags, aux, img, s, dw, db,
                     slope=0.2, out_scale=1.0):
        """The input-gradient conv whose result is the fromRGB output's gradient, with the
        fromRGB weight / bias gradients (dw [C*3], db [C], accumulated) in its epilogue
        instead of storing the result (include/pggan_hip.h: PG_CONV_RGBW)."""
        self._cuda(x, wpk, aux, img, dw, db)
        d = ConvDesc(B, H, W, cin, cout, x.shape[-1], cout, aux.shape[-1], 0,
                     flags | CONV_RGBW, slope, out_scale, 0)
        self._chk(self.lib.pg_conv3x3_rgbw(self._dt(x), ctypes.byref(d), _p(x), _p(wpk), _p(aux),
                                           _p(img), float(s), _p(dw), _p(db),
                                           self._scr(), self._s()),
                  "conv3x3_rgbw")

    def conv3x3_rgbo(self, x, wpk, y, *, B, H, W, cin, cout, flags, bias, w_rgb, b_rgb, c, img,
                     y2=None, slope=0.2):
        """The generator's top conv b forward with PixelNorm (flags PIXNORM | LRELU | BIAS) and
        the toRGB output img = c (W_rgb y + b_rgb) of its stored y in the epilogue
        (include/pggan_hip.h: PG_CONV_RGBO); y and y2 as conv3x3."""
        self._cuda(x, wpk, y, bias, y2, w_rgb, b_rgb, img)
        d = ConvDesc(B, H, W, cin, cout, x.shape[-1], y.shape[-1], 0,
                     y2.shape[-1] if y2 is not None else 0, flags | CONV_RGBO, slope, 1.0, 0)
        self._chk(self.lib.pg_conv3x3_rgbo(self._dt(y), ctypes.byref(d), _p(x), _p(wpk), _p(bias),
                                           _p(y), _p(y2), _p(w_rgb), _p(b_rgb), float(c), _p(img),
                                           self._s()),
                  "conv3x3_rgbo")

    def conv3x3_rgbd(self, x, wpk, *, B, H, W, cin, cout, flags, aux, w_rgb, f, gimg,
                     norms=None, dw=None, s=0.0, slope=0.2, out_scale=1.0):
        """The input-gradient conv whose result is the fromRGB output's gradient gz, with the
        fromRGB input gradient gimg = f W^T gz (written), the per-sample squared norms of gimg
        (norms, accumulated) and s * sum gz (x) gimg (dw, accumulated) in its epilogue instead of
        storing gz (include/pggan_hip.h: PG_CONV_RGBD)."""
        self._cuda(x, wpk, aux, w_rgb, gimg, norms, dw)
        d = ConvDesc(B, H, W, cin, cout, x.shape[-1], cout, aux.shape[-1], 0,
                     flags | CONV_RGBD, slope, out_scale, 0)
        self._chk(self.lib.pg_conv3x3_rgbd(self._dt(x), ctypes.byref(d), _p(x), _p(wpk), _p(aux),
                                           _p(w_rgb), float(f), _p(gimg), _p(norms), _p(dw),
                                           float(s), self._scr(), self._s()),
                  "conv3x3_rgbd")

    def conv_supported(self, *, B, H, W, cin, cout, flags, ws_bytes=0):
        """Whether the conv kernel picked for this shape supports `flags` (fused epilogues)."""
        if flags & CONV_GZ_BITS:       # the weight-gradient operand form (bf16 kernel only)
            return self.dt == PG_BF16 and H % 2 == 0 and W % 2 == 0 and cout % 8 == 0
        d = ConvDesc(B, H, W, cin, cout, 0, 0, 0, 0, flags, 0.2, 1.0, 0)
        return bool(self.lib.pg_conv3x3_supported(self.dt, ctypes.byref(d), ws_bytes))

    def conv_workspace_bytes(self, *, B, H, W, cin, cout):
        d = ConvDesc(B, H, W, cin, cout, 0, 0, 0, 0, 0, 0.0, 1.0, 0)
        return int(self.lib.pg_conv3x3_workspace_size(ctypes.byref(d)))

    def wgrad_workspace_bytes(self, *, B, H, W, cin, cout, ups=False):
        d = ConvDesc(B, H, W, cin, cout, 0, 0, 0, 0, CONV_UPS_IN if ups else 0, 0.0, 1.0, 0)
        return int(self.lib.pg_conv3x3_wgrad_workspace_size(self.dt, ctypes.byref(d)))

    def conv_wgrad(self, x, gz, dw, *, B, H, W, cin, cout, ups, scale, db=None, ws=None,
                   gzbits=None, slope=0.2):
        """ws: optional fp32 workspace (see wgrad_workspace_bytes) for split reductions.
        gzbits: the gradient is up2(gz) * lrelu'(gzbits) (gz at H/2, bits uint8 at H)."""
        self._cuda(x, gz, dw, db, ws, gzbits)
        fl = (CONV_UPS_IN if ups else 0) | (CONV_GZ_BITS if gzbits is not None else 0)
        d = ConvDesc(B, H, W, cin, cout, x.shape[-1], gz.shape[-1], 0, 0, fl, slope, 1.0,
                     gzbits.shape[-1] if gzbits is not None else 0)
        wsb = ws.numel() * ws.element_size() if ws is not None else 0
        self._chk(self.lib.pg_conv3x3_wgrad_ex(self._dt(gz), ctypes.byref(d), _p(x), _p(gz),
                                               _p(gzbits), scale, _p(dw), _p(db), _p(ws), wsb,
                                               self._s()),
                  "conv3x3_wgrad")

    def bias_grad(self, g, db, C, scale):
        self._cuda(g, db)
        npix = g.numel() // g.shape[-1]
        self._chk(self.lib.pg_bias_grad(self._dt(g), npix, C, g.shape[-1], _p(g), scale, _p(db),
                                        self._scr(), self._s()), "bias_grad")

    # -- pixel norm ------------------------------------------------------
    def pixnorm(self, x, y, C):
        self._cuda(x, y)
        npix = x.numel() // x.shape[-1]
        self._chk(self.lib.pg_pixnorm_fwd(self._dt(x), npix, C, x.shape[-1], _p(x), _p(y),
                                          self._s()), "pixnorm_fwd")

    def pixnorm_lrelu_bwd(self, u, gy, gz, C, slope, mask=True):
        self._cuda(u, gy, gz)
        npix = u.numel() // u.shape[-1]
        self._chk(self.lib.pg_pixnorm_lrelu_bwd(self._dt(u), npix, C, u.shape[-1], _p(u), _p(gy),
                                                slope, 1 if mask else 0, _p(gz), self._s()),
                  "pixnorm_lrelu_bwd")

    def pixnorm_lrelu_bwd_y(self, y, r, gy, gz, C, slope):
        """Backward of lrelu -> PixelNorm from the fused conv's normalised output y and its
        per-pixel factor r (fp32, one per pixel)."""
        self._cuda(y, r, gy, gz)
        npix = y.numel() // y.shape[-1]
        self._chk(self.lib.pg_pixnorm_lrelu_bwd_y(self._dt(y), npix, C, y.shape[-1], _p(y), _p(r),
                                                  _p(gy), slope, _p(gz), self._s()),
                  "pixnorm_lrelu_bwd_y")

    # -- elementwise -------------------------------------------------------
    def unpool_mask(self, g, y, out, *, B, H, W, C, scale, slope, ups, bits=None):
        """bits: the lrelu' operand as sign bits (uint8 [B, H, W, C / 8]) instead of y."""
        self._cuda(g, y, out, bits)
        if bits is not None:
            self._chk(self.lib.pg_unpool_mask_bits(self._dt(out), B, H, W, C, g.shape[-1], _p(g),
                                                   _p(bits), scale, slope, 1 if ups else 0,
                                                   out.shape[-1], _p(out), self._s()),
                      "unpool_mask_bits")
            return
        self._chk(self.lib.pg_unpool_mask(self._dt(out), B, H, W, C, g.shape[-1], _p(g),
                                          y.shape[-1] if y is not None else 0, _p(y), scale, slope,
                                          1 if ups else 0, out.shape[-1], _p(out), self._s()),
                  "unpool_mask")

    def avgpool2(self, x, y, *, B, H, W, C):
        self._cuda(x, y)
        self._chk(self.lib.pg_avgpool2(self._dt(x), B, H, W, C, x.shape[-1], _p(x), y.shape[-1],
                                       _p(y), self._s()), "avgpool2")

    def blend(self, a, x, b, y, out):
        self._cuda(x, y, out)
        self._chk(self.lib.pg_blend(self._dt(out), out.numel(), a, _p(x), b, _p(y), _p(out),
                                    self._s()), "blend")

    # -- RGB ---------------------------------------------------------------
    def rgb_out(self, x, w, b, c, img, *, B, R, C, xp=None, wp=None, bp=None, cp=0.0, Cp=0,
                alpha=1.0):
        self._cuda(x, w, b, img, xp, wp, bp)
        self._chk(self.lib.pg_rgb_out(self._dt(x), B, R, C, x.shape[-1], _p(x), _p(w), _p(b), c, Cp,
                                      xp.shape[-1] if xp is not None else 0, _p(xp), _p(wp), _p(bp),
                                      cp, alpha, _p(img), self._s()), "rgb_out")

    def rgb_out_bwd(self, x, w, c, gimg, gx, dw, db, *, B, R, C, xp=None, wp=None, cp=0.0, Cp=0,
                    alpha=1.0, gxp=None, dwp=None, dbp=None):
        self._cuda(x, w, gimg, gx, dw, db, xp, wp, gxp, dwp, dbp)
        self._chk(self.lib.pg_rgb_out_bwd(self._dt(x), B, R, C, x.shape[-1], _p(x), _p(w), c, Cp,
                                          xp.shape[-1] if xp is not None else 0, _p(xp), _p(wp), cp,
                                          alpha, _p(gimg), _p(gx), _p(gxp), _p(dw), _p(db), _p(dwp),
                                          _p(dbp), self._scr(), self._s()), "rgb_out_bwd")

    def rgb_out_bwd_pn(self, y, r, w, c, gimg, gz, *, B, R, C, slope, dw=None, db=None):
        """toRGB input gradient + the PixelNorm / LReLU backward of its input y (pg_rgb_out_bwd_pn);
        with dw / db also the toRGB weight / bias gradients of the same pass (_wg)."""
        if dw is not None:
            self._cuda(y, r, w, gimg, gz, dw, db)
            self._chk(self.lib.pg_rgb_out_bwd_pn_wg(self._dt(y), B, R, C, y.shape[-1], _p(y), _p(r),
                                                    _p(w), c, _p(gimg), slope, gz.shape[-1], _p(gz),
                                                    _p(dw), _p(db), self._scr(), self._s()),
                      "rgb_out_bwd_pn_wg")
            return
        self._cuda(y, r, w, gimg, gz)
        self._chk(self.lib.pg_rgb_out_bwd_pn(self._dt(y), B, R, C, y.shape[-1], _p(y), _p(r), _p(w), c,
                                             _p(gimg), slope, gz.shape[-1], _p(gz), self._s()),
                  "rgb_out_bwd_pn")

    def _src(self, img):
        """pg_img_src of an image operand (a tensor or an ImgMix)."""
        if img is None:
            return None
        if isinstance(img, ImgMix):
            self._cuda(img.x0, img.x1, img.a, img.c)
            return ImgSrcDesc(img.x0.data_ptr(), img.x1.data_ptr() if img.x1 is not None else None,
                              img.a.data_ptr() if img.a is not None else None,
                              img.c.data_ptr() if img.c is not None else None)
        self._cuda(img)
        return ImgSrcDesc(img.data_ptr(), None, None, None)

    def from_rgb(self, img, w, b, c, y, *, B, R, C, down, slope=0.2, mask_y=None, ybits=None,
                 mask_bits=None):
        """ybits: also write the lrelu sign bits of y (uint8 [B, R, R, C / 8]); mask_bits: the
        tangent's lrelu' mask from those bits instead of mask_y (pg_from_rgb_bits)."""
        self._cuda(w, b, y, mask_y, ybits, mask_bits)
        src = self._src(img)
        if ybits is not None or mask_bits is not None:
            self._chk(self.lib.pg_from_rgb_bits(self._dt(y), B, R, C, ctypes.byref(src),
                                                1 if down else 0, _p(w), _p(b), c, slope,
                                                _p(mask_bits), y.shape[-1], _p(y), _p(ybits),
                                                self._s()), "from_rgb_bits")
            return
        self._chk(self.lib.pg_from_rgb_src(self._dt(y), B, R, C, ctypes.byref(src), 1 if down else 0,
                                           _p(w), _p(b), c, slope, _p(mask_y), y.shape[-1], _p(y),
                                           self._s()), "from_rgb")

    def from_rgb_bwd(self, gz, w, c, *, B, R, C, down, img=None, gimg=None, dw=None, db=None,
                     gimg_overwrite=False, norms=None):
        """gimg_overwrite: write gimg instead of accumulating into it; norms: += per-sample sum
        of squares of the final gimg (the penalties' squared norms)."""
        self._cuda(gz, w, gimg, dw, db, norms)
        src = self._src(img)
        self._chk(self.lib.pg_from_rgb_bwd_src(self._dt(gz), B, R, C,
                                               ctypes.byref(src) if src is not None else None,
                                               1 if down else 0, _p(w), c, gz.shape[-1], _p(gz),
                                               _p(gimg), 1 if gimg_overwrite else 0, _p(norms),
                                               _p(dw), _p(db), self._scr(), self._s()), "from_rgb_bwd")

    def penalty_scale(self, mode, norms, w, loss, scale):
        """mode "r1" / "wgan-gp": the penalty into loss[0] and the per-sample tangent scale
        from the squared norms (pg_penalty_scale)."""
        self._cuda(norms, loss, scale)
        self._chk(self.lib.pg_penalty_scale(0 if mode == "r1" else 1, norms.numel(), _p(norms), w,
                                            _p(loss), _p(scale), self._s()), "penalty_scale")

    def img_fade(self, x, alpha, out):
        self._cuda(x, out)
        B, C, R, _ = x.shape
        self._chk(self.lib.pg_img_fade(B, C, R, _p(x), alpha, _p(out), self._s()), "img_fade")

    # -- linear ------------------------------------------------------------
    def _lin(self, B, K, N, flags, scale, slope, x_t, y_t):
        in_cs = x_t.shape[-1] if (flags & LIN_IN_CHW) else 0
        out_cs = y_t.shape[-1] if (flags & LIN_OUT_CHW) else 0
        if x_t.dtype == torch.float32 and self.dt != PG_F32:
            flags |= LIN_F32_IN
        if y_t.dtype == torch.float32 and self.dt != PG_F32:
            flags |= LIN_F32_OUT
        return LinearDesc(B, K, N, in_cs, out_cs, flags, scale, slope)

    def _lin_ws(self, d, pass_, device):
        """fp32 split-reduction workspace of the bf16 linear kernels (grown on demand,
        reused: launches are stream-ordered)."""
        need = int(self.lib.pg_linear_workspace_size(self.dt, ctypes.byref(d), pass_))
        if not need:
            return None, 0
        ws = getattr(self, "_linws", None)
        if ws is None or ws.numel() * 4 < need or ws.device != device:
            ws = self._linws = torch.empty((need + 3) // 4, dtype=torch.float32, device=device)
        return ws, ws.numel() * 4

    def linear(self, x, w, b, y, *, B, flags, scale, slope=0.2, aux=None):
        self._cuda(x, w, b, y, aux)
        N, K = w.shape
        d = self._lin(B, K, N, flags, scale, slope, x, y)
        ws, wsb = self._lin_ws(d, 0, y.device)
        self._chk(self.lib.pg_linear_fwd_ws(self.dt, ctypes.byref(d), _p(x), _p(w), _p(b), _p(aux),
                                            _p(y), _p(ws), wsb, self._s()), "linear_fwd")

    def linear_dgrad(self, gy, w, gx, *, B, flags, scale, slope=0.2, aux=None):
        self._cuda(gy, w, gx, aux)
        N, K = w.shape
        d = self._lin(B, K, N, flags, scale, slope, gx, gy)
        ws, wsb = self._lin_ws(d, 1, gx.device)
        self._chk(self.lib.pg_linear_dgrad_ws(self.dt, ctypes.byref(d), _p(gy), _p(w), _p(aux),
                                              _p(gx), _p(ws), wsb, self._s()), "linear_dgrad")

    def linear_wgrad(self, x, gy, dw, db, *, B, flags, scale):
        self._cuda(x, gy, dw, db)
        N, K = dw.shape
        d = self._lin(B, K, N, flags, scale, 0.0, x, gy)
        self._chk(self.lib.pg_linear_wgrad(self.dt, ctypes.byref(d), _p(x), _p(gy), _p(dw), _p(db),
                                           self._s()), "linear_wgrad")

    # -- minibatch stddev ----------------------------------------------------
    def mbstd_fwd(self, x, y, *, B, HW, C):
        self._cuda(x, y)
        self._chk(self.lib.pg_mbstd_fwd(self._dt(x), B, HW, C, x.shape[-1], _p(x), y.shape[-1],
                                        _p(y), self._s()), "mbstd_fwd")

    def mbstd_bwd(self, x, gy, gx, *, B, HW, C):
        self._cuda(x, gy, gx)
        self._chk(self.lib.pg_mbstd_bwd(self._dt(x), B, HW, C, x.shape[-1], _p(x), gy.shape[-1],
                                        _p(gy), _p(gx), self._s()), "mbstd_bwd")

    def mbstd_r1(self, x, a, gy, tout, inj, *, B, HW, C):
        self._cuda(x, a, gy, tout, inj)
        self._chk(self.lib.pg_mbstd_r1(self._dt(x), B, HW, C, x.shape[-1], _p(x), _p(a),
                                       gy.shape[-1], _p(gy), _p(tout), _p(inj), self._s()),
                  "mbstd_r1")

    # -- losses / optimizer / rng ------------------------------------------
    def bce(self, logits, target, w, loss, u, h):
        self._cuda(logits, loss, u, h)
        self._chk(self.lib.pg_bce_loss(logits.numel(), _p(logits), 1 if target else 0, w, _p(loss),
                                       _p(u), _p(h), self._s()), "bce_loss")

    def drift(self, logits, w, loss, u):
        self._cuda(logits, loss, u)
        self._chk(self.lib.pg_drift_loss(logits.numel(), _p(logits), w, _p(loss), _p(u), self._s()),
                  "drift_loss")

    def r1_penalty(self, g, B, r1, gbar):
        self._cuda(g, r1, gbar)
        self._chk(self.lib.pg_r1_penalty(B, g.numel(), _p(g), _p(r1), _p(gbar), self._scr(),
                                         self._s()), "r1_penalty")

    def gp_interp(self, xr, xf, eps, out):
        self._cuda(xr, xf, eps, out)
        B = xr.shape[0]
        self._chk(self.lib.pg_gp_interp(B, xr.numel() // B, _p(xr), _p(xf), _p(eps), _p(out),
                                        self._s()), "gp_interp")

    def gp_penalty(self, g, w, gp, norms, gbar):
        self._cuda(g, gp, norms, gbar)
        B = g.shape[0]
        self._chk(self.lib.pg_gp_penalty(B, g.numel() // B, _p(g), w, _p(gp), _p(norms), _p(gbar),
                                         self._scr(), self._s()), "gp_penalty")

    def mul_add(self, x, y, z, out):
        self._cuda(x, y, z, out)
        self._chk(self.lib.pg_mul_add(out.numel(), _p(x), _p(y), _p(z), _p(out), self._s()),
                  "mul_add")

    def adam(self, p, g, m, v, *, lr, beta1, beta2, eps, step):
        self._cuda(p, g, m, v)
        self._chk(self.lib.pg_adam(p.numel(), _p(p), _p(g), _p(m), _p(v), lr, beta1, beta2, eps,
                                   step, self._s()), "adam")

    def adam_table(self, lr, beta1, beta2, device):
        """Device table of pg_adam_dev's bias corrections for (lr, beta1, beta2), cached."""
        key = (float(lr), float(beta1), float(beta2), str(device))
        tabs = self.__dict__.setdefault("_adam_tabs", {})
        if key not in tabs:
            n = int(self.lib.pg_adam_table_len(lr, beta1, beta2))
            host = (ctypes.c_float * (2 * n))()
            self._chk(self.lib.pg_adam_table(lr, beta1, beta2, n, host), "adam_table")
            t = torch.frombuffer(bytearray(bytes(host)), dtype=torch.float32).to(device)
            tabs[key] = (t, n)
        return tabs[key]

    def adam_dev(self, p, g, m, v, *, lr, beta1, beta2, eps, step_dev):
        """Adam with the step count in device memory (bumped by the launch): replayable."""
        self._cuda(p, g, m, v, step_dev)
        tab, n = self.adam_table(lr, beta1, beta2, p.device)
        self._chk(self.lib.pg_adam_dev(p.numel(), _p(p), _p(g), _p(m), _p(v), beta1, beta2, eps,
                                       _p(tab), n, _p(step_dev), self._s()), "adam_dev")

    def randn_dev(self, out, seed, offset_dev):
        """pg_randn with the offset in device memory (advanced by out.numel())."""
        self._cuda(out, offset_dev)
        self._chk(self.lib.pg_randn_dev(out.numel(), seed, _p(offset_dev), _p(out), self._s()),
                  "randn_dev")

    def randn(self, out, seed, offset):
        self._cuda(out)
        self._chk(self.lib.pg_randn(out.numel(), seed, offset, _p(out), self._s()), "randn")

    def augment_u8(self, src, params, dst, ws=None):
        """src uint8 [B,H,W,3], params fp32 [B,12] (include/pggan_hip.h), dst fp32
        [B,3,H,W]: flip + ColorJitter + ToTensor + Normalize (lib/dataset.py:106-117)."""
        self._cuda(src, params, dst)
        B, H, W, _ = src.shape
        need = self.lib.pg_augment_workspace_bytes(B, H, W)
        if ws is None or ws.numel() * 4 < need:
            ws = torch.empty((need + 3) // 4, dtype=torch.float32, device=src.device)
        self._chk(self.lib.pg_augment_u8(B, H, W, _p(src), _p(params), _p(ws), ws.numel() * 4,
                                         _p(dst), self._s()), "augment_u8")
        return ws

    def cast(self, x, y):
        self._cuda(x, y)
        self._chk(self.lib.pg_cast(self._dt(x), self._dt(y), x.numel(), _p(x), _p(y), self._s()),
                  "cast")
