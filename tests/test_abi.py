"""The C-ABI boundary without a GPU: libpggan_hip.so loads, exports every function
include/pggan_hip.h declares, the ctypes table of pggan_amd/_lib.py declares each of them,
and the host-only entry points (step plan, workspace sizes, packed sizes) answer."""
import ctypes
import os
import re

import pytest

from pggan_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pggan_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pg_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libpggan_hip.so not built")
    return _lib.load_library()


def test_every_declared_symbol_is_exported_and_bound(lib):
    names = header_functions()
    assert len(names) >= 40, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared in include/pggan_hip.h but not exported: {missing}"
    unbound = [n for n in names if n not in _lib.SYMBOLS]
    assert not unbound, f"exported but missing from pggan_amd/_lib.py _SIGS: {unbound}"


def test_step_plan_on_the_host(lib):
    """pg_step_plan_* at the benchmark configuration (C5: stage 8, batch 4, bf16): one line
    per conv layer of G and D, the low-resolution kernel at 4^2 / 8^2, the persistent
    high-resolution tiles at 1024^2, a split workspace for the 16^2 convs."""
    depths = [512, 512, 512, 512, 256, 128, 64, 32, 16]
    ops = _lib.HipOps.__new__(_lib.HipOps)    # host-only: no tensors, no stream
    ops.lib, ops.dt = lib, _lib.PG_BF16
    ws, text = ops.step_plan(depths, 8, 4)
    lines = text.strip().splitlines()
    assert lines[0].startswith("stage 8 batch 4 dtype bf16")
    assert len(lines) == 1 + 2 * (1 + 2 * 8)
    assert ws > 0 and "splitK" in text
    assert any(l.startswith("G a") and "8x8" in l and "conv_lr" in l for l in lines), text
    assert any(l.startswith("D b") and "1024x1024" in l and "conv_hr" in l for l in lines), text
    with pytest.raises(RuntimeError):
        ops.step_plan(depths, 9, 4)          # stage beyond the depth list
