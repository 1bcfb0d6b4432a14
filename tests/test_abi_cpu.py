"""The C-ABI library builds, loads without a GPU, exports every symbol include/m3.h declares,
and fails loudly (no CPU fallback) when no device is present."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, gpu_available
from match3tile import _native


def header_symbols():
    text = open(os.path.join(ROOT, "include", "m3.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(m3_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_binding_list():
    assert header_symbols() == sorted(_native.EXPORTS)


def test_library_exports_every_header_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (m3_\w+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing


def test_no_torch_in_product_library():
    out = subprocess.run(["ldd", _native.LIB_PATH], capture_output=True, text=True).stdout
    libs = [line.split()[0] for line in out.splitlines() if line.strip()]  # names only, not load addresses
    assert not [x for x in libs if "torch" in x or "c10" in x], libs
    assert any("libamdhip64" in x for x in libs) and any("librccl" in x for x in libs), libs


def test_loads_and_reports_shapes():
    L = _native.lib()
    assert L.m3_abi_version() == 1
    assert _native.supported(9, 9, 6) and _native.supported(16, 16, 8)
    # any other BoardConfig in the 16 x 16 frame: rows / columns 3..16, types 2..15
    assert _native.supported(7, 7, 5) and _native.supported(3, 3, 3) and _native.supported(16, 3, 15)
    assert _native.supported(9, 9, 2) and _native.supported(5, 5, 2)
    assert _native.supported(8, 10, 5)  # rows < columns: resets only (the reference raises on a step)
    # a side above 16: the 32 x 32 frame
    assert _native.supported(20, 20, 6) and _native.supported(17, 9, 6) and _native.supported(32, 32, 15)
    assert _native.supported(9, 17, 6) and _native.supported(32, 3, 4)
    # types 16..31: the 5-bit token layout
    assert _native.supported(9, 9, 16) and _native.supported(12, 12, 31) and _native.supported(20, 20, 24)
    for bad in ((2, 9, 6), (33, 9, 6), (9, 33, 6), (9, 9, 32), (9, 9, 1)):
        assert not _native.supported(*bad), bad
    a, w = np.zeros(1, np.int32), np.zeros(1, np.int32)
    _native.check(L.m3_action_space(9, 9, _native.ptr(a), _native.ptr(w)))
    assert a[0] == 144 and w[0] == 5


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU error path")
def test_fails_loudly_without_gpu():
    assert _native.device_count() == 0
    with pytest.raises(_native.M3Error) as e:
        _native.Context(9, 9, 6)
    assert e.value.code == -5


def test_unsupported_shape_error():
    with pytest.raises(_native.M3Error) as e:
        _native.Context(33, 9, 6)
    assert e.value.code == -2
