"""CPU suite: the C-ABI library builds for gfx950, loads, and exports every symbol include/druidgpu.h declares."""
import ctypes
import importlib
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(REPO, "include", "druidgpu.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dg_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header_symbols():
    N = importlib.import_module("incubator-druid_amd._native")
    lib = ctypes.CDLL(N.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"missing export {s}"
    assert sorted(N.EXPORTS) == syms


def test_abi_version_and_structs():
    N = importlib.import_module("incubator-druid_amd._native")
    assert N.lib().dg_abi_version() == 3
    # struct layouts the header fixes (LP64)
    assert ctypes.sizeof(N.dg_filter) == 64
    assert ctypes.sizeof(N.dg_agg) == 32
    assert ctypes.sizeof(N.dg_scan) == 72
    assert ctypes.sizeof(N.dg_metrics) == 104
    assert ctypes.sizeof(N.dg_topn_lists) == 40
    assert ctypes.sizeof(N.dg_topn) == 56


def test_gpu_kernels_are_gfx950_code_objects():
    N = importlib.import_module("incubator-druid_amd._native")
    data = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    for k in (b"k_lz4_decode", b"k_concise_or", b"k_roaring_or", b"k_scan_agg", b"k_topn_radix", b"k_topn_compact", b"k_gb_keygen",
              b"k_rs_scatter", b"k_gb_reduce", b"k_fsum_runs"):
        assert k in data, k


def test_no_device_in_container_is_reported_not_faked():
    N = importlib.import_module("incubator-druid_amd._native")
    n = ctypes.c_int(-1)
    N.lib().dg_device_count(ctypes.byref(n))
    if n.value == 0:
        h = ctypes.c_void_p()
        assert N.lib().dg_context_create(0, ctypes.byref(h)) == 7  # DG_ERR_DEVICE, no CPU fallback
