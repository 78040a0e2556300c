"""ctypes binding for the segment writer's native helpers (csrc/segment_tools.c)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "libdruid_tools.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"{_LIB_PATH} missing: run __graft_entry__.build() (make -C incubator-druid_amd/csrc)")
        l = ctypes.CDLL(_LIB_PATH)
        l.dgt_concise_encode.restype = ctypes.c_int64
        l.dgt_concise_encode.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        l.dgt_concise_encode_column.restype = ctypes.c_int64
        l.dgt_concise_encode_column.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                                ctypes.c_void_p, ctypes.c_void_p]
        l.dgt_lzf_compress.restype = ctypes.c_int64
        l.dgt_lzf_compress.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
        _lib = l
    return _lib


def concise_encode(rows) -> np.ndarray:
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    out = np.empty(len(rows) + 2, dtype=np.int32)
    n = lib().dgt_concise_encode(rows.ctypes.data, len(rows), out.ctypes.data)
    return out[:n].copy()


def concise_encode_column(ids, cardinality: int):
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    words = np.empty(len(ids) + 2 * cardinality + 2, dtype=np.int32)
    counts = np.empty(max(cardinality, 1), dtype=np.int64)
    n = lib().dgt_concise_encode_column(ids.ctypes.data, len(ids), cardinality, words.ctypes.data,
                                        counts.ctypes.data)
    if n < 0:
        raise ValueError("dictionary id out of range")
    return words[:n], counts[:cardinality]


def lzf_compress(data: bytes) -> bytes:
    """compress-lzf chunked LZF (LZFEncoder.appendEncoded layout) of one block."""
    cap = len(data) + len(data) // 16 + 64
    out = ctypes.create_string_buffer(cap)
    n = lib().dgt_lzf_compress(data, len(data), out, cap)
    if n < 0:
        raise RuntimeError("LZF compression failed")
    return out.raw[:n]
