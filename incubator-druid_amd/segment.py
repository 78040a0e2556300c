"""Device-resident segments (the QueryableIndex / StorageAdapter side of the boundary).

``GpuSegment(path, device)`` maps a Druid v9 segment directory into HBM through
``dg_segment_attach`` (IndexIO.loadIndex, processing/.../segment/IndexIO.java:569-663) and exposes
the StorageAdapter facts the runners need: row count, data interval, min/max time
(StorageAdapter.getMinTime/getMaxTime), column types and dictionaries (lookupName).
"""
from __future__ import annotations

import ctypes
import threading
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _native as N
from . import ordering as O


class GpuContext:
    """One HIP device + stream (``dg_context``); shared by every segment attached to that device."""

    _by_device: Dict[int, "GpuContext"] = {}
    _lock = threading.Lock()

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        N.check(N.lib().dg_context_create(device, ctypes.byref(h)))
        self.device = device
        self.handle = h

    @classmethod
    def get(cls, device: int = 0) -> "GpuContext":
        with cls._lock:
            if device not in cls._by_device:
                cls._by_device[device] = GpuContext(device)
            return cls._by_device[device]

    def set_stream(self, hip_stream_ptr: Optional[int]):
        N.check(N.lib().dg_context_set_stream(self.handle, ctypes.c_void_p(hip_stream_ptr or 0)))


def device_count() -> int:
    n = ctypes.c_int()
    N.lib().dg_device_count(ctypes.byref(n))
    return n.value


class GpuSegment:
    """A Druid segment resident on one GPU (QueryableIndexSegment equivalent)."""

    _ids = 0

    def __init__(self, path: str, device: int = 0, context: Optional[GpuContext] = None):
        self.context = context or GpuContext.get(device)
        h = ctypes.c_void_p()
        N.check(N.lib().dg_segment_attach(self.context.handle, path.encode(), ctypes.byref(h)))
        self._init(h, path)

    @classmethod
    def from_handle(cls, handle: ctypes.c_void_p, context: GpuContext, name: str) -> "GpuSegment":
        """A segment the engine built otherwise (dg_segment_from_rows: an in-memory index)."""
        seg = cls.__new__(cls)
        seg.context = context
        seg._init(handle, name)
        return seg

    def _init(self, h: ctypes.c_void_p, path: str):
        self.handle = h
        self.path = path
        GpuSegment._ids += 1
        self.identifier = f"{path}#{GpuSegment._ids}"
        L = N.lib()
        self.num_rows = int(L.dg_segment_num_rows(h))
        s, e = ctypes.c_int64(), ctypes.c_int64()
        L.dg_segment_interval(h, ctypes.byref(s), ctypes.byref(e))
        self.interval = (s.value, e.value)
        L.dg_segment_time_bounds(h, ctypes.byref(s), ctypes.byref(e))
        self.min_time, self.max_time = s.value, e.value
        self._dicts: Dict[str, List[Optional[str]]] = {}
        self._orders: Dict[Tuple[str, int], O.DictionaryOrder] = {}
        self._types: Dict[str, int] = {}  # a segment's columns never change once attached / built
        self._values: Dict[str, Dict[int, Optional[str]]] = {}  # dim_value lookups already made

    # -- StorageAdapter-ish facts ------------------------------------------------------------
    def columns(self) -> List[str]:
        L = N.lib()
        return [L.dg_segment_column_name(self.handle, i).decode() for i in range(L.dg_segment_num_columns(self.handle))]

    def column_type(self, name: str) -> int:
        t = self._types.get(name)
        if t is None:
            t = self._types[name] = N.lib().dg_segment_column_type(self.handle, name.encode())
        return t

    def device_bytes(self) -> int:
        return int(N.lib().dg_segment_device_bytes(self.handle))

    def cardinality(self, dim: str) -> int:
        return int(N.lib().dg_segment_dim_cardinality(self.handle, dim.encode()))

    def dictionary(self, dim: str) -> List[Optional[str]]:
        """Sorted dictionary of a string dimension; null (empty) values are None."""
        if dim not in self._dicts:
            if self.column_type(dim) != N.COL_STRING:
                self._dicts[dim] = [None]
            else:
                card = self.cardinality(dim)
                offs = np.zeros(card + 1, dtype=np.int64)
                total = ctypes.c_int64()
                N.check(N.lib().dg_segment_dim_dictionary(self.handle, dim.encode(), None, None, ctypes.byref(total)))
                buf = ctypes.create_string_buffer(max(total.value, 1))
                N.check(N.lib().dg_segment_dim_dictionary(self.handle, dim.encode(), offs.ctypes.data, buf,
                                                          ctypes.byref(total)))
                raw = buf.raw
                vals: List[Optional[str]] = []
                for i in range(card):
                    a, b = int(offs[i]), int(offs[i + 1])
                    vals.append(raw[a:b].decode("utf-8") if b > a else None)
                self._dicts[dim] = vals
        return self._dicts[dim]

    def dim_order(self, dim: str, ordering: str, inverted: bool = False) -> Optional[O.DictionaryOrder]:
        """The dictionary's order under a topN comparator, handed to the engine once
        (dg_segment_set_dim_order); None for a missing dimension (its only value is null)."""
        if self.column_type(dim) != N.COL_STRING:
            return None
        slot = O.order_slot(ordering, inverted)
        key = (dim, slot)
        if key not in self._orders:
            order = O.DictionaryOrder(self.dictionary(dim), ordering, inverted)
            rank = np.ascontiguousarray(order.rank, dtype=np.int32)
            N.check(N.lib().dg_segment_set_dim_order(self.handle, dim.encode(), slot, rank.ctypes.data, len(rank),
                                                     int(order.has_ties)))
            self._orders[key] = order
        return self._orders[key]

    def dim_value(self, dim: str, idx: int) -> Optional[str]:
        """DimensionSelector.lookupName for one id (no full dictionary export)."""
        d = self._dicts.get(dim)
        if d is not None:
            return d[idx]
        seen = self._values.get(dim)
        if seen is not None and idx in seen:
            return seen[idx]
        if self.column_type(dim) != N.COL_STRING:
            return None
        p, n = ctypes.c_void_p(), ctypes.c_int32()
        N.check(N.lib().dg_segment_dim_value(self.handle, dim.encode(), int(idx), ctypes.byref(p), ctypes.byref(n)))
        v = ctypes.string_at(p.value, n.value).decode("utf-8") if n.value > 0 else None
        if seen is None:
            seen = self._values[dim] = {}
        if len(seen) < 65536:  # the ids a query's results name again (topN heads), bounded
            seen[int(idx)] = v
        return v

    def filter_bitmap(self, flt, query_module) -> Tuple[np.ndarray, int]:
        """Filter.getBitmapResult as a dense row bitset (uint32 words) + cardinality."""
        fp = N.FilterProgram(flt, query_module, [self])
        words = np.zeros((self.num_rows + 31) // 32, dtype=np.uint32)
        cnt = ctypes.c_int64()
        arr = ctypes.cast(fp.array, ctypes.POINTER(N.dg_filter)) if fp.array is not None else None
        N.check(N.lib().dg_filter_bitmap(self.handle, arr, len(fp.nodes), words.ctypes.data, ctypes.byref(cnt)))
        return words, cnt.value

    def close(self):
        if self.handle:
            N.lib().dg_segment_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
