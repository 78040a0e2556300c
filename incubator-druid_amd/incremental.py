"""In-memory (realtime) segments: an IncrementalIndex's rows queried on the GPU.

The reference ingests rows into an ``IncrementalIndex`` (segment/incremental/IncrementalIndex.java,
OnheapIncrementalIndex.java) and queries it through ``IncrementalIndexStorageAdapter`` before the
rows are persisted. This module keeps the index's host-side bookkeeping — what ingestion does per row —
and hands the rows to the engine with ``dg_segment_from_rows``:

* dimension values are encoded per dimension in insertion order (``DimensionDictionary.add``,
  StringDimensionIndexer.java), "" and missing values are null (``NullHandling.emptyToNullIfNeeded``);
  a list value is a multi-value row (sorted values, an empty list has no values);
* with rollup, rows with equal (truncated timestamp, dimension values) fold into one fact whose metric
  columns combine the ingested values (``IncrementalIndex.addToFacts``; the ingestion aggregators
  longSum / doubleSum / floatSum / count / min / max). The timestamp is truncated by the index's
  queryGranularity (``IncrementalIndex.toIncrementalIndexRow``: ``gran.bucketStart``);
* facts iterate in ``IncrementalIndexRowComparator`` order (IncrementalIndex.java:1144-1190): time,
  then each dimension's value (``compareUnsortedEncodedKeyComponents``: String.compareTo, nulls
  first); without rollup equal keys keep their insertion order.

``to_segment()`` uploads the facts as a device segment (dictionaries re-sorted on the device side);
``to_spec()`` gives the same rows in the persisted layout (``IndexMergerV9``: sorted dictionaries), so
a test can check that querying the in-memory index and its persisted segment agree — the reference's
own test strategy (QueryRunnerTestHelper.makeQueryRunners runs every query over an incremental index
and over its persisted, memory-mapped form).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from . import query as Q
from .segment import GpuContext, GpuSegment

# ingestion aggregators: (output column type, combine)
_KINDS = {
    "count": ("long", None),
    "longSum": ("long", lambda a, b: a + b),
    "doubleSum": ("double", lambda a, b: a + b),
    "floatSum": ("float", lambda a, b: float(np.float32(np.float32(a) + np.float32(b)))),
    "longMin": ("long", min),
    "longMax": ("long", max),
    "doubleMin": ("double", lambda a, b: _java_min(a, b)),
    "doubleMax": ("double", lambda a, b: _java_max(a, b)),
    "floatMin": ("float", lambda a, b: _java_min(a, b)),
    "floatMax": ("float", lambda a, b: _java_max(a, b)),
}


def _java_min(a: float, b: float) -> float:
    """Math.min: NaN wins, -0.0 < 0.0."""
    if a != a or b != b:
        return float("nan")
    if a == b == 0.0:
        return a if np.signbit(a) else b
    return a if a < b else b


def _java_max(a: float, b: float) -> float:
    if a != a or b != b:
        return float("nan")
    if a == b == 0.0:
        return b if np.signbit(a) else a
    return a if a > b else b


def _java_key(s: Optional[str]):
    return (0, b"") if s is None else (1, s.encode("utf-16-be", "surrogatepass"))


class IncrementalIndex:
    """Rows of one realtime index (OnheapIncrementalIndex): explicit dimensions (DimensionsSpec),
    ingestion metrics as (name, kind, input field) with kind in longSum / doubleSum / floatSum / count /
    longMin / longMax / doubleMin / doubleMax / floatMin / floatMax."""

    def __init__(self, dimensions: Sequence[str], metrics: Sequence[Tuple[str, str, Optional[str]]],
                 query_granularity="none", rollup: bool = True, interval: Optional[Tuple[int, int]] = None):
        for _, kind, _f in metrics:
            if kind not in _KINDS:
                raise ValueError(f"unsupported ingestion aggregator {kind!r}")
        self.dimensions = list(dimensions)
        self.metrics = list(metrics)
        self.gran = Q.Granularity.of(query_granularity) if query_granularity != "none" else None
        self.rollup = rollup
        self.interval = interval
        self._dicts: List[Dict[Optional[str], int]] = [dict() for _ in self.dimensions]
        self._values: List[List[Optional[str]]] = [[] for _ in self.dimensions]
        self._facts: Dict[tuple, list] = {}
        self._multi = [False] * len(self.dimensions)  # hasMultipleValues
        self._order = 0

    def _id(self, d: int, v) -> int:
        v = None if v is None or v == "" else str(v)
        i = self._dicts[d].get(v)
        if i is None:
            i = self._dicts[d][v] = len(self._values[d])
            self._values[d].append(v)
        return i

    def _encode(self, d: int, v) -> tuple:
        """StringDimensionIndexer.processRowValsToUnsortedEncodedKeyComponent (:247-300): null / a
        scalar -> one id; a list: empty -> no ids (null still enters the dictionary), else its values
        sorted (MultiValueHandling SORTED_ARRAY, naturalNullsFirst) -> their ids."""
        if isinstance(v, (list, tuple)):
            vals = [None if x is None or x == "" else str(x) for x in v]
            if not vals:
                self._id(d, None)
                return ()
            if len(vals) > 1:
                self._multi[d] = True
                vals.sort(key=_java_key)
            return tuple(self._id(d, x) for x in vals)
        return (self._id(d, v),)

    def add(self, timestamp: int, event: Dict) -> int:
        """IncrementalIndex.add: returns the number of facts."""
        t = int(timestamp) if self.gran is None else self.gran.bucket_start(int(timestamp))
        key = (t, tuple(self._encode(d, event.get(name)) for d, name in enumerate(self.dimensions)))
        if not self.rollup:
            key = key + (self._order,)
        self._order += 1
        vals = []
        for _, kind, field in self.metrics:
            typ, _ = _KINDS[kind]
            x = 1 if kind == "count" else event.get(field, 0)
            x = int(x) if typ == "long" else (float(np.float32(x)) if typ == "float" else float(x))
            vals.append(x)
        acc = self._facts.get(key)
        if acc is None:
            self._facts[key] = vals
        else:
            for i, (_, kind, _f) in enumerate(self.metrics):
                acc[i] = acc[i] + 1 if kind == "count" else _KINDS[kind][1](acc[i], vals[i])
        return len(self._facts)

    def __len__(self):
        return len(self._facts)

    def _ordered(self):
        # IncrementalIndexRowComparator: time, then per dimension compareUnsortedEncodedKeyComponents
        # (the row's value count first, then its values, String.compareTo with nulls first)
        def key(k):
            dims = tuple((len(ids), tuple(_java_key(self._values[d][i]) for i in ids)) for d, ids in enumerate(k[1]))
            return (k[0], dims) + ((k[2],) if len(k) > 2 else ())
        return sorted(self._facts.items(), key=lambda kv: key(kv[0]))

    def _row_ids(self, d: int, ids: tuple):
        """A single-valued dimension stores one id per row (an empty list as null)."""
        if self._multi[d]:
            return ids
        return ids[0] if ids else self._dicts[d][None]

    def _columns(self):
        facts = self._ordered()
        ts = np.array([k[0] for k, _ in facts], dtype=np.int64)
        ids = []
        for d in range(len(self.dimensions)):
            rows = [self._row_ids(d, k[1][d]) for k, _ in facts]
            if self._multi[d]:
                offs = np.zeros(len(rows) + 1, np.int32)
                offs[1:] = np.cumsum([len(r) for r in rows])
                flat = np.array([i for r in rows for i in r], dtype=np.int32)
                ids.append((flat, offs))
            else:
                ids.append(np.array(rows, dtype=np.int32))
        mets = []
        for i, (name, kind, _f) in enumerate(self.metrics):
            typ = _KINDS[kind][0]
            dt = {"long": np.int64, "float": np.float32, "double": np.float64}[typ]
            mets.append((name, typ, np.array([v[i] for _, v in facts], dtype=dt)))
        return ts, ids, mets

    def _interval(self, ts: np.ndarray) -> Tuple[int, int]:
        if self.interval is not None:
            return self.interval
        return (int(ts[0]), int(ts[-1]) + 1) if len(ts) else (0, 0)

    def to_segment(self, device: int = 0, context: Optional[GpuContext] = None) -> GpuSegment:
        """IncrementalIndexStorageAdapter over the current facts, resident on the GPU."""
        ts, ids, mets = self._columns()
        keep = []
        cols = []
        for d, name in enumerate(self.dimensions):
            vals = self._values[d]
            arr = (ctypes.c_char_p * max(len(vals), 1))(*[None if v is None else v.encode() for v in vals])
            flat, offs = ids[d] if self._multi[d] else (ids[d], None)
            flat = flat if len(flat) else np.zeros(1, np.int32)
            keep += [arr, flat, offs]
            cols.append(N.dg_row_column(name.encode(), 4, len(vals), ctypes.cast(arr, ctypes.c_void_p),
                                        flat.ctypes.data, None, None if offs is None else offs.ctypes.data))
        for name, typ, v in mets:
            keep.append(v)
            cols.append(N.dg_row_column(name.encode(), {"long": 1, "float": 2, "double": 3}[typ], 0, None, None,
                                        v.ctypes.data, None))
        carr = (N.dg_row_column * max(len(cols), 1))(*cols)
        iv = self._interval(ts)
        ctx = context or GpuContext.get(device)
        h = ctypes.c_void_p()
        N.check(N.lib().dg_segment_from_rows(ctx.handle, len(ts), ts.ctypes.data, iv[0], iv[1],
                                             ctypes.cast(carr, ctypes.c_void_p), len(cols), ctypes.byref(h)))
        return GpuSegment.from_handle(h, ctx, f"incremental:{id(self)}")

    def to_spec(self):
        """The same rows as the persisted segment IndexMergerV9 writes (sorted dictionaries)."""
        from .writer import SegmentSpec
        ts, ids, mets = self._columns()
        dims = {}
        for d, name in enumerate(self.dimensions):
            vals = self._values[d]
            order = sorted(range(len(vals)), key=lambda i: _java_key(vals[i]))
            remap = np.zeros(max(len(vals), 1), np.int32)
            remap[order] = np.arange(len(order), dtype=np.int32)
            dct = ["" if vals[i] is None else vals[i] for i in order]
            if self._multi[d]:  # IndexMergerV9: the multi-value column format, values in row order
                flat, offs = ids[d]
                dims[name] = (dct, [remap[flat[offs[r]:offs[r + 1]]] for r in range(len(offs) - 1)])
            else:
                dims[name] = (dct, remap[ids[d]])
        return SegmentSpec(timestamps=ts, dims=dims, metrics={n: (t, v) for n, t, v in mets},
                           interval=self._interval(ts))
