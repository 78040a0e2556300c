"""Query runners: the QueryRunnerFactory / QueryToolChest surface over the GPU engine.

Mirrors the reference's per-segment runner + merge structure:

* ``TimeseriesQueryRunnerFactory`` (query/timeseries/TimeseriesQueryRunnerFactory.java:66-105):
  ``createRunner(segment)`` -> per-segment results (one Result per granularity bucket,
  TimeseriesQueryEngine.java:57-111); ``mergeRunners`` -> results combined per bucket with
  ``AggregatorFactory.combine`` (TimeseriesBinaryFn.java:55-81).
* ``TopNQueryRunnerFactory`` (query/topn/TopNQueryRunnerFactory.java:61-90): per-segment top
  ``max(threshold, minTopNThreshold)`` (TopNQueryQueryToolChest.java:553-561) from the GPU, merged
  pairwise by TopNBinaryFn (TopNBinaryFn.java:75-135) with the query threshold, then truncated.
* ``GroupByQueryRunnerFactory`` (GroupByStrategyV2.process/mergeRunners, GroupByStrategyV2.java:453-477):
  per-segment grouping on the GPU, merged by dimension values (GroupByMergingQueryRunnerV2.java:170-290)
  and ordered by timestamp then dimension values.

Segments that share a device are executed as ONE batched native call (all their rows in one
launch sequence); results are still kept per segment and merged exactly like the reference merges
per-segment runners. Cross-device / cross-rank merging is in distributed.py.
"""
from __future__ import annotations

import ctypes
import time
import dataclasses
import heapq
import math
from collections import OrderedDict, defaultdict
from decimal import Decimal
from fractions import Fraction
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from . import ordering as O
from . import query as Q
from .segment import GpuSegment


# ----------------------------------------------------------------------------------------------
# slot decoding
# ----------------------------------------------------------------------------------------------
def _decode_slots(aggs: Sequence[Q.AggregatorFactory], slots: np.ndarray) -> List[np.ndarray]:
    """[n, naggs] uint64 ABI slots -> one typed column per aggregator."""
    out = []
    for a, col in zip(aggs, slots.T):  # (strided views of the slot rows; floats are narrowed)
        if a.output_type == "long":
            out.append(col.view(np.int64))
        elif a.output_type == "double":
            out.append(col.view(np.float64))
        else:
            out.append((col & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32))
    return out


def _py(v, out_type):
    return int(v) if out_type == "long" else float(v)


def _group_by_device(segments: Sequence[GpuSegment]) -> "OrderedDict[int, List[int]]":
    g: "OrderedDict[int, List[int]]" = OrderedDict()
    for i, s in enumerate(segments):
        g.setdefault(id(s.context), []).append(i)
    return g


def _handles(segs: Sequence[GpuSegment]):
    arr = (ctypes.c_void_p * len(segs))(*[s.handle.value for s in segs])
    return arr


class RunStats:
    """Per-call QueryMetrics counters accumulated over native calls."""

    def __init__(self):
        self.calls: List[Dict] = []

    def add(self, m: N.dg_metrics, span=None):
        d = m.as_dict()
        if span is not None:  # host wall clock (time.perf_counter) at the call's start and end
            d["t_start"], d["t_end"] = span
        self.calls.append(d)

    def total(self, key):
        return sum(c[key] for c in self.calls)


# ----------------------------------------------------------------------------------------------
# timeseries
# ----------------------------------------------------------------------------------------------
def timeseries_per_segment(segments: Sequence[GpuSegment], query: Q.TimeseriesQuery,
                           stats: Optional[RunStats] = None,
                           cancel: Optional[ctypes.c_int32] = None) -> List[List[Q.Result]]:
    split = segment_queries(query, segments)
    if split is not None:  # every segment on its own calendar chain
        return [timeseries_per_segment([s], q, stats, cancel)[0] if q is not None else []
                for s, q in zip(segments, split)]
    out: List[List[Q.Result]] = [[] for _ in segments]
    na = len(query.aggregations)
    for _, idx in _group_by_device(segments).items():
        segs = [segments[i] for i in idx]
        cap = _bucket_cap(segs, query)
        scan, keep = N.make_scan(query, Q, segments=segs, cancel=cancel)
        n = len(segs)
        nb = np.zeros(n, dtype=np.int32)
        times = np.zeros(n * cap, dtype=np.int64)
        rows = np.zeros(n * cap, dtype=np.int64)
        vals = np.zeros(n * cap * max(na, 1), dtype=np.uint64)
        m = N.dg_metrics()
        N.check(N.lib().dg_timeseries_run(_handles(segs), n, ctypes.byref(scan), cap, nb.ctypes.data,
                                          times.ctypes.data, rows.ctypes.data, vals.ctypes.data, ctypes.byref(m)))
        if stats is not None:
            stats.add(m)
        for k, i in enumerate(idx):
            res = []
            cols = _decode_slots(query.aggregations, vals.reshape(-1, max(na, 1))[k * cap:k * cap + nb[k], :na])
            for b in range(nb[k]):
                if query.skip_empty_buckets and rows[k * cap + b] == 0:
                    continue
                res.append(Q.Result(int(times[k * cap + b]),
                                    {a.name: _py(c[b], a.output_type) for a, c in zip(query.aggregations, cols)}))
            out[i] = res
    return out


def run_timeseries(segments: Sequence[GpuSegment], query: Q.TimeseriesQuery,
                   stats: Optional[RunStats] = None) -> List[Q.Result]:
    """QueryRunnerFactory.mergeRunners over segments on any devices: one dg_timeseries_run per device,
    then every segment's bucket list (in segment order) folded natively by dg_timeseries_merge
    (TimeseriesBinaryFn, ResultMergeQueryRunner order: time, then runner)."""
    na = len(query.aggregations)
    groups = list(_group_by_device(segments).items())
    caps = {dev: _bucket_cap([segments[i] for i in idx], query) for dev, idx in groups}
    cap = max(caps.values()) if caps else 1
    n_all = len(segments)
    nb = np.zeros(max(n_all, 1), dtype=np.int32)
    times = np.zeros(max(n_all, 1) * cap, dtype=np.int64)
    rows = np.zeros(max(n_all, 1) * cap, dtype=np.int64)
    vals = np.zeros(max(n_all, 1) * cap * max(na, 1), dtype=np.uint64)
    scan = keep = None
    for dev, idx in groups:
        segs = [segments[i] for i in idx]
        c = caps[dev]
        scan, keep = N.make_scan(query, Q, segments=segs)
        n = len(segs)
        d_nb = np.zeros(n, dtype=np.int32)
        d_t = np.zeros(n * c, dtype=np.int64)
        d_r = np.zeros(n * c, dtype=np.int64)
        d_v = np.zeros(n * c * max(na, 1), dtype=np.uint64)
        m = N.dg_metrics()
        N.check(N.lib().dg_timeseries_run(_handles(segs), n, ctypes.byref(scan), c, d_nb.ctypes.data, d_t.ctypes.data,
                                          d_r.ctypes.data, d_v.ctypes.data, ctypes.byref(m)))
        if stats is not None:
            stats.add(m)
        for k, i in enumerate(idx):  # into the segment's slot of the call-wide lists
            nb[i] = d_nb[k]
            times[i * cap:i * cap + c] = d_t[k * c:(k + 1) * c]
            rows[i * cap:i * cap + c] = d_r[k * c:(k + 1) * c]
            vals[i * cap * na:(i * cap + c) * na] = d_v[k * c * na:(k + 1) * c * na]
    if scan is None:
        scan, keep = N.make_scan(query, Q, filters=False)
    g = query.granularity
    if g.is_calendar:  # TimeseriesBinaryFn keys a result by gran.bucketStart(its timestamp)
        starts = {}
        for i in range(n_all):
            for k in range(int(nb[i])):
                t = int(times[i * cap + k])
                if t not in starts:
                    starts[t] = g.bucket_start(t)
                times[i * cap + k] = starts[t]
    out_cap = max(n_all, 1) * cap
    on = ctypes.c_int32()
    o_t = np.zeros(out_cap, dtype=np.int64)
    o_v = np.zeros(out_cap * max(na, 1), dtype=np.uint64)
    N.check(N.lib().dg_timeseries_merge(ctypes.byref(scan), n_all, nb.ctypes.data, cap, times.ctypes.data,
                                        rows.ctypes.data, vals.ctypes.data, int(query.skip_empty_buckets), out_cap,
                                        ctypes.byref(on), o_t.ctypes.data, None, o_v.ctypes.data))
    m = on.value
    cols = _decode_slots(query.aggregations, o_v.reshape(-1, max(na, 1))[:m, :na])
    return [Q.Result(int(o_t[b]), {a.name: _py(c[b], a.output_type) for a, c in zip(query.aggregations, cols)})
            for b in range(m)]


def _bucket_cap(segs, query) -> int:
    g = query.granularity
    if g.is_all:
        return 1
    cap = 1
    qs, qe = query.interval
    for s in segs:
        lo = max(qs, s.min_time)
        hi = min(qe, g.bucket_end(s.max_time))
        if hi > lo:
            if g.is_calendar:  # buckets of the segment's actual interval on the query's bucket list
                cap = max(cap, len(g.iterable((lo, hi))))
            else:
                cap = max(cap, (hi - g.bucket_start(lo) + g.period_ms - 1) // g.period_ms)
    return int(cap)


def merge_timeseries(query: Q.TimeseriesQuery, per_segment: List[List[Q.Result]]) -> List[Q.Result]:
    """ResultMergeQueryRunner + TimeseriesBinaryFn: combine results of the same bucket."""
    gran = query.granularity
    merged: Dict[int, Q.Result] = {}
    flat = sorted(((r.timestamp, si, k, r) for si, rs in enumerate(per_segment) for k, r in enumerate(rs)),
                  key=lambda x: (x[0], x[1], x[2]))
    for ts, _, _, r in flat:
        key = 0 if gran.is_all else gran.bucket_start(ts)
        if key not in merged:
            merged[key] = Q.Result(r.timestamp if gran.is_all else key, dict(r.value))
        else:
            acc = merged[key].value
            for a in query.aggregations:
                acc[a.name] = a.combine(acc[a.name], r.value[a.name])
    out = [merged[k] for k in sorted(merged)]
    if query.descending:
        out.reverse()
    return out


# ----------------------------------------------------------------------------------------------
# topN
# ----------------------------------------------------------------------------------------------
def _java_key(s: Optional[str]):
    return (0, b"") if s is None else (1, s.encode("utf-16-be", "surrogatepass"))


class _HeapItem:
    __slots__ = ("mk", "dk", "entry")

    def __init__(self, mk, dk, entry):
        self.mk, self.dk, self.entry = mk, dk, entry

    def __lt__(self, o):
        return (self.mk, self.dk) < (o.mk, o.dk)


class TopNResultBuilder:
    """TopNNumericResultBuilder (TopNNumericResultBuilder.java:94-235): bounded priority queue,
    add only when below threshold or strictly better than the current minimum metric."""

    def __init__(self, query: Q.TopNQuery, threshold: int):
        spec = query.metric
        agg = next(a for a in query.aggregations if a.name == spec.metric)
        self.metric = spec.metric
        self.dim = query.dimension
        self.inverted = spec.type == "inverted"
        self.agg = agg
        self.threshold = threshold
        self.heap: List[_HeapItem] = []

    def _mk(self, v):
        k = self.agg.compare_key(v)
        return _Rev(k) if self.inverted else k

    def add(self, entry: Dict):
        mk = self._mk(entry[self.metric])
        if len(self.heap) < self.threshold or self.heap[0].mk < mk:
            heapq.heappush(self.heap, _HeapItem(mk, _java_key(entry[self.dim]), entry))
        if len(self.heap) > self.threshold:
            heapq.heappop(self.heap)

    def build(self) -> List[Dict]:
        items = sorted(self.heap, key=lambda h: (_Rev(h.mk), h.dk))
        return [h.entry for h in items]


class JavaPriorityQueue:
    """java.util.PriorityQueue with a comparator (offer = siftUp, poll = siftDown, toArray = the
    heap array): which of several comparator-equal entries a poll removes, and the order a stable
    sort leaves them in, follow from this exact layout."""

    def __init__(self, cmp):
        self.cmp = cmp
        self.q: List = []

    def __len__(self):
        return len(self.q)

    def offer(self, x):
        q, cmp = self.q, self.cmp
        k = len(q)
        q.append(x)
        while k > 0:
            parent = (k - 1) >> 1
            if cmp(x, q[parent]) >= 0:
                break
            q[k] = q[parent]
            k = parent
        q[k] = x

    def poll(self):
        q, cmp = self.q, self.cmp
        top = q[0]
        x = q.pop()
        n = len(q)
        if n:
            k = 0
            while k < (n >> 1):
                child = 2 * k + 1
                if child + 1 < n and cmp(q[child], q[child + 1]) > 0:
                    child += 1
                if cmp(x, q[child]) <= 0:
                    break
                q[k] = q[child]
                k = child
            q[k] = x
        return top


def _memo_key(key):
    """key(v) computed once per value (a comparator calls it on both sides of every comparison)."""
    memo: Dict = {}

    def k(v):
        r = memo.get(v, memo)
        if r is memo:
            r = memo[v] = key(v)
        return r
    return k


def _key_cmp(key):
    def cmp(a, b):
        ka, kb = key(a), key(b)
        return (ka > kb) - (ka < kb)
    return cmp


class LexicographicResultBuilder:
    """TopNLexicographicResultBuilder (query/topn/TopNLexicographicResultBuilder.java:40-176) with
    the topN comparator given as a sort key (ordering.sort_key): shouldAdd takes every non-null
    value once the queue is full (the head's topN metric value it compares against is never set),
    values must come after previousStop; the queue's head is the largest value, polled past the
    threshold; build() sorts the queue's array by the comparator, stably."""

    def __init__(self, query: Q.TopNQuery, threshold: int):
        spec = query.metric
        self.dim = query.dimension
        self.key = _memo_key(O.sort_key(spec.ordering, spec.inverted))
        self.cmp = _key_cmp(self.key)
        self.threshold = threshold
        self.stop = spec.previous_stop
        self.pq = JavaPriorityQueue(lambda a, b: self.cmp(b[self.dim], a[self.dim]))

    def add(self, entry: Dict):
        v = entry[self.dim]
        if len(self.pq) >= self.threshold and v is None:
            return
        if self.stop is not None and self.cmp(v, self.stop) <= 0:
            return
        self.pq.offer(entry)
        if len(self.pq) > self.threshold:
            self.pq.poll()

    def build(self) -> List[Dict]:
        return sorted(self.pq.q, key=lambda e: self.key(e[self.dim]))


def _result_builder(query: Q.TopNQuery, threshold: int):
    if query.metric.type == "dimension":
        return LexicographicResultBuilder(query, threshold)
    return TopNResultBuilder(query, threshold)


class _Rev:
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def __lt__(self, o):
        return o.v < self.v

    def __eq__(self, o):
        return self.v == o.v


class TopNRaw:
    """dg_topn_run output for segments of one device: list L = i * bcap + b (segment i, cursor b; bcap = 1
    for ALL granularity) has `cnt[L]` entries (-1 = no cursor), entry j at L * K + j of `ids`
    (segment-local dictionary ids) and `vals` (n_aggs slots); `ts[L]` is the list's result timestamp."""

    def __init__(self, segments, cnt, ids, vals, K, ts, bcap=1):
        self.segments, self.cnt, self.ids, self.vals, self.K, self.ts = segments, cnt, ids, vals, K, ts
        self.bcap = bcap


def _topn_struct(query: Q.TopNQuery, threshold: int, segments: Optional[Sequence[GpuSegment]] = None):
    """dg_topn for a numeric / inverted metric, or a dimension ordering (then the segments'
    dictionary orders are registered and their previousStop cuts computed). Returns the struct and
    the buffers it points into."""
    t = N.dg_topn()
    dim = query.dimension.encode()
    t.dimension = dim
    t.threshold = threshold
    spec = query.metric
    keep = [dim]
    if spec.type == "dimension":
        t.metric_agg, t.inverted = 0, 0
        t.dim_order = O.order_slot(spec.ordering, spec.inverted)
        if spec.previous_stop is not None:
            stop = spec.previous_stop.encode()
            t.previous_stop = stop
            keep.append(stop)
        if segments is not None:
            mins = np.zeros(len(segments), dtype=np.int32)
            for i, seg in enumerate(segments):
                order = seg.dim_order(query.dimension, spec.ordering, spec.inverted)
                if order is not None:
                    mins[i] = order.min_rank(spec.previous_stop)
                else:  # missing dimension: its one value is null, never after a previousStop
                    mins[i] = 0 if spec.previous_stop is None else 1
            t.min_rank = mins.ctypes.data
            keep.append(mins)
    else:
        t.metric_agg = [a.name for a in query.aggregations].index(spec.metric)
        t.inverted = int(spec.type == "inverted")
        t.dim_order = -1
    return t, keep


def _check_topn(query: Q.TopNQuery):
    pass


def topn_raw(segments: Sequence[GpuSegment], query: Q.TopNQuery, stats: Optional[RunStats] = None) -> TopNRaw:
    """One batched dg_topn_run over segments that share a device (PooledTopNAlgorithm +
    TopNNumericResultBuilder per segment, threshold max(threshold, minTopNThreshold))."""
    _check_topn(query)
    if len(_group_by_device(segments)) != 1:
        raise ValueError("topn_raw: segments must share one device")
    na = len(query.aggregations)
    K = query.segment_threshold
    scan, keep = N.make_scan(query, Q, segments=segments)
    t, keep_t = _topn_struct(query, K, segments)
    n = len(segments)
    bcap = _bucket_cap(segments, query)
    cnt = np.zeros(n * bcap, dtype=np.int32)
    ids = np.zeros(n * bcap * K, dtype=np.int32)
    vals = np.zeros(n * bcap * K * max(na, 1), dtype=np.uint64)
    bt = np.zeros(n * bcap, dtype=np.int64)
    t.bucket_cap = bcap
    t.out_bucket_time = bt.ctypes.data
    m = N.dg_metrics()
    N.check(N.lib().dg_topn_run(_handles(segments), n, ctypes.byref(scan), ctypes.byref(t), cnt.ctypes.data,
                                ids.ctypes.data, vals.ctypes.data, ctypes.byref(m)))
    if stats is not None:
        stats.add(m)
    if query.granularity.is_all:  # the cursor's time: start of the segment's part of the interval
        ts = np.array([max(query.interval[0], s.min_time) for s in segments], dtype=np.int64)
    else:
        ts = bt
    return TopNRaw(list(segments), cnt, ids, vals, K, ts, bcap)


def topn_merge_raw(query: Q.TopNQuery, cnt: np.ndarray, keys: np.ndarray, vals: np.ndarray, K: int,
                   ts: np.ndarray, handles=None):
    """dg_topn_merge over lists ordered by (timestamp, index) (TopNQueryQueryToolChest merge order).
    Returns (timestamp, list index, keys, value slots) of the merged entries, or None when no list
    has a cursor. handles: per-list segment handles (segment mode) or None (global ids)."""
    na = len(query.aggregations)
    live = [i for i in range(len(cnt)) if cnt[i] >= 0]
    if not live:
        return None
    order = np.array(sorted(live, key=lambda i: (int(ts[i]), i)), dtype=np.int64)
    n = len(order)
    if n == len(cnt) and not np.any(order != np.arange(n)):  # every list, already in merge order
        o_cnt = np.ascontiguousarray(cnt, dtype=np.int32)
        o_keys = np.ascontiguousarray(keys, dtype=np.int64)
        o_vals = np.ascontiguousarray(vals)
    else:
        o_cnt = np.ascontiguousarray(cnt[order].astype(np.int32))
        o_keys = np.ascontiguousarray(keys.reshape(-1, K)[order].astype(np.int64))
        o_vals = np.ascontiguousarray(vals.reshape(-1, K, max(na, 1))[order])
    lists = N.dg_topn_lists()
    lists.n_lists = n
    lists.list_n = o_cnt.ctypes.data
    lists.stride = K
    lists.keys = o_keys.ctypes.data
    lists.values = o_vals.ctypes.data
    scan, keep = N.make_scan(query, Q, filters=False)  # the fold needs the aggregators only
    t, dim = _topn_struct(query, query.threshold)
    out_n = ctypes.c_int32()
    T = query.threshold
    out_list = np.zeros(T, dtype=np.int32)
    out_keys = np.zeros(T, dtype=np.int64)
    out_vals = np.zeros(T * max(na, 1), dtype=np.uint64)
    hs = None
    if handles is not None:
        hs = (ctypes.c_void_p * n)(*[handles[i] for i in order])
    N.check(N.lib().dg_topn_merge(hs, ctypes.byref(scan), ctypes.byref(t), ctypes.byref(lists), ctypes.byref(out_n),
                                  out_list.ctypes.data, out_keys.ctypes.data, out_vals.ctypes.data))
    k = out_n.value
    if k < 0:
        return None
    return int(ts[order[0]]), order[out_list[:k]], out_keys[:k], out_vals[:k * na].reshape(k, na) if na else None


def _topn_entries(query: Q.TopNQuery, values: List[Optional[str]], slots) -> List[Dict]:
    # (tolist: Python ints / floats per column at once, as _py of each element would give)
    cols = [c.tolist() for c in _decode_slots(query.aggregations, slots)] if len(values) and query.aggregations else []
    names = [a.name for a in query.aggregations]
    dim = query.dimension
    out = []
    for j, v in enumerate(values):
        e = {dim: v}
        for name, col in zip(names, cols):
            e[name] = col[j]
        out.append(e)
    return out


def merge_dimension_lists(query: Q.TopNQuery, lists: Sequence[Tuple[int, int, "callable", np.ndarray]],
                          tie_free: bool) -> List[Q.Result]:
    """TopNBinaryFn fold of dimension-ordered per-segment lists, given in merge order as
    (timestamp, length, value_of(j), [length, n_aggs] slots), with the builder's literal queue
    (LexicographicResultBuilder). Each list is its segment's values in comparator order. When no
    two values compare equal (`tie_free`: no segment order has ties, and the head entries checked
    here have distinct keys), every value the fold keeps or ranks sits in the first `threshold`
    non-null entries of each list holding it, and the queue sizes the fold sees (which decide
    whether a late null is taken) are the same over those heads: the fold runs over the heads only."""
    if not lists:
        return []
    spec = query.metric
    T = query.threshold

    def head(c, value_of):  # the first T non-null entries (a list's null comes first)
        return min(c, T + (1 if c and value_of(0) is None else 0))

    def fold(limit):
        per = []
        for ts, c, value_of, slots in lists:
            k = c if limit is None else head(c, value_of)
            per.append([Q.Result(ts, _topn_entries(query, [value_of(j) for j in range(k)], slots[:k]))])
        return merge_topn(query, per)

    if not tie_free:
        return fold(None)
    key = O.sort_key(spec.ordering, spec.inverted)
    heads = {value_of(j) for _, c, value_of, _ in lists for j in range(head(c, value_of))}
    keys = sorted(key(v) for v in heads)
    if any(a == b for a, b in zip(keys, keys[1:])):
        return fold(None)
    return fold(T)


def _merge_topn_dimension(query: Q.TopNQuery, segments: Sequence[GpuSegment], raw: TopNRaw) -> List[Q.Result]:
    spec = query.metric
    K, na = raw.K, len(query.aggregations)
    live = sorted((i for i in range(len(segments)) if raw.cnt[i] >= 0), key=lambda i: (int(raw.ts[i]), i))
    orders = [segments[i].dim_order(query.dimension, spec.ordering, spec.inverted) for i in live]
    tie_free = not any(o is not None and o.has_ties for o in orders)
    slots = raw.vals.reshape(-1, max(na, 1))
    lists = []
    for i in live:
        seg, base = segments[i], i * K
        memo: Dict[int, Optional[str]] = {}  # (each entry's value looked up once)

        def value_of(j, seg=seg, base=base, memo=memo):
            v = memo.get(j, memo)
            if v is memo:
                v = memo[j] = seg.dim_value(query.dimension, int(raw.ids[base + j]))
            return v
        lists.append((int(raw.ts[i]), int(raw.cnt[i]), value_of, slots[base:base + int(raw.cnt[i])]))
    return merge_dimension_lists(query, lists, tie_free)


def run_topn(segments: Sequence[GpuSegment], query: Q.TopNQuery, stats: Optional[RunStats] = None) -> List[Q.Result]:
    """Per-segment topN on the GPU + TopNBinaryFn merge in the engine (one device); falls back to the
    Python merge when the segments span devices."""
    _check_topn(query)
    if len(_group_by_device(segments)) != 1 or not query.granularity.is_all:
        return merge_topn(query, topn_per_segment(segments, query, stats))
    if query.metric.type == "dimension":
        return _merge_topn_dimension(query, segments, topn_raw(segments, query, stats))
    raw = topn_raw(segments, query, stats)
    handles = [s.handle for s in segments]
    res = topn_merge_raw(query, raw.cnt, raw.ids, raw.vals, raw.K, raw.ts, handles)
    if res is None:
        return []
    ts, lists, keys, slots = res
    values = [segments[int(l)].dim_value(query.dimension, int(k)) for l, k in zip(lists, keys)]
    return [Q.Result(ts, _topn_entries(query, values, slots))]


def topn_per_segment(segments: Sequence[GpuSegment], query: Q.TopNQuery,
                     stats: Optional[RunStats] = None) -> List[List[Q.Result]]:
    """Per-segment results (what each segment's QueryRunner returns), as Result lists."""
    _check_topn(query)
    split = segment_queries(query, segments)
    if split is not None:  # every segment on its own calendar chain
        return [topn_per_segment([s], q, stats)[0] if q is not None else [] for s, q in zip(segments, split)]
    out: List[List[Q.Result]] = [[] for _ in segments]
    na = len(query.aggregations)
    for _, idx in _group_by_device(segments).items():
        segs = [segments[i] for i in idx]
        raw = topn_raw(segs, query, stats)
        K, bcap = raw.K, raw.bcap
        for k, i in enumerate(idx):
            seg = segs[k]
            res = []
            for b in range(bcap):
                L = k * bcap + b
                if raw.cnt[L] < 0:  # no cursor: the segment does not overlap the interval / bucket
                    continue
                c = int(raw.cnt[L])
                values = [seg.dim_value(query.dimension, int(x)) for x in raw.ids[L * K:L * K + c]]
                slots = raw.vals.reshape(-1, max(na, 1))[L * K:L * K + c, :na]
                res.append(Q.Result(int(raw.ts[L]), _topn_entries(query, values, slots)))
            out[i] = res
    return out


def topn_binary_fn(query: Q.TopNQuery, r1: Optional[Q.Result], r2: Optional[Q.Result]) -> Optional[Q.Result]:
    """TopNBinaryFn.apply (TopNBinaryFn.java:75-135)."""
    if r1 is None:
        return r2
    if r2 is None:
        return r1
    dim = query.dimension
    ret: Dict = {}
    for v in r1.value:
        ret[v[dim]] = v
    for v in r2.value:
        k = v[dim]
        if k in ret:
            a = ret[k]
            c = {dim: k}
            for agg in query.aggregations:
                c[agg.name] = agg.combine(a[agg.name], v[agg.name])
            ret[k] = c
        else:
            ret[k] = v
    bob = _result_builder(query, query.threshold)
    for v in ret.values():
        bob.add(v)
    ts = r1.timestamp if query.granularity.is_all else query.granularity.bucket_start(r1.timestamp)
    return Q.Result(ts, bob.build())


def merge_topn(query: Q.TopNQuery, per_segment: List[List[Q.Result]]) -> List[Q.Result]:
    gran = query.granularity
    flat = sorted(((r.timestamp, si, r) for si, rs in enumerate(per_segment) for r in rs), key=lambda x: (x[0], x[1]))
    merged: Dict[int, Q.Result] = {}
    for ts, _, r in flat:
        key = 0 if gran.is_all else gran.bucket_start(ts)
        merged[key] = topn_binary_fn(query, merged.get(key), r)
    out = [Q.Result(merged[k].timestamp, merged[k].value[:query.threshold]) for k in sorted(merged)]
    # result ordering ResultGranularTimestampComparator.create(gran, descending) (TopNQueryQueryToolChest.java:132;
    # a TopNQuery is never descending, TopNQuery.java:74)
    return out[::-1] if getattr(query, "descending", False) else out


# ----------------------------------------------------------------------------------------------
# groupBy
# ----------------------------------------------------------------------------------------------
class GroupByPartial:
    """Columnar per-segment groupBy output: bucket times, dimension values, aggregate columns.
    Engine partials also carry `codes` (segment-local dictionary ids per dimension) and `dicts` (the
    segments' sorted dictionaries): the merge then works on integer codes, and the value columns are
    only materialised when asked for."""

    def __init__(self, times: np.ndarray, dims: Optional[List[np.ndarray]], aggs: List[np.ndarray],
                 codes: Optional[List[np.ndarray]] = None, dicts: Optional[List[List[Optional[str]]]] = None,
                 merged: bool = False):
        self.times, self._dims, self.aggs = times, dims, aggs
        self.codes, self.dicts = codes, dicts
        self.merged = merged  # already one merged, ordered result (a whole device's engine call)

    @property
    def dims(self) -> List[np.ndarray]:
        if self._dims is None:
            self._dims = [np.array(dd, dtype=object)[c] for c, dd in zip(self.codes, self.dicts)]
        return self._dims

    def __len__(self):
        return len(self.times)


class PinnedPool:
    """Pinned host memory for result delivery (dg_host_alloc), allocated once and reused: the shim's
    direct ByteBuffers (the processing pool allocates its buffers once at startup,
    OffheapBufferGenerator.java:53). Fetches into it go by DMA, no staging copy on the host."""

    def __init__(self, nbytes: int):
        self.ptr = ctypes.c_void_p()
        N.check(N.lib().dg_host_alloc(int(nbytes), ctypes.byref(self.ptr)))
        self.nbytes, self.off = int(nbytes), 0
        self._holder = None  # weak reference to the partial whose arrays are views of this memory

    def _check_free(self, what: str):
        if self._holder is not None and self._holder() is not None:
            raise RuntimeError(f"PinnedPool.{what}: the memory is still in use by a fetched partial (drop it first)")
        self._holder = None

    def hold(self, partial) -> None:
        """Mark the pool as backing `partial` (one fetch at a time): reset() and close() refuse while it
        lives, and the partial keeps the pool alive."""
        import weakref
        self._holder = weakref.ref(partial)
        partial._pool = self

    def reset(self):
        self._check_free("reset")
        self.off = 0

    def take(self, dtype, n: int) -> np.ndarray:
        dt = np.dtype(dtype)
        self.off = (self.off + 63) & ~63
        nb = n * dt.itemsize
        if self.off + nb > self.nbytes:
            raise MemoryError(f"pinned pool of {self.nbytes} bytes: {self.off + nb} needed")
        buf = (ctypes.c_char * nb).from_address(self.ptr.value + self.off)
        self.off += nb
        return np.frombuffer(buf, dtype=dt, count=n)

    def close(self):
        if self.ptr:
            self._check_free("close")
            N.lib().dg_host_free(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass


class GroupByResult:
    """A dg_result: the merged groups of one dg_groupby_run (or of a dg_merge across devices, whose
    ids index the caller's cluster dictionaries), resident in HBM until fetched."""

    def __init__(self, handle: ctypes.c_void_p, query: Q.GroupByQuery,
                 dictionaries: Optional[List[List[Optional[str]]]] = None):
        self.handle, self.query = handle, query
        self.groups = int(N.lib().dg_result_groups(handle))
        self._dicts = dictionaries
        self.time_map: Optional[np.ndarray] = None  # bucket index -> time (a dg_merge over a calendar grid)

    def dictionary(self, d: int) -> List[Optional[str]]:
        if self._dicts is not None:
            return self._dicts[d]
        L = N.lib()
        card = int(L.dg_result_dim_cardinality(self.handle, d))
        offs = np.zeros(card + 1, dtype=np.int64)
        total = ctypes.c_int64()
        N.check(L.dg_result_dim_dictionary(self.handle, d, None, None, ctypes.byref(total)))
        buf = ctypes.create_string_buffer(max(total.value, 1))
        N.check(L.dg_result_dim_dictionary(self.handle, d, offs.ctypes.data, buf, ctypes.byref(total)))
        raw = buf.raw
        return [raw[int(offs[i]):int(offs[i + 1])].decode("utf-8") if offs[i + 1] > offs[i] else None
                for i in range(card)]

    def fetch(self, start: int = 0, count: Optional[int] = None, pool: "Optional[PinnedPool]" = None) -> "GroupByPartial":
        """Groups [start, start + count) to the host. Under ALL granularity no bucket times cross PCIe
        (every group's is the universal timestamp, the query interval's start). pool: pinned host
        memory (dg_host_alloc) the columns land in by DMA; the partial's arrays are views of it."""
        q = self.query
        nd, na = len(q.dimensions), len(q.aggregations)
        count = self.groups - start if count is None else count
        all_gran = q.granularity.is_all and self.time_map is None
        if pool is not None:
            pool.reset()
            t = None if all_gran else pool.take(np.int64, max(count, 1))
            ids = pool.take(np.int32, max(count * nd, 1))
            vals = pool.take(np.uint64, max(count * na, 1))
        else:
            # (np.empty: the library's staged copy is the first touch of these pages, spread over threads)
            t = None if all_gran else np.empty(max(count, 1), dtype=np.int64)
            ids = np.empty(max(count * nd, 1), dtype=np.int32)
            vals = np.empty(max(count * na, 1), dtype=np.uint64)
        if count:
            N.check(N.lib().dg_result_fetch_groups(self.handle, start, count, t.ctypes.data if t is not None else None,
                                                   ids.ctypes.data if nd else None, vals.ctypes.data if na else None))
        if all_gran:  # GroupByStrategyV2.getUniversalTimestamp (:125-138), one value for every group
            t = np.broadcast_to(np.int64(q.interval[0]), (count,))
        if self.time_map is not None:
            t[:count] = self.time_map[t[:count]]
        ids = ids[:count * nd].reshape(count, nd) if nd else np.zeros((count, 0), np.int32)
        codes = [ids[:, d] for d in range(nd)]  # strided views of the [count][ndims] id rows
        aggs = _decode_slots(q.aggregations, vals[:count * na].reshape(count, na)) if na else []
        part = GroupByPartial(t[:count], None, aggs, codes, [self.dictionary(d) for d in range(nd)], merged=True)
        if pool is not None:
            pool.hold(part)
        return part

    def apply_limit_push_down(self) -> bool:
        """LimitedBufferHashGrouper's outcome on the device (dg_result_limit): when the query pushes
        its limit down (GroupByQuery.isApplyLimitPushDown), keep the first `limit` groups in the
        push-down row order (GroupByQuery.getRowOrderingForPushDown :423-528). Every dimension is
        passed as a column: the ORDER BY ones with their comparator and direction, then the others
        ascending under LEXICOGRAPHIC (UTF-8 byte order, which differs from the dictionary's Java
        String order only for values beyond U+D7FF, so the id order is used when none has one)."""
        q = self.query
        if self.groups == 0 or not q.apply_limit_push_down():
            return False
        order = q.order_by_dims()
        cols, keep, seen = [], [], set()
        spec = [(d, c.direction == "descending", c.dimensionOrder) for d, c in zip(order, q.limitSpec.columns)]
        spec += [(d, False, "lexicographic") for d in range(len(q.dimensions)) if d not in order]
        for d, desc, ordering in spec:
            if d in seen:
                continue
            seen.add(d)
            rank = None
            if ordering != "lexicographic" or _beyond_bmp_low(self.dictionary(d)):
                rank = np.ascontiguousarray(O.DictionaryOrder(self.dictionary(d), ordering).rank, dtype=np.int32)
                keep.append(rank)
            cols.append(N.dg_order_column(d, int(desc), rank.ctypes.data if rank is not None else None))
        arr = (N.dg_order_column * len(cols))(*cols)
        lim = N.dg_limit(ctypes.cast(arr, ctypes.c_void_p), len(cols), int(q.limitSpec.limit),
                         int(q._ctx_bool("sortByDimsFirst", False)))
        N.check(N.lib().dg_result_limit(self.handle, ctypes.byref(lim)))
        self.groups = int(N.lib().dg_result_groups(self.handle))
        return True

    def release(self):
        if self.handle:
            N.lib().dg_result_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


def _beyond_bmp_low(values) -> bool:
    """Whether any value holds a character whose UTF-8 order differs from its UTF-16 order."""
    return any(v is not None and any(ord(ch) > 0xD7FF for ch in v) for v in values)


def groupby_run(segments: Sequence[GpuSegment], query: Q.GroupByQuery,
                stats: Optional[RunStats] = None, limit_push_down: bool = False,
                cancel: Optional[ctypes.c_int32] = None) -> GroupByResult:
    """One dg_groupby_run over segments of ONE device: GroupByStrategyV2.mergeRunners over their
    per-segment runners (GroupByMergingQueryRunnerV2.java:170-290), the groups left in HBM. With
    `limit_push_down`, a query that pushes its limit down keeps only its first `limit` groups
    (GroupByResult.apply_limit_push_down); a result meant for the cross-device exchange stays whole.
    cancel: a flag another thread may set (Thread.interrupt): the call then fails DG_ERR_INTERRUPTED;
    the query context's "timeout" (ms) fails it with DG_ERR_TIMEOUT."""
    if len(_group_by_device(segments)) != 1:
        raise ValueError("groupby_run: segments must share one device")
    nd = len(query.dimensions)
    scan, keep = N.make_scan(query, Q, segments=segments, cancel=cancel)
    dims = (ctypes.c_char_p * max(nd, 1))(*[d.encode() for d in query.dimensions])
    g = N.dg_groupby()
    g.dimensions = ctypes.cast(dims, ctypes.POINTER(ctypes.c_char_p))
    g.n_dims = nd
    res = ctypes.c_void_p()
    m = N.dg_metrics()
    t0 = time.perf_counter()
    N.check(N.lib().dg_groupby_run(_handles(segments), len(segments), ctypes.byref(scan), ctypes.byref(g),
                                   ctypes.byref(res), ctypes.byref(m)))
    if stats is not None:
        stats.add(m, (t0, time.perf_counter()))
    out = GroupByResult(res, query)
    if limit_push_down:
        out.apply_limit_push_down()
    return out


def groupby_per_device(segments: Sequence[GpuSegment], query: Q.GroupByQuery,
                       stats: Optional[RunStats] = None) -> List[GroupByPartial]:
    """The merged, ordered groups of every device's segments (one engine call per device)."""
    out = []
    for _, idx in _group_by_device(segments).items():
        r = groupby_run([segments[i] for i in idx], query, stats, limit_push_down=True)
        try:
            out.append(r.fetch())
        finally:
            r.release()
    return out


def _per_device_concurrently(groups, fn, release=None):
    """fn(segment indices of one device) for every device at once, one host thread each, results in
    device order (ChainedExecutionQueryRunner submits every runner to the processing pool; the native
    calls release the GIL, so the devices' kernels are in flight together). Every future is waited
    for; if one fails, `release` frees the results of the others before the first error is raised
    (ChainedExecutionQueryRunner cancels the pending futures the same way, :158-167)."""
    items = list(groups.values())
    if len(items) == 1:
        return [fn(items[0])]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=len(items)) as ex:
        futs = [ex.submit(fn, idx) for idx in items]
        results, err = [], None
        for f in futs:
            try:
                results.append(f.result())
            except BaseException as e:  # noqa: BLE001 (re-raised below, after the cleanup)
                results.append(None)
                err = err or e
    if err is not None:
        if release is not None:
            for r in results:
                if r is not None:
                    release(r)
        raise err
    return results


def groupby_merge_devices(segments: Sequence[GpuSegment], query: Q.GroupByQuery, stats: Optional[RunStats] = None,
                          targets: Optional[Sequence] = None) -> "List[GroupByResult]":
    """mergeRunners over segments of several devices in one process: one dg_groupby_run per device, all
    devices at once, then dg_groupby_merge_devices moves key ranges between the devices itself (peer
    copies) and merges them there, every target concurrently. targets: the contexts owning the key
    ranges (default: every participating device's context, so no device funnels the others' groups);
    returns the per-target results in key order."""
    groups = _group_by_device(segments)
    parts = []
    try:
        def one(idx):
            return groupby_run([segments[i] for i in idx], query, stats)
        parts = _per_device_concurrently(groups, one, release=lambda r: r.release())
        ctxs = [segments[idx[0]].context for idx in groups.values()] if targets is None else list(targets)
        outs = (ctypes.c_void_p * len(ctxs))()
        hp = (ctypes.c_void_p * len(parts))(*[p.handle.value for p in parts])
        ht = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
        m = N.dg_metrics()
        N.check(N.lib().dg_groupby_merge_devices(hp, len(parts), ht, len(ctxs), outs, ctypes.byref(m)))
        if stats is not None:
            stats.add(m)
    finally:
        for p in parts:
            p.release()
    return [GroupByResult(ctypes.c_void_p(o), query) for o in outs]


def groupby_per_segment(segments: Sequence[GpuSegment], query: Q.GroupByQuery,
                        stats: Optional[RunStats] = None) -> List[GroupByPartial]:
    """What each segment's QueryRunner returns (createRunner(segment).run), one engine call each
    (a calendar granularity on the segment's own bucket chain, segment_queries)."""
    split = segment_queries(query, segments) or [query] * len(segments)
    return [groupby_per_device([s], q, stats)[0] for s, q in zip(segments, split) if q is not None]


def merge_groupby_columnar(query: Q.GroupByQuery, partials: Sequence[GroupByPartial]):
    """Merge per-segment partials by (bucket, dimension values); returns sorted columnar arrays."""
    gran = query.granularity
    parts = [p for p in partials if p is not None and len(p)]
    nd = len(query.dimensions)
    if not parts:
        return np.zeros(0, np.int64), [np.zeros(0, object) for _ in range(nd)], [np.zeros(0) for _ in query.aggregations]
    if len(parts) == 1 and parts[0].merged:  # the engine merged and ordered the call's segments already
        return parts[0].times, parts[0].dims, parts[0].aggs
    times = np.concatenate([p.times for p in parts])
    keys_t = times if not gran.is_all else np.zeros(len(times), np.int64)
    if gran.is_calendar and len(times):
        # segments on their own bucket chains (segment_queries): the toolchest's mergeResults orders
        # and combines rows by gran.bucketStart(timestamp) and emits that start
        # (GroupByQuery.getRowOrdering(true), GroupByQuery.java:575-576; GroupByBinaryFnV2.java:78-81)
        u, inv = np.unique(times, return_inverse=True)
        keys_t = np.array([gran.bucket_start(int(x)) for x in u], np.int64)[inv]
    dim_codes = []
    dim_values = []
    coded = all(p.codes is not None for p in parts)
    for d in range(nd):
        if coded:
            # segment dictionaries are sorted (GenericIndexed STRING_STRATEGY): merge them into one
            # global dictionary and remap each segment's ids with one vectorised lookup
            dicts = [p.dicts[d] for p in parts]
            if all(dd is dicts[0] or dd == dicts[0] for dd in dicts[1:]):
                uniq, maps = list(dicts[0]), [None] * len(parts)
            else:
                uniq = sorted(set().union(*map(set, dicts)), key=_java_key)
                index = {v: i for i, v in enumerate(uniq)}
                maps = [np.array([index[v] for v in dd], dtype=np.int64) for dd in dicts]
            dim_codes.append(np.concatenate([p.codes[d].astype(np.int64) if m is None else m[p.codes[d]]
                                             for p, m in zip(parts, maps)]))
            dim_values.append(np.array(uniq, dtype=object))
            continue
        col = np.concatenate([p.dims[d] for p in parts])
        uniq = sorted(set(col.tolist()), key=_java_key)  # global dictionary in Java order, null first
        index = {v: i for i, v in enumerate(uniq)}
        dim_codes.append(np.fromiter((index[v] for v in col), dtype=np.int64, count=len(col)))
        dim_values.append(np.array(uniq, dtype=object))
    order_keys = [keys_t] + dim_codes
    # one composite int64 key (time rank, then each dimension's code) when the ranges fit: a single
    # argsort instead of a multi-key lexsort
    if len(keys_t) and keys_t.min() == keys_t.max():
        t_rank, n_t = np.zeros(len(keys_t), np.int64), 1
    else:
        t_vals, t_rank = np.unique(keys_t, return_inverse=True)
        n_t = len(t_vals)
    radices = [n_t] + [len(v) for v in dim_values]
    if float(np.prod([float(r) for r in radices])) < 2.0 ** 62:
        comp = t_rank.astype(np.int64)
        for c, r in zip(dim_codes, radices[1:]):
            comp = comp * r + c
        order = np.argsort(comp, kind="stable")  # equal keys fold in partial (segment) order
        sc = comp[order]
        change = np.ones(len(order), dtype=bool)
        if len(order) > 1:
            change[1:] = sc[1:] != sc[:-1]
        sk = [k[order] for k in order_keys]
    else:
        order = np.lexsort(tuple(reversed(order_keys)))
        sk = [k[order] for k in order_keys]
        change = np.ones(len(order), dtype=bool)
        if len(order) > 1:
            diff = np.zeros(len(order) - 1, dtype=bool)
            for k in sk:
                diff |= k[1:] != k[:-1]
            change[1:] = diff
    starts = np.nonzero(change)[0]
    out_aggs = []
    for a_i, a in enumerate(query.aggregations):
        col = np.concatenate([p.aggs[a_i] for p in parts])[order]
        out_aggs.append(_reduce(a, col, starts))
    # ALL granularity: every merged row carries the universal timestamp, the query interval's start
    # (GroupByStrategyV2.getUniversalTimestamp, strategy/GroupByStrategyV2.java:125-138)
    out_times = np.full(len(starts), query.interval[0], np.int64) if gran.is_all else sk[0][starts]
    out_dims = [dim_values[d][sk[1 + d][starts]] for d in range(nd)]
    return out_times, out_dims, out_aggs


def _java_minmax_reduce(col: np.ndarray, starts: np.ndarray, is_min: bool) -> np.ndarray:
    """Math.min / Math.max folded over runs (DoubleMinAggregator.combine, java/lang/Math.java): NaN
    wins, and -0.0 < 0.0 — reduced on order-preserving integer keys (the engine's ord_key)."""
    if col.dtype == np.float32:
        bits, sign, udt = col.view(np.uint32).astype(np.uint64), np.uint64(1 << 31), np.uint32
    else:
        bits, sign, udt = col.view(np.uint64), np.uint64(1 << 63), np.uint64
    neg = (bits & sign) != 0
    key = np.where(neg, ~bits & (sign | (sign - np.uint64(1))), bits | sign)
    nan = np.isnan(col)
    red = (np.minimum if is_min else np.maximum).reduceat(key, starts)
    any_nan = np.logical_or.reduceat(nan, starts) if len(col) else np.zeros(0, bool)
    neg_key = (red & sign) == 0
    mask = sign | (sign - np.uint64(1))
    raw = np.where(neg_key, ~red & mask, red & ~sign).astype(udt)
    out = raw.view(col.dtype).copy()
    out[any_nan] = np.nan
    return out


def _reduce(a: Q.AggregatorFactory, col: np.ndarray, starts: np.ndarray) -> np.ndarray:
    k = a.kind
    if k in (0, 1):
        return np.add.reduceat(col.astype(np.int64), starts)
    if k == 4:
        return np.minimum.reduceat(col, starts)
    if k == 5:
        return np.maximum.reduceat(col, starts)
    if k in (2, 3):
        return np.add.reduceat(col, starts)
    return _java_minmax_reduce(col, starts, k in (6, 8))


def merge_groupby(query: Q.GroupByQuery, partials: Sequence[GroupByPartial]) -> List[Q.Row]:
    t, dims, aggs = merge_groupby_columnar(query, partials)
    rows = []
    for r in range(len(t)):
        ev = {d: dims[i][r] for i, d in enumerate(query.dimensions)}
        for a, col in zip(query.aggregations, aggs):
            ev[a.name] = _py(col[r], a.output_type)
        rows.append(Q.Row(int(t[r]), ev))
    if query.apply_limit_push_down():
        # the partials hold (at least) the first `limit` groups of every device in the push-down
        # order; across devices the cut is taken again in that order
        rows = sorted(rows, key=_push_down_key(query))[:query.limitSpec.limit]
    elif query._ctx_bool("sortByDimsFirst", False) and not query.granularity.is_all:
        # getRowOrdering(false) with sortByDimsFirst: dimensions, then time (GroupByQuery.java:543-553)
        rows.sort(key=lambda r: tuple(_java_key(r.event[d]) for d in query.dimensions))
    return postprocess_groupby(query, rows)


def _push_down_key(query: Q.GroupByQuery):
    """Sort key of GroupByQuery.getRowOrderingForPushDown (:423-528): ORDER BY dimensions under their
    comparator and direction, the other dimensions ascending under LEXICOGRAPHIC, the time first (last
    with sortByDimsFirst; absent for ALL)."""
    fields, seen = [], set()
    for c in query.limitSpec.columns:
        fields.append((c.dimension, O.sort_key(c.dimensionOrder), c.direction == "descending"))
        seen.add(c.dimension)
    fields += [(d, O.sort_key("lexicographic"), False) for d in query.dimensions if d not in seen]
    gran_all = query.granularity.is_all
    dims_first = query._ctx_bool("sortByDimsFirst", False)

    def key(r):
        ks = tuple(O._Desc(f(r.event.get(n))) if desc else f(r.event.get(n)) for n, f, desc in fields)
        if gran_all:
            return ks
        return ks + (r.timestamp,) if dims_first else (r.timestamp,) + ks
    return key


# ----------------------------------------------------------------------------------------------
# groupBy post-processing (GroupByQuery.postProcess: having, then the limitSpec;
# GroupByStrategyV2.applyPostProcessing). Host-side over the merged rows, which arrive in the
# natural (time, dimensions) order.
# ----------------------------------------------------------------------------------------------
def _double_key(v: float):
    if v != v:
        return (1, 0.0, 0)  # Doubles.compare: NaN greatest, -0.0 < 0.0
    return (0, v, 1 if (v == 0.0 and math.copysign(1.0, v) > 0) else 0)


def _having_compare(metric, value) -> int:
    """HavingSpecMetricComparator.compare (having/HavingSpecMetricComparator.java:36-80)."""
    if metric is None:
        a, b = _double_key(0.0), _double_key(float(value))
        return (a > b) - (a < b)
    if isinstance(metric, int):
        if isinstance(value, int):
            return (metric > value) - (metric < value)
        x, y = Fraction(metric), Fraction(Decimal(repr(float(value))))  # BigDecimal.valueOf
        return (x > y) - (x < y)
    m = float(metric)
    if isinstance(value, int):
        x, y = Fraction(Decimal(repr(m))), Fraction(value)
        return (x > y) - (x < y)
    a, b = _double_key(m), _double_key(float(value))
    return (a > b) - (a < b)


def _having_eval(h: Q.HavingSpec, row: Q.Row) -> bool:
    t = h.type
    if t == "always":
        return True
    if t == "never":
        return False
    if t == "and":
        return all(_having_eval(x, row) for x in h.specs)
    if t == "or":
        return any(_having_eval(x, row) for x in h.specs)
    if t == "not":
        return not _having_eval(h.specs[0], row)
    if t == "dimSelector":  # DimensionSelectorHavingSpec.eval: emptyToNull on both sides
        return (row.event.get(h.dimension) or None) == (h.value or None)
    metric = row.event.get(h.aggregation)
    if t == "equalTo" and metric is None and h.value is None:
        return True
    if h.value is None:
        return False
    c = _having_compare(metric, h.value)
    return c > 0 if t == "greaterThan" else (c < 0 if t == "lessThan" else c == 0)


def _limit_needs_sort(query: Q.GroupByQuery) -> bool:
    """DefaultLimitSpec.build (orderby/DefaultLimitSpec.java:122-188): whether the natural order is
    not good enough (then a sort by makeComparator, else just the limit)."""
    ls = query.limitSpec
    if len(query.dimensions) < len(ls.columns):
        return True
    aggs = {a.name for a in query.aggregations}
    for i, c in enumerate(ls.columns):
        if c.dimension in aggs:
            return True
        if c.dimension not in query.dimensions:
            raise ValueError(f"Unknown column in order clause[{c.dimension}]")
        # string dimensions: the natural comparator is LEXICOGRAPHIC
        if c.direction != "ascending" or c.dimensionOrder != "lexicographic" or c.dimension != query.dimensions[i]:
            return True
    return not query.granularity.is_all and query._ctx_bool("sortByDimsFirst", False)


def postprocess_groupby(query: Q.GroupByQuery, rows: List[Q.Row]) -> List[Q.Row]:
    if query.having is not None:
        rows = [r for r in rows if _having_eval(query.having, r)]
    ls = query.limitSpec
    if ls is None:
        return rows
    if _limit_needs_sort(query):
        aggs = {a.name: a for a in query.aggregations}
        dims = set(query.dimensions)
        parts = []
        for c in ls.columns:
            if c.dimension in aggs:
                fn = aggs[c.dimension].compare_key
                kf = (lambda f, n: lambda r: f(r.event[n]))(fn, c.dimension)
            elif c.dimension in dims:
                sk = O.sort_key(c.dimensionOrder)
                kf = (lambda f, n: lambda r: f(r.event.get(n)))(sk, c.dimension)
            else:
                raise ValueError(f"Unknown column in order clause[{c.dimension}]")
            parts.append((kf, c.direction == "descending"))
        by_dims_first = query._ctx_bool("sortByDimsFirst", False)
        gran_all = query.granularity.is_all

        def key(r):
            ks = tuple(O._Desc(f(r)) if desc else f(r) for f, desc in parts)
            if gran_all:
                return ks
            return ks + (r.timestamp,) if by_dims_first else (r.timestamp,) + ks

        rows = sorted(rows, key=key)  # stable: ties keep the natural order
    return rows if ls.limit is None else rows[:ls.limit]


# ----------------------------------------------------------------------------------------------
# factories (QueryRunnerFactory surface)
# ----------------------------------------------------------------------------------------------
def exact_granularity(query, segments: Sequence[GpuSegment]):
    """A period granularity on the fixed grid that is exact only from some instant on
    (Granularity.exact_from: the hours branch gives timestamps before its origin the aligned point
    after them, PeriodGranularity.java:313-326; truncateMillisPeriod's Java remainders misalign
    negative timestamps): when the data reaches before that instant, the query with the calendar
    restatement instead, its interval clipped to the data so the bucket list stays finite."""
    g = query.granularity
    ef = getattr(g, "exact_from", None)
    if ef is None:
        return query
    live = [s for s in segments if s.num_rows]
    if not live or min(s.min_time for s in live) >= ef or query.interval[0] >= ef:
        return query
    lo = max(query.interval[0], min(s.min_time for s in live))
    hi = min(query.interval[1], max(s.max_time for s in live) + 1)
    return dataclasses.replace(query, intervals=[(lo, max(hi, lo + 1))], granularity=g.calendar_form())


def segment_queries(query, segments: Sequence[GpuSegment]):
    """Calendar granularities: makeCursors iterates gran.getIterable(actualInterval) per segment
    (QueryableIndexStorageAdapter.java:367-456; actualInterval = [max(query start, minTime),
    min(query end, bucketEnd(maxTime)))), i.e. bucketStart(actual start) and increments from there.
    With an origin whose day clamps (P1M from Jan 31: truncate gives Apr 30, the chain from the query
    start Apr 28) that chain is not a slice of the query interval's, which the engine buckets every
    segment of a call on. Returns None when every segment's chain lies on the query's list (the
    batched path is exact); else one query per segment (None for a segment outside the interval)
    whose interval is the segment's actual interval, so each runs on its own chain."""
    g = query.granularity
    if not g.is_calendar:
        return None
    qs, qe = query.interval
    qlist = g.bucket_starts((qs, qe))
    qpos = {t: i for i, t in enumerate(qlist)}
    out, diverge = [], False
    for s in segments:
        lo, hi = max(qs, s.min_time), min(qe, g.bucket_end(s.max_time))
        if s.num_rows == 0 or hi <= lo:
            out.append(None)
            continue
        sl = g.bucket_starts((lo, hi))
        i = qpos.get(sl[0])
        diverge |= i is None or qlist[i:i + len(sl)] != sl
        out.append(dataclasses.replace(query, intervals=[(lo, hi)]))
    return out if diverge else None


def _run_split(factory, segments, queries, query, stats):
    """Per segment on its own bucket chain (segment_queries), merged by the toolchest (the
    reference's per-segment runners + mergeResults)."""
    per = []
    for s, q in zip(segments, queries):
        if q is not None:
            per.extend(factory.per_segment([s], q, stats))
    return factory.toolchest.merge(query, per)


class SegmentQueryRunner:
    """QueryRunner for one segment (QueryRunnerFactory.createRunner)."""

    def __init__(self, factory, segment: GpuSegment):
        self.factory, self.segment = factory, segment

    def run(self, query):
        query = exact_granularity(query, [self.segment])
        split = segment_queries(query, [self.segment])
        if split is not None:
            return _run_split(self.factory, [self.segment], split, query, None)
        return self.factory.toolchest.merge(query, self.factory.per_segment([self.segment], query))


class MergedQueryRunner:
    """QueryRunnerFactory.mergeRunners: all segments of one device run as one batched native call."""

    def __init__(self, factory, runners: Iterable[SegmentQueryRunner]):
        self.factory = factory
        self.segments = [r.segment for r in runners]
        self.stats = RunStats()

    def run(self, query):
        query = exact_granularity(query, self.segments)
        split = segment_queries(query, self.segments)
        if split is not None:
            return _run_split(self.factory, self.segments, split, query, self.stats)
        return self.factory.run_merged(self.segments, query, self.stats)


class _ToolChest:
    def __init__(self, merge_fn):
        self.merge = merge_fn


class TimeseriesQueryRunnerFactory:
    toolchest = _ToolChest(merge_timeseries)

    @staticmethod
    def per_segment(segments, query, stats=None):
        return timeseries_per_segment(segments, query, stats)

    def run_merged(self, segments, query, stats=None):
        # every device's segments in one engine call, the buckets folded natively (dg_timeseries_merge)
        return run_timeseries(segments, query, stats)

    def createRunner(self, segment):
        return SegmentQueryRunner(self, segment)

    def mergeRunners(self, runners):
        return MergedQueryRunner(self, runners)


class TopNQueryRunnerFactory(TimeseriesQueryRunnerFactory):
    toolchest = _ToolChest(merge_topn)

    @staticmethod
    def per_segment(segments, query, stats=None):
        return topn_per_segment(segments, query, stats)

    def run_merged(self, segments, query, stats=None):
        # TopNBinaryFn fold inside the engine (dg_topn_merge)
        return run_topn(segments, query, stats)


class GroupByQueryRunnerFactory(TimeseriesQueryRunnerFactory):
    toolchest = _ToolChest(merge_groupby)

    @staticmethod
    def per_segment(segments, query, stats=None):
        return groupby_per_segment(segments, query, stats)

    def run_merged(self, segments, query, stats=None):
        # the engine merges each device's segments (GroupByMergingQueryRunnerV2) and the devices'
        # results by value on the device (dg_groupby_merge_devices: peer copies, no host merge)
        if len(_group_by_device(segments)) == 1:
            return self.toolchest.merge(query, groupby_per_device(segments, query, stats))
        res = groupby_merge_devices(segments, query, stats)
        try:
            for r in res:  # (each key range keeps its first `limit` groups; the toolchest re-limits)
                r.apply_limit_push_down()
            return self.toolchest.merge(query, [r.fetch() for r in res])
        finally:
            for r in res:
                r.release()


FACTORIES = {Q.TimeseriesQuery: TimeseriesQueryRunnerFactory(), Q.TopNQuery: TopNQueryRunnerFactory(),
             Q.GroupByQuery: GroupByQueryRunnerFactory()}


def run_query(query, segments: Sequence[GpuSegment], stats: Optional[RunStats] = None):
    """QueryRunnerFactoryConglomerate lookup + mergeRunners over the given segments."""
    if isinstance(query, dict):
        query = Q.query_from_json(query)
    f = FACTORIES[type(query)]
    runner = f.mergeRunners([f.createRunner(s) for s in segments])
    if stats is not None:
        runner.stats = stats
    return runner.run(query)
