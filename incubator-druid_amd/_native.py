"""ctypes binding of the C-ABI (include/druidgpu.h) — the same entry points a JNI shim binds.

The library is built in-tree (``lib/libdruidgpu.so``). There is no fallback: if the HIP library
cannot be loaded the product path raises, it never silently runs on the CPU.
"""
from __future__ import annotations

import ctypes

import numpy as np
import json
import os
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
# DRUID_AMD_LIB: an alternative in-tree build of the same library (A/B variants of a kernel)
LIB_PATH = os.environ.get("DRUID_AMD_LIB") or os.path.join(_HERE, "lib", "libdruidgpu.so")

DG_OK = 0
ERRORS = {1: "DG_ERR_FORMAT", 2: "DG_ERR_UNSUPPORTED", 3: "DG_ERR_OOM", 4: "DG_ERR_INTERRUPTED",
          5: "DG_ERR_TABLE_FULL", 6: "DG_ERR_ARG", 7: "DG_ERR_DEVICE", 8: "DG_ERR_NOT_FOUND", 9: "DG_ERR_TIMEOUT"}
ERR_INTERRUPTED, ERR_TIMEOUT = 4, 9
COL_MISSING, COL_LONG, COL_FLOAT, COL_DOUBLE, COL_STRING, COL_UNSUPPORTED = range(6)
F_AND, F_OR, F_NOT, F_SELECTOR, F_IN, F_BOUND = 1, 2, 3, 4, 5, 6
ORDER = {"lexicographic": 0, "numeric": 1}
LIMIT_GROUP_ELEMENTS = 1


class DruidGpuError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class UnsupportedQuery(DruidGpuError):
    """DG_ERR_UNSUPPORTED: the reference keeps its CPU engine for this shape."""


class QueryInterrupted(DruidGpuError):
    pass


class ResourceLimitExceeded(DruidGpuError):
    pass


class dg_filter(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("n_children", ctypes.c_int32), ("dimension", ctypes.c_char_p),
                ("values", ctypes.POINTER(ctypes.c_char_p)), ("n_values", ctypes.c_int32),
                ("lower", ctypes.c_char_p), ("upper", ctypes.c_char_p), ("lower_strict", ctypes.c_int32),
                ("upper_strict", ctypes.c_int32), ("ordering", ctypes.c_int32)]


class dg_agg(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("field", ctypes.c_char_p), ("filter", ctypes.c_void_p),
                ("n_filter", ctypes.c_int32)]


class dg_scan(ctypes.Structure):
    _fields_ = [("interval_start", ctypes.c_int64), ("interval_end", ctypes.c_int64),
                ("period_ms", ctypes.c_int64), ("origin_ms", ctypes.c_int64),
                ("filter", ctypes.POINTER(dg_filter)), ("n_filter", ctypes.c_int32),
                ("aggs", ctypes.POINTER(dg_agg)), ("n_aggs", ctypes.c_int32),
                ("cancel", ctypes.POINTER(ctypes.c_int32)), ("bucket_starts", ctypes.c_void_p),
                ("n_bucket_starts", ctypes.c_int32), ("descending", ctypes.c_int32),
                ("seg_bounds", ctypes.c_void_p), ("timeout_ms", ctypes.c_int64)]


class dg_metrics(ctypes.Structure):
    _fields_ = [("segment_rows", ctypes.c_int64), ("pre_filtered_rows", ctypes.c_int64),
                ("selected_rows", ctypes.c_int64), ("bytes_read", ctypes.c_int64),
                ("bitmap_ms", ctypes.c_double), ("decode_ms", ctypes.c_double),
                ("aggregate_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("keygen_ms", ctypes.c_double), ("sort_ms", ctypes.c_double), ("reduce_ms", ctypes.c_double),
                ("sort_passes", ctypes.c_int32), ("key_bits", ctypes.c_int32), ("groups", ctypes.c_int64),
                ("decode_side_ms", ctypes.c_double), ("bytes_side", ctypes.c_int64),
                ("lz4_general_ms", ctypes.c_double), ("lz4_general_bytes", ctypes.c_int64),
                ("lz4_general_blocks", ctypes.c_int32), ("lz4_general_launches", ctypes.c_int32),
                ("bitmap_bytes", ctypes.c_int64), ("reduce_kernel_ms", ctypes.c_double),
                ("lz4_fused_blocks", ctypes.c_int64), ("lz4_general_wall_ms", ctypes.c_double),
                ("lz4_flow_blocks", ctypes.c_int64), ("lz4_flow_bytes", ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class dg_topn(ctypes.Structure):
    _fields_ = [("dimension", ctypes.c_char_p), ("metric_agg", ctypes.c_int32), ("inverted", ctypes.c_int32),
                ("threshold", ctypes.c_int32), ("dim_order", ctypes.c_int32), ("previous_stop", ctypes.c_char_p),
                ("min_rank", ctypes.c_void_p), ("bucket_cap", ctypes.c_int32), ("out_bucket_time", ctypes.c_void_p)]


class dg_topn_lists(ctypes.Structure):
    _fields_ = [("n_lists", ctypes.c_int32), ("list_n", ctypes.c_void_p), ("stride", ctypes.c_int32),
                ("keys", ctypes.c_void_p), ("values", ctypes.c_void_p)]


class dg_groupby(ctypes.Structure):
    _fields_ = [("dimensions", ctypes.POINTER(ctypes.c_char_p)), ("n_dims", ctypes.c_int32)]


class dg_record_layout(ctypes.Structure):
    _fields_ = [("n_aggs", ctypes.c_int32), ("kinds", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("record_size", ctypes.c_int32), ("big_endian", ctypes.c_int32)]


class dg_row_column(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("type", ctypes.c_int32), ("card", ctypes.c_int32),
                ("dict", ctypes.c_void_p), ("ids", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("offsets", ctypes.c_void_p)]


class dg_order_column(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("descending", ctypes.c_int32), ("rank", ctypes.c_void_p)]


class dg_limit(ctypes.Structure):
    _fields_ = [("columns", ctypes.c_void_p), ("n_columns", ctypes.c_int32), ("limit", ctypes.c_int32),
                ("sort_by_dims_first", ctypes.c_int32)]


class dg_keyspace(ctypes.Structure):
    _fields_ = [("n_dims", ctypes.c_int32), ("card", ctypes.c_void_p), ("period_ms", ctypes.c_int64),
                ("bucket0", ctypes.c_int64), ("n_buckets", ctypes.c_int64), ("universal_time", ctypes.c_int64),
                ("n_aggs", ctypes.c_int32), ("agg_kinds", ctypes.c_void_p)]


# every symbol the header declares (checked by the CPU test suite)
EXPORTS = [
    "dg_last_error", "dg_abi_version", "dg_device_count", "dg_context_create", "dg_context_release",
    "dg_context_set_stream", "dg_segment_attach", "dg_segment_release", "dg_segment_num_rows",
    "dg_segment_interval", "dg_segment_time_bounds", "dg_segment_num_columns", "dg_segment_column_name",
    "dg_segment_column_type", "dg_segment_device_bytes", "dg_segment_dim_cardinality", "dg_segment_dim_value",
    "dg_segment_dim_dictionary", "dg_segment_set_dim_order", "dg_filter_bitmap", "dg_timeseries_run", "dg_topn_run", "dg_topn_merge", "dg_groupby_run",
    "dg_result_groups", "dg_result_fetch_groups", "dg_result_fetch_rows", "dg_result_dim_cardinality",
    "dg_result_dim_dictionary", "dg_result_release", "dg_keyspace_bits", "dg_result_export", "dg_keys_partition",
    "dg_merge", "dg_records_pack", "dg_debug_lz4_decode", "dg_result_limit",
    "dg_segment_from_rows", "dg_context_set_limit", "dg_groupby_merge_devices", "dg_timeseries_merge",
    "dg_debug_lz4_classify", "dg_host_alloc", "dg_host_free", "dg_set_phase_timing", "dg_debug_probe",
]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                           "(make -C incubator-druid_amd/csrc); there is no CPU fallback")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7, the
    # engine's NEEDED name). Loaded first, it is the one the engine binds to, so torch tensors,
    # streams and RCCL (torch.distributed) share the engine's device runtime. Loaded after the
    # engine's /opt/rocm copy, torch would map a second runtime that finds no devices.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    l = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, cp = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_char_p
    P = ctypes.POINTER
    sig = {
        "dg_last_error": (cp, []),
        "dg_abi_version": (ctypes.c_int, []),
        "dg_device_count": (ctypes.c_int, [P(ctypes.c_int)]),
        "dg_context_create": (ctypes.c_int, [ctypes.c_int, P(vp)]),
        "dg_context_release": (None, [vp]),
        "dg_context_set_stream": (ctypes.c_int, [vp, vp]),
        "dg_context_set_limit": (ctypes.c_int, [vp, i32, i64]),
        "dg_segment_attach": (ctypes.c_int, [vp, cp, P(vp)]),
        "dg_segment_release": (None, [vp]),
        "dg_segment_from_rows": (ctypes.c_int, [vp, i64, vp, i64, i64, vp, i32, P(vp)]),
        "dg_segment_num_rows": (i64, [vp]),
        "dg_segment_interval": (ctypes.c_int, [vp, P(i64), P(i64)]),
        "dg_segment_time_bounds": (ctypes.c_int, [vp, P(i64), P(i64)]),
        "dg_segment_num_columns": (ctypes.c_int, [vp]),
        "dg_segment_column_name": (cp, [vp, ctypes.c_int]),
        "dg_segment_column_type": (ctypes.c_int, [vp, cp]),
        "dg_segment_device_bytes": (i64, [vp]),
        "dg_segment_dim_cardinality": (i32, [vp, cp]),
        "dg_segment_dim_value": (ctypes.c_int, [vp, cp, i32, P(ctypes.c_void_p), P(i32)]),
        "dg_segment_dim_dictionary": (ctypes.c_int, [vp, cp, vp, vp, P(i64)]),
        "dg_segment_set_dim_order": (ctypes.c_int, [vp, cp, i32, vp, i32, i32]),
        "dg_filter_bitmap": (ctypes.c_int, [vp, P(dg_filter), i32, vp, P(i64)]),
        "dg_timeseries_run": (ctypes.c_int, [P(vp), i32, P(dg_scan), i32, vp, vp, vp, vp, P(dg_metrics)]),
        "dg_topn_run": (ctypes.c_int, [P(vp), i32, P(dg_scan), P(dg_topn), vp, vp, vp, P(dg_metrics)]),
        "dg_topn_merge": (ctypes.c_int, [vp, P(dg_scan), P(dg_topn), P(dg_topn_lists), P(i32), vp, vp, vp]),
        "dg_groupby_run": (ctypes.c_int, [P(vp), i32, P(dg_scan), P(dg_groupby), P(vp), P(dg_metrics)]),
        "dg_result_groups": (i64, [vp]),
        "dg_result_fetch_groups": (ctypes.c_int, [vp, i64, i64, vp, vp, vp]),
        "dg_result_fetch_rows": (ctypes.c_int, [vp, i64, i64, vp]),
        "dg_result_dim_cardinality": (i32, [vp, i32]),
        "dg_result_dim_dictionary": (ctypes.c_int, [vp, i32, vp, vp, P(i64)]),
        "dg_result_release": (None, [vp]),
        "dg_result_limit": (ctypes.c_int, [vp, P(dg_limit)]),
        "dg_keyspace_bits": (ctypes.c_int, [P(dg_keyspace), P(i32)]),
        "dg_result_export": (ctypes.c_int, [vp, P(dg_keyspace), P(vp), vp, vp]),
        "dg_keys_partition": (ctypes.c_int, [vp, vp, i64, vp, i32, vp]),
        "dg_merge": (ctypes.c_int, [vp, P(dg_keyspace), vp, vp, i64, P(vp), P(dg_metrics)]),
        "dg_groupby_merge_devices": (ctypes.c_int, [P(vp), i32, P(vp), i32, P(vp), P(dg_metrics)]),
        "dg_timeseries_merge": (ctypes.c_int, [P(dg_scan), i32, vp, i32, vp, vp, vp, i32, i32, P(i32), vp, vp, vp]),
        "dg_records_pack": (ctypes.c_int, [vp, i64, P(dg_record_layout), vp]),
        "dg_debug_lz4_decode": (ctypes.c_int, [vp, P(vp), P(i32), i32, vp, P(i32), P(ctypes.c_double), vp]),
        "dg_debug_lz4_classify": (ctypes.c_int, [vp, i32, P(i32)]),
        "dg_host_alloc": (ctypes.c_int, [i64, P(vp)]),
        "dg_host_free": (None, [vp]),
        "dg_set_phase_timing": (ctypes.c_int, [ctypes.c_int32]),
        "dg_debug_probe": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                          P(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(l, name)
        fn.restype = res
        fn.argtypes = args
    _lib = l
    return l


def check(rc: int):
    if rc == DG_OK:
        return
    msg = lib().dg_last_error().decode("utf-8", "replace")
    if rc == 2:
        raise UnsupportedQuery(rc, msg)
    if rc == 4:
        raise QueryInterrupted(rc, msg)
    if rc == 5:
        raise ResourceLimitExceeded(rc, msg)
    raise DruidGpuError(rc, msg)


def _b(s: Optional[str]) -> Optional[bytes]:
    return None if s is None else str(s).encode("utf-8")


class FilterProgram:
    """DimFilter tree -> prefix-ordered dg_filter array (keeps the backing strings alive)."""

    def __init__(self, flt, query_module, segments=None):
        self._keep: List = []
        self.nodes: List[dg_filter] = []
        self.Q = query_module
        self.segments = segments
        if flt is not None:
            self._emit(flt)
        self.array = (dg_filter * max(len(self.nodes), 1))(*self.nodes) if self.nodes else None

    def _strs(self, vals: Sequence[Optional[str]]):
        arr = (ctypes.c_char_p * max(len(vals), 1))(*[_b(v) for v in vals])
        self._keep.append(arr)
        return arr

    def _emit(self, f):
        Q = self.Q
        node = dg_filter()
        if isinstance(f, Q.AndDimFilter) or isinstance(f, Q.OrDimFilter):
            node.kind = F_AND if isinstance(f, Q.AndDimFilter) else F_OR
            node.n_children = len(f.fields)
            self.nodes.append(node)
            for c in f.fields:
                self._emit(c)
            return
        if isinstance(f, Q.NotDimFilter):
            node.kind = F_NOT
            node.n_children = 1
            self.nodes.append(node)
            self._emit(f.field)
            return
        dim = _b(f.dimension)
        self._keep.append(dim)
        node.dimension = dim
        if isinstance(f, Q.SelectorDimFilter):
            node.kind = F_SELECTOR
            node.values = self._strs([f.value])
            node.n_values = 1
        elif isinstance(f, Q.InDimFilter):
            node.kind = F_IN
            node.values = self._strs(list(f.values))
            node.n_values = len(f.values)
        elif isinstance(f, Q.PREDICATE_FILTERS) or (isinstance(f, Q.BoundDimFilter) and f.ordering not in ORDER):
            # predicate over dictionary values (Filters.matchPredicate): the host evaluates it on the
            # dictionaries of the segments of this call, the engine unions the matching values' bitmaps
            if self.segments is None:
                raise UnsupportedQuery(2, f"filter {type(f).__name__} needs the segments' dictionaries")
            if any(s.column_type(f.dimension) in (COL_LONG, COL_FLOAT, COL_DOUBLE) for s in self.segments):
                # over String.valueOf(number) of every row: no dictionary to evaluate it on
                raise UnsupportedQuery(2, f"filter {type(f).__name__} on numeric column {f.dimension}")
            vals = predicate_values(f, self.segments, Q)
            node.kind = F_IN
            node.values = self._strs(vals)
            node.n_values = len(vals)
        elif isinstance(f, Q.BoundDimFilter):
            node.kind = F_BOUND
            lo, hi = _b(f.lower), _b(f.upper)
            self._keep += [lo, hi]
            node.lower, node.upper = lo, hi
            node.lower_strict, node.upper_strict = int(f.lowerStrict), int(f.upperStrict)
            if f.ordering not in ORDER:
                raise UnsupportedQuery(2, f"bound ordering {f.ordering}")
            node.ordering = ORDER[f.ordering]
        else:
            raise UnsupportedQuery(2, f"filter {type(f).__name__}")
        self.nodes.append(node)


def predicate_values(f, segments, Q) -> List[Optional[str]]:
    """Dictionary values (over the given segments) a predicate filter accepts, null included when the
    predicate accepts it (missing columns then read as all-true, Filters.matchPredicate). Cached per
    segment and filter."""
    key = (f.dimension, json.dumps(f.to_json(), sort_keys=True))
    pred = f.predicate if not isinstance(f, Q.BoundDimFilter) else _bound_predicate(f)
    out = set()
    for seg in segments:
        cache = seg.__dict__.setdefault("_pred_cache", {})
        if key not in cache:
            vals = seg.dictionary(f.dimension)
            cache[key] = frozenset(v for v in vals if pred(v))
        out |= cache[key]
    if pred(None):
        out.add(None)
    return sorted(out, key=lambda v: (v is not None, v or ""))


def _bound_predicate(f):
    """BoundFilter.doesMatch (segment/filter/BoundFilter.java:249-275) for orderings the engine does not
    evaluate itself (alphanumeric, strlen), through the comparator's sort key."""
    from . import ordering as O
    from .query import _empty_to_null
    key = O.sort_key(f.ordering)
    lower, upper = _empty_to_null(f.lower), _empty_to_null(f.upper)
    has_lower, has_upper = f.lower is not None, f.upper is not None

    def pred(v):
        if v is None:
            return ((not has_lower) or (lower is None and not f.lowerStrict)) and \
                   ((not has_upper) or upper is not None or not f.upperStrict)
        kv = key(v)
        lc = 1 if not has_lower else (kv > key(f.lower)) - (kv < key(f.lower))
        uc = 1 if not has_upper else (key(f.upper) > kv) - (key(f.upper) < kv)
        return (lc > 0 if f.lowerStrict else lc >= 0) and (uc > 0 if f.upperStrict else uc >= 0)
    return pred


def make_scan(query, query_module, cancel: Optional[ctypes.c_int32] = None, segments=None, filters: bool = True):
    """Build a dg_scan (+ keep-alive list) from a query's interval, granularity, filter and aggs.
    segments: the segments of the call (predicate filters are resolved over their dictionaries);
    filters=False leaves the query and aggregator filters out (merges only need the aggregators)."""
    keep = []
    fp = FilterProgram(query.effective_filter() if filters else None, query_module, segments)
    keep.append(fp)
    aggs = (dg_agg * max(len(query.aggregations), 1))()
    for i, a in enumerate(query.aggregations):
        aggs[i].kind = a.kind
        fld = _b(a.fieldName) if a.kind != 0 else None
        keep.append(fld)
        aggs[i].field = fld
        if a.filter is not None and filters:  # FilteredAggregatorFactory: the delegate's row matcher
            afp = FilterProgram(a.filter.optimize(), query_module, segments)
            keep.append(afp)
            if afp.array is not None:
                aggs[i].filter = ctypes.cast(afp.array, ctypes.c_void_p)
                aggs[i].n_filter = len(afp.nodes)
    keep.append(aggs)
    s = dg_scan()
    s.interval_start, s.interval_end = query.interval
    gran = query.granularity
    if gran.is_calendar:
        # Granularity.getIterable(interval) of the query interval (the engine buckets by these starts)
        starts = np.asarray(gran.bucket_starts(tuple(query.interval)), dtype=np.int64)
        keep.append(starts)
        s.bucket_starts = starts.ctypes.data
        s.n_bucket_starts = len(starts)
        if segments:  # per segment: where its iterable starts, where its dataInterval ends
            qs = query.interval[0]
            b = np.asarray([[gran.bucket_start(max(qs, sg.min_time)), gran.bucket_end(sg.max_time)] if sg.num_rows
                            else [0, 0] for sg in segments], np.int64).reshape(-1)
            keep.append(b)
            s.seg_bounds = b.ctypes.data
    else:
        s.period_ms = gran.period_ms
        s.origin_ms = gran.origin_ms
    s.descending = int(bool(getattr(query, "descending", False)))
    if fp.array is not None:
        s.filter = ctypes.cast(fp.array, ctypes.POINTER(dg_filter))
        s.n_filter = len(fp.nodes)
    s.aggs = ctypes.cast(aggs, ctypes.POINTER(dg_agg))
    s.n_aggs = len(query.aggregations)
    if cancel is not None:
        s.cancel = ctypes.pointer(cancel)
        keep.append(cancel)
    # QueryContexts.getTimeout: the context's "timeout" (ms; 0 = none)
    s.timeout_ms = int((getattr(query, "context", None) or {}).get("timeout", 0) or 0)
    return s, keep
