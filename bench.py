"""Benchmark: filtered rows aggregated per second (+ HBM GB/s vs the MI355X roofline).

Default workload = BASELINE.json configs[2], the largest single-GPU configuration: GroupByV2 over
two high-cardinality string dimensions (dimUniform ~100k values x dimHyperUnique 100k values, both
3-byte dictionary ids, ~1 group per row) with longSum(sumLongSequential) + doubleSum(sumFloatNormal),
100M rows = 8 segments x 12.5M rows per GPU, 'basic' schema columns written as Druid v9 segments
with the reference's default IndexSpec (Concise bitmaps, LZ4-HC blocks, LONGS encoding).

A step = one groupBy query over the rank's 8 segments: per-segment grouping + the
GroupByMergingQueryRunnerV2 merge by value, i.e. the merged, ordered groups, produced in HBM
(dg_groupby_run; LZ4 blocks decoded again every step, as the reference decompresses per query).
The groups are not copied to the host inside the timed region (the boundary hands them over as a
dg_result; the PCIe-inclusive rate is measured after the loop and reported as `pcie_fetch`).
For N > 1 (weak scaling, one process per GPU) the ranks' groups are exchanged by key range over RCCL
and merged on the receiving GPU (dg_merge), so every rank ends with its range of the final result.

The other configs (--config) are secondary lines / parity shapes: topn (configs[1]), timeseries
(configs[0]), filtered (configs[3], one GPU's share), ts_hourly / groupby_hourly (configs[4]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config groupby|topn|...]

--gpus N > 1 starts N ranks itself (launch_ranks) unless a launcher already did (WORLD_SIZE set,
which must equal N); LOCAL_RANK picks the GPU (DG_BENCH_DEVICE overrides it for a one-GPU rehearsal).
"""
import argparse
import ctypes
import json
import os
import shutil
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import importlib  # noqa: E402

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

BASIC = {"dims": None, "metrics": None}
GB_COLS = {"dims": ["dimUniform", "dimHyperUnique"], "metrics": ["rows", "sumLongSequential", "sumFloatNormal"]}
PHASE_STEPS = 3  # untimed steps after the timed region that sample the phase times (phases_ms)

CONFIGS = {
    # name: (rows per segment, segments per GPU, description, columns written)
    "groupby": (12_500_000, 8, "BASELINE configs[2]: GroupByV2 dimUniform x dimHyperUnique (3-byte ids, ~1 group/row) "
                               "+ longSum/doubleSum, 100M rows = 8 x 12.5M-row segments per MI355X", GB_COLS),
    "topn": (750_000, 4, "BASELINE configs[1]: TopNBenchmark basic, topN dimUniform threshold=10 by doubleSum, "
                         "4 x 750k rows/GPU", BASIC),
    "topn_numeric": (750_000, 4, "TopNBenchmark basic.numericSort: DimensionTopNMetricSpec(NUMERIC), longSum, "
                                 "4 x 750k rows/GPU", BASIC),
    "topn_alphanumeric": (750_000, 4, "TopNBenchmark basic.alphanumericSort: DimensionTopNMetricSpec(ALPHANUMERIC), "
                                      "longSum, 4 x 750k rows/GPU", BASIC),
    "timeseries": (750_000, 1, "BASELINE configs[0]: TimeseriesBenchmark basic, ALL count+longSum+doubleSum, "
                               "selector dimSequential=399", BASIC),
    "ts_hourly": (15_625_000, 8, "BASELINE configs[4]a: 1B-row dataset (64 x 15.625M rows, 30 days), 8 segments/GPU: "
                                 "timeseries HOUR count+longSum+doubleSum+longMax+doubleMin", BASIC),
    "groupby_hourly": (15_625_000, 8, "BASELINE configs[4]b: same 1B-row dataset, 8 segments/GPU: groupBy HOUR "
                                      "(dimZipf, dimSequential) longSum+doubleSum", BASIC),
    "filtered": (12_500_000, 1, "BASELINE configs[3] (one GPU's 12.5M-row share): compound AND/OR bound+selector+in "
                                "filter, timeseries count", BASIC),
}


def make_query(Q, name):
    iv = ["1970-01-01/2020-01-01"]
    if name == "topn":
        return Q.TopNQuery(intervals=iv, dimension="dimUniform", metric="sumFloatNormal", threshold=10,
                           aggregations=[Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")])
    if name in ("topn_numeric", "topn_alphanumeric"):
        ordering = name.split("_")[1]
        return Q.TopNQuery(intervals=iv, dimension="dimUniform", threshold=10,
                           metric={"type": "dimension", "ordering": ordering, "previousStop": None},
                           aggregations=[Q.long_sum("sumLongSequential")])
    if name == "timeseries":
        return Q.TimeseriesQuery(intervals=iv, aggregations=[Q.count("rows"), Q.long_sum("sumLongSequential"),
                                                             Q.double_sum("sumFloatNormal")],
                                 filter=Q.SelectorDimFilter("dimSequential", "399"))
    if name == "ts_hourly":
        return Q.TimeseriesQuery(intervals=iv, granularity="hour",
                                 aggregations=[Q.count("rows"), Q.long_sum("sumLongSequential"),
                                               Q.double_sum("sumFloatNormal"), Q.long_max("maxLongUniform"),
                                               Q.double_min("minFloatZipf")])
    if name == "groupby_hourly":
        return Q.GroupByQuery(intervals=iv, granularity="hour", dimensions=["dimZipf", "dimSequential"],
                              aggregations=[Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")])
    if name == "groupby":
        return Q.GroupByQuery(intervals=iv, dimensions=["dimUniform", "dimHyperUnique"],
                              aggregations=[Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")])
    if name == "filtered":
        f = Q.OrDimFilter([Q.AndDimFilter([Q.BoundDimFilter("dimSequential", "100", "200"),
                                           Q.InDimFilter("dimZipf", ["1", "2", "3"])]),
                           Q.SelectorDimFilter("dimUniform", "199"),
                           Q.NotDimFilter(Q.SelectorDimFilter("dimZipf", "7"))])
        return Q.TimeseriesQuery(intervals=iv, aggregations=[Q.count("rows")], filter=f)
    raise ValueError(name)


DATASET_1B = {"segments": 64, "interval": (0, 30 * 86_400_000),
              "dims": ["dimZipf", "dimSequential"],
              "metrics": ["sumLongSequential", "sumFloatNormal", "maxLongUniform", "minFloatZipf"]}


def _write_one(job):
    DG = importlib.import_module("incubator-druid_amd.datagen")
    p, rows, seed, bitmap, compression, lz4_mode, part, long_encoding, cols = job
    if part is None:
        DG.write_basic_segment(p, rows, seed=seed, bitmap=bitmap, compression=compression, lz4_mode=lz4_mode,
                               long_encoding=long_encoding, dims=cols["dims"], metrics=cols["metrics"])
    else:  # time chunk `part` of the 1B-row dataset; the segment's interval is its chunk
        W = importlib.import_module("incubator-druid_amd.writer")
        n_all = DATASET_1B["segments"]
        start, end = DATASET_1B["interval"]
        spec = DG.basic_columns(rows, seed, interval=DATASET_1B["interval"], row_offset=part * rows,
                                total_rows=n_all * rows, dims=DATASET_1B["dims"], metrics=DATASET_1B["metrics"])
        span = (end - start) // n_all
        spec.interval = (start + part * span, end if part == n_all - 1 else start + (part + 1) * span)
        idx = np.arange(part * rows, (part + 1) * rows, dtype=np.int64)
        spec.timestamps = ts = start + idx * (end - start) // (n_all * rows)  # row r at floor(r * 30d / 1e9)
        assert spec.interval[0] <= int(ts[0]) and int(ts[-1]) < spec.interval[1], (part, spec.interval, ts[0], ts[-1])
        W.write_segment(p, spec, bitmap=bitmap, compression=compression, lz4_mode=lz4_mode,
                        long_encoding=long_encoding)
    return p


def ensure_segments(root, rank, nseg, rows, compression, bitmap, lz4_mode, cols, partitioned=False, workers=8,
                    long_encoding="longs"):
    """This rank's segments (seed 9999 + global segment index). partitioned: consecutive time chunks
    of the 1B-row dataset (rank r holds global chunks r*nseg ..); otherwise every segment spans the
    basic interval like the JMH benchmarks' segments. Written once, in parallel, and reused."""
    tag = ("p1b_" if partitioned else "") + ("auto_" if long_encoding == "auto" else "")
    if cols["dims"] is not None:
        tag += "c" + "-".join(cols["dims"] + cols["metrics"]) + "_"
    d = os.path.join(root, f"{tag}r{rows}_s{nseg}_{compression}_{bitmap}_{lz4_mode}", f"rank{rank}")
    marker = os.path.join(d, "DONE")
    paths = [os.path.join(d, f"seg{i:04d}") for i in range(nseg)]
    if not os.path.exists(marker):
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d, exist_ok=True)
        jobs = [(p, rows, 9999 + rank * nseg + i, bitmap, compression, lz4_mode,
                 (rank * nseg + i) if partitioned else None, long_encoding, cols) for i, p in enumerate(paths)]
        t0 = time.time()
        if len(jobs) > 1 and workers > 1:
            import multiprocessing as mp
            with mp.get_context("spawn").Pool(min(workers, len(jobs))) as pool:
                for p in pool.imap_unordered(_write_one, jobs):
                    print(f"[rank {rank}] wrote {p} ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
        else:
            for j in jobs:
                print(f"[rank {rank}] wrote {_write_one(j)} ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
        open(marker, "w").close()
    return paths


def _cpu_model():
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads():
    """The cores this process can actually use: its affinity set (sched_getaffinity, as SURVEY §8(d)
    asks for), capped by the cgroup CPU quota (a 16-core quota on a 256-thread affinity set runs 16
    cores' worth of work, however many threads are spawned)."""
    try:
        aff = max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        aff = max(1, os.cpu_count() or 1)
    q = _cpu_quota()
    return max(1, min(aff, int(q))) if q else aff


def _cpu_quota():
    """The cgroup CPU quota in cores (cpu.max), or None when unlimited / unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def _cpu_lib():
    """oracle/libdruid_cpu.so (C -O3 -march=native restatement of the reference's per-segment loops)."""
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "libdruid_cpu.so"))
    vp, i32, i64, cp = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_char_p
    lib.or_open.restype = vp
    lib.or_open.argtypes = [cp, cp, ctypes.c_int]
    lib.or_close.argtypes = [vp]
    lib.cpu_groupby2.restype = i64
    lib.cpu_groupby2.argtypes = [ctypes.POINTER(vp), ctypes.c_int, cp, cp, cp, cp, vp, vp, i32, ctypes.c_int,
                                 i64, i64, i64, i32, ctypes.POINTER(ctypes.c_double), vp, vp, vp, vp,
                                 ctypes.POINTER(ctypes.c_double)]
    lib.cpu_timeseries.restype = ctypes.c_int
    lib.cpu_timeseries.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp, vp,
                                   ctypes.c_int, i64, i64, i64, i64, i64, i32, ctypes.c_int, vp, vp, vp, vp,
                                   ctypes.POINTER(ctypes.c_double)]
    lib.cpu_topn.restype = ctypes.c_int
    lib.cpu_topn.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp, vp, ctypes.c_int,
                             cp, vp, ctypes.c_int, vp, vp, ctypes.c_int, i32, i32, vp, i32, vp, vp,
                             ctypes.POINTER(ctypes.c_double)]
    return lib


class _CpuSegments:
    """The segments opened by the CPU engine's own reader (and the oracle's, for dictionaries)."""

    def __init__(self, paths):
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        self.O = O
        self.lib = _cpu_lib()
        self.osegs = [O.OracleSegment(p) for p in paths]
        err = ctypes.create_string_buffer(512)
        hs = [self.lib.or_open(p.encode(), err, 512) for p in paths]
        if not all(hs):
            raise IOError(err.value.decode())
        self.hs = hs
        self.handles = (ctypes.c_void_p * len(hs))(*hs)
        self.rows = sum(s.num_rows for s in self.osegs)
        self._keep = []

    def close(self):
        for s, h in zip(self.osegs, self.hs):
            s.close()
            self.lib.or_close(h)

    def merged(self, dim):
        """Merged dictionary (Java String order, nulls first) and per-segment local -> merged id maps."""
        dicts = [s.dictionary(dim) for s in self.osegs]
        merged = sorted(set().union(*map(set, dicts)), key=lambda v: (v is not None, (v or "").encode("utf-16-be")))
        index = {v: i for i, v in enumerate(merged)}
        maps = [np.array([index[v] for v in dd], dtype=np.int32) for dd in dicts]
        return merged, maps

    def filter_program(self, filt):
        """The query filter (DimFilter.optimize) as the engine's postfix program over bitmap leaves, with
        every leaf's dictionary ids per segment (-1 terminated): selector / in / bound leaves under
        And / Or / Not (Filter.getBitmapResult)."""
        O = self.O
        Q = importlib.import_module("incubator-druid_amd.query")
        f = O.o_optimize(filt) if filt is not None else None
        prog, leaves = [], []

        def walk(node):
            if isinstance(node, (Q.AndDimFilter, Q.OrDimFilter)):
                op = -1 if isinstance(node, Q.AndDimFilter) else -2
                for k, ch in enumerate(node.fields):
                    walk(ch)
                    if k:
                        prog.append(op)
            elif isinstance(node, Q.NotDimFilter):
                walk(node.field)
                prog.append(-3)
            else:
                leaves.append(node)
                prog.append(len(leaves) - 1)

        if f is not None:
            walk(f)
        ids = []
        for seg in self.osegs:
            for lf in leaves:
                sel = O.filter_id_set(seg, lf) if seg.is_dim(lf.dimension) else []
                a = np.array(list(sel) + [-1], dtype=np.int32)
                self._keep.append(a)
                ids.append(a.ctypes.data)
        dims = [lf.dimension.encode() for lf in leaves]
        self._keep += [dims]
        P = (ctypes.c_int32 * max(len(prog), 1))(*prog)
        D = (ctypes.c_char_p * max(len(dims), 1))(*dims)
        I = (ctypes.c_void_p * max(len(ids), 1))(*ids)
        self._keep += [P, D, I]
        return P, len(prog), D, I, len(leaves)


def _query_buckets(query, segs):
    """Granularity buckets of a timeseries / groupBy query over the segments: (t_lo, t_hi, origin,
    period, bucket0, nbuckets); ALL = one bucket (fixed UTC periods only, as the benched queries use)."""
    t_lo, t_hi = query.interval
    g = query.granularity
    if g.is_all:
        return t_lo, t_hi, 0, 0, 0, 1
    P, org = g.period_ms, g.origin_ms
    lo = min(s.interval[0] for s in segs)
    hi = max(s.interval[1] for s in segs)
    b0 = (max(lo, t_lo) - org) // P
    b1 = (min(hi, t_hi) - 1 - org) // P
    return t_lo, t_hi, org, P, b0, int(b1 - b0 + 1)


def _baseline_line(value, threads, kind, sample, extra=None):
    d = {"value": value, "unit": "rows/s", "cores": threads, "kind": kind, "sample": sample, "cpu_model": _cpu_model(),
         "nproc": os.cpu_count(), "cgroup_quota_cores": _cpu_quota()}
    if extra:
        d.update(extra)
    return d


def cpu_baseline_timeseries(paths, query, threads):
    """oracle/cpu_engine.c cpu_timeseries on the whole step workload: the filter's bitmaps per segment,
    then the TimeseriesQueryEngine loop over 1 M-row chunks on `threads` cores (LZ4 decoded inside the
    timing). Returns (baseline line, {bucket timestamp: (rows, [agg values])})."""
    cs = _CpuSegments(paths)
    try:
        P, nprog, D, I, nleaf = cs.filter_program(query.filter)
        t_lo, t_hi, org, per, b0, nb = _query_buckets(query, cs.osegs)
        aggs = query.aggregations
        kinds = (ctypes.c_int32 * len(aggs))(*[a.kind for a in aggs])
        cols = (ctypes.c_char_p * len(aggs))(*[(a.fieldName or "").encode() for a in aggs])
        rows = np.zeros(nb, np.int64)
        state = np.zeros(nb * len(aggs), np.uint64)
        secs = ctypes.c_double()
        rc = cs.lib.cpu_timeseries(cs.handles, len(paths), threads, P, nprog, D, I, nleaf, t_lo, t_hi, org, per, b0, nb,
                                   len(aggs), kinds, cols, rows.ctypes.data, state.ctypes.data, ctypes.byref(secs))
        if rc:
            raise RuntimeError("cpu_timeseries failed")
        out = {}
        for b in range(nb):
            if rows[b] or query.granularity.is_all:
                vals = []
                for k, a in enumerate(aggs):
                    v = state[k * nb + b]
                    vals.append(float(v.view(np.float64)) if a.output_type == "double" else int(v.view(np.int64)))
                ts = t_lo if query.granularity.is_all else org + (b0 + b) * per
                out[ts] = (int(rows[b]), vals)
        sel = int(rows.sum())
        line = _baseline_line(sel / secs.value, threads, "port",
                              f"the whole step workload: {len(paths)} segments x {cs.rows // len(paths)} rows, "
                              f"{sel} selected rows in {secs.value:.3f} s (oracle/cpu_engine.c cpu_timeseries, C -O3 "
                              f"-march=native, {threads} threads over 1M-row chunks, bitmap filter + LZ4 decode inside "
                              f"the timing); value = filtered (selected) rows aggregated/s, the GPU line's unit",
                              {"scanned_rows_per_s": cs.rows / secs.value})
        return line, out
    finally:
        cs.close()


def check_timeseries(gpu, cpu, query):
    """Per-bucket equality of the GPU's merged timeseries result with the CPU engine's: the same
    non-empty buckets, counts / long aggregators bit-exact, double aggregators within 1e-9 relative."""
    g = {}
    for r in gpu:
        vals = [r.value[a.name] for a in query.aggregations]
        if query.granularity.is_all or any(v != 0 for v in vals):
            g[r.timestamp] = vals
    c = {ts: v for ts, (n, v) in cpu.items()}
    if query.granularity.is_all:  # one bucket (its timestamp is the cursor's start, not checked here)
        g = {0: v for v in g.values()}
        c = {0: v for v in c.values()}
    out = {"buckets": len(c), "buckets_equal": sorted(g) == sorted(c)}
    longs_ok, maxrel = True, 0.0
    for ts in set(g) & set(c):
        for a, x, y in zip(query.aggregations, g[ts], c[ts]):
            if a.output_type == "double":
                if x != y:
                    rel = abs(x - y) / max(abs(x), abs(y), 1e-300)
                    if rel == rel:
                        maxrel = max(maxrel, rel)
                    else:
                        maxrel = float("inf")
            elif int(x) != int(y):
                longs_ok = False
    out["longs_equal"] = longs_ok
    out["double_max_rel_err"] = maxrel
    out["doubles_within_1e-9"] = maxrel <= 1e-9
    out["per_bucket_equal"] = out["buckets_equal"] and longs_ok and out["doubles_within_1e-9"]
    return out


def cpu_baseline_topn(paths, query, threads):
    """oracle/cpu_engine.c cpu_topn: PooledTopNAlgorithm per segment on `threads` cores (one segment per
    thread, as ChainedExecutionQueryRunner), top max(threshold, 1000) per segment, TopNBinaryFn fold in
    segment order. A numeric metric orders by the aggregator; a DimensionTopNMetricSpec by the value's
    rank under its comparator (the merged dictionary ranked here, before the timing, by the oracle's
    StringComparators restatement), with the LEXICOGRAPHIC optimizer's id cut when it applies (no
    previousStop, no filter, segments inside the interval). Returns (baseline line, [(value, [aggs])])."""
    cs = _CpuSegments(paths)
    try:
        P, nprog, D, I, nleaf = cs.filter_program(query.filter)
        merged, maps = cs.merged(query.dimension)
        R = (ctypes.c_void_p * len(maps))(*[m.ctypes.data for m in maps])
        aggs = query.aggregations
        kinds = (ctypes.c_int32 * len(aggs))(*[a.kind for a in aggs])
        cols = (ctypes.c_char_p * len(aggs))(*[(a.fieldName or "").encode() for a in aggs])
        min_t = int(query.context.get("minTopNThreshold", 1000))
        rank, id_limit, metric = None, 0, 0
        spec = query.metric
        if spec.type == "dimension":
            if spec.previous_stop is not None:
                raise ValueError("cpu_topn: previousStop is not restated")
            import functools
            cmp = cs.O.topn_comparator(spec)  # (InvertedTopNMetricSpec's inverse included)
            order = sorted(range(len(merged)),
                           key=functools.cmp_to_key(lambda a, b: cmp(merged[a], merged[b]) or (a > b) - (a < b)))
            rank = np.empty(len(merged), np.int32)
            rank[np.asarray(order, dtype=np.int64)] = np.arange(len(merged), dtype=np.int32)
            covered = all(query.interval[0] <= s.interval[0] and s.interval[1] <= query.interval[1] for s in cs.osegs)
            if spec.ordering == "lexicographic" and not spec.inverted and query.filter is None and covered:
                id_limit = max(query.threshold, min_t)
        else:
            metric = [a.name for a in aggs].index(spec.metric)
        ids = np.zeros(query.threshold, np.int32)
        vals = np.zeros(query.threshold * len(aggs), np.uint64)
        secs = ctypes.c_double()
        n = cs.lib.cpu_topn(cs.handles, len(paths), threads, P, nprog, D, I, nleaf, query.dimension.encode(), R, len(aggs),
                            kinds, cols, metric, query.threshold, min_t,
                            rank.ctypes.data if rank is not None else None, id_limit,
                            ids.ctypes.data, vals.ctypes.data, ctypes.byref(secs))
        if n < 0:
            raise RuntimeError("cpu_topn failed")
        out = []
        for i in range(n):
            vs = []
            for k, a in enumerate(aggs):
                v = vals[i * len(aggs) + k]
                vs.append(float(v.view(np.float64)) if a.output_type == "double" else int(v.view(np.int64)))
            out.append((merged[ids[i]], vs))
        line = _baseline_line(cs.rows / secs.value, min(threads, len(paths)), "port",
                              f"the whole step workload: {len(paths)} segments x {cs.rows // len(paths)} rows in "
                              f"{secs.value:.3f} s (oracle/cpu_engine.c cpu_topn, C -O3 -march=native, one segment per "
                              f"thread like ChainedExecutionQueryRunner: {min(threads, len(paths))} of {threads} cores "
                              f"busy, LZ4 decode inside the timing)")
        return line, out
    finally:
        cs.close()


def check_topn(gpu, cpu, query):
    """The GPU's final topN list vs the CPU engine's: same dimension values in the same order, long
    aggregators bit-exact, doubles within 1e-9 relative."""
    rows = gpu[0].value if gpu else []
    out = {"entries": len(rows), "values_equal": [r[query.dimension] for r in rows] == [v for v, _ in cpu]}
    longs_ok, maxrel = True, 0.0
    for r, (_, vs) in zip(rows, cpu):
        for a, y in zip(query.aggregations, vs):
            x = r[a.name]
            if a.output_type == "double":
                if x != y:
                    maxrel = max(maxrel, abs(x - y) / max(abs(x), abs(y), 1e-300))
            elif int(x) != int(y):
                longs_ok = False
    out["longs_equal"] = longs_ok
    out["double_max_rel_err"] = maxrel
    out["doubles_within_1e-9"] = maxrel <= 1e-9
    out["per_entry_equal"] = out["values_equal"] and longs_ok and out["doubles_within_1e-9"]
    return out


def cpu_baseline_groupby(paths, query, threads, want_groups=False):
    """oracle/libdruid_cpu.so: the reference's per-segment GroupByV2 loop (LZ4 decode, hash grouping,
    merge by value, ordered result) in C -O3 -march=native over row chunks of the segments on
    `threads` host threads, on the whole workload. Merged-dictionary maps are built before timing (the
    GPU engine caches them too). want_groups: also return every merged group (key = (bucket index x
    card1 + merged id 1) << 32 | merged id 2, long sum, double sum) for the per-group comparison."""
    cs = _CpuSegments(paths)
    try:
        d1, d2 = query.dimensions
        (merged1, m1), (merged2, m2) = cs.merged(d1), cs.merged(d2)
        card1 = len(merged1)
        ptr1 = (ctypes.c_void_p * len(paths))(*[a.ctypes.data for a in m1])
        ptr2 = (ctypes.c_void_p * len(paths))(*[a.ctypes.data for a in m2])
        _, _, org, per, b0, nb = _query_buckets(query, cs.osegs)
        sums = (ctypes.c_double * 3)()
        rows = cs.rows
        out = None
        if want_groups:
            out = {"key": np.empty(rows, np.uint64), "lsum": np.empty(rows, np.int64), "dsum": np.empty(rows, np.float64)}
        ls, ds = query.aggregations[0].fieldName, query.aggregations[1].fieldName
        secs = ctypes.c_double()
        ng = cs.lib.cpu_groupby2(cs.handles, len(paths), d1.encode(), d2.encode(), ls.encode(), ds.encode(), ptr1, ptr2,
                                 card1, threads, org, per, b0, nb, sums, out["key"].ctypes.data if out else None, None,
                                 out["lsum"].ctypes.data if out else None, out["dsum"].ctypes.data if out else None,
                                 ctypes.byref(secs))
        if ng < 0:
            raise RuntimeError("cpu_groupby2 failed")
        el = secs.value
        gran = "ALL" if not per else f"{per} ms buckets"
        res = _baseline_line(rows / el, threads, "port",
                             f"the whole step workload: {len(paths)} segments x {rows // len(paths)} rows, GroupByV2 "
                             f"{d1} x {d2} ({gran}) longSum+doubleSum -> {ng} merged groups in {el:.2f} s "
                             f"(oracle/cpu_engine.c + druid_oracle.c, C -O3 -march=native, {threads} threads over 1M-row "
                             f"chunks, LZ4 decoded per block inside the timing)",
                             {"affinity_cores": len(os.sched_getaffinity(0)), "groups": int(ng)})
        if out is not None:
            for k in out:
                out[k] = out[k][:ng]
            res["_groups"] = out
            res["_dicts"] = [merged1, merged2]
            res["_buckets"] = (org, per, b0, card1)
        return res
    finally:
        cs.close()


def compare_groups(part, dicts, cpu):
    """Per-group equality of the GPU's merged result with the CPU engine's, over every group: the same
    dimension values in the same order, long sums bit-exact, double sums within 1e-9 relative."""
    g = cpu["_groups"]
    n = len(part)
    out = {"groups_equal": n == len(g["key"]), "dicts_equal": dicts == cpu["_dicts"]}
    if not (out["groups_equal"] and out["dicts_equal"]):
        out["per_group_equal"] = False
        return out
    org, per, b0, card1 = cpu["_buckets"]
    hi = part.codes[0].astype(np.uint64)
    if per:
        hi = ((part.times.astype(np.int64) - org) // per - b0).astype(np.uint64) * np.uint64(card1) + hi
    keys = (hi << np.uint64(32)) | part.codes[1].astype(np.uint64)
    out["keys_equal"] = bool(np.array_equal(keys, g["key"]))
    out["long_sums_equal"] = bool(np.array_equal(np.asarray(part.aggs[0], dtype=np.int64), g["lsum"]))
    a, b = np.asarray(part.aggs[1], dtype=np.float64), g["dsum"]
    rel = np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), 1e-300)
    rel[a == b] = 0.0
    out["double_max_rel_err"] = float(rel.max()) if n else 0.0
    out["doubles_within_1e-9"] = bool(out["double_max_rel_err"] <= 1e-9)
    out["per_group_equal"] = out["keys_equal"] and out["long_sums_equal"] and out["doubles_within_1e-9"]
    return out


def cpu_baseline_oracle(query, path, rows, seconds, selected_fraction):
    """Secondary configs: the oracle (scalar C + numpy restatement, one thread) on one segment."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    t0 = time.perf_counter()
    runs = 0
    while True:
        seg = O.OracleSegment(path)
        O.run(query, [seg])
        seg.close()
        runs += 1
        el = time.perf_counter() - t0
        if el >= seconds or runs >= 50:
            break
    return {"value": rows * selected_fraction * runs / el, "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": f"{runs} run(s) of the query over 1 segment x {rows} rows (oracle/ C+numpy restatement, "
                      f"single thread, decode included), {el:.1f} s; value = scanned rows/s x selectivity "
                      f"{selected_fraction:.4g}", "cpu_model": _cpu_model()}


# ------------------------------------------------------------------------------------------------
# N-rank result checks (world > 1): order-independent properties of the final, exchanged result against
# every rank's local CPU-engine result (GroupByMergingQueryRunnerV2.java:170-290, TimeseriesBinaryFn.java:
# 67-70, TopNBinaryFn.java:75-135), so the first multi-GPU run checks its own answer.
# ------------------------------------------------------------------------------------------------
SAMPLE_BITS = 10  # groups whose key hashes to 0 mod 2^SAMPLE_BITS are compared one by one


def sample_mask(t, c1, c2):
    """Deterministic 1-in-1024 sample of groupBy keys (bucket time, cluster id 1, cluster id 2)."""
    m = np.uint64
    h = (np.asarray(t).astype(np.int64).view(np.uint64) * m(0x9E3779B97F4A7C15)) ^ \
        (np.asarray(c1).astype(m) * m(0xC2B2AE3D27D4EB4F)) ^ (np.asarray(c2).astype(m) * m(0x165667B19E3779F9))
    h ^= h >> m(29)
    return (h & m((1 << SAMPLE_BITS) - 1)) == 0


def _lex_lt(a, b):
    return tuple(a) < tuple(b)


def rank_groupby_summary(final, cpu_groups, cpu_dicts, cpu_buckets, maps, local_dicts, universal, gpu_local_groups):
    """One rank's facts for evaluate_dist_groupby: `final` = this rank's key range of the exchanged result
    (times, cluster ids, [long sums, double sums]); cpu_groups = the CPU engine's groups over this rank's
    segments (key = (bucket * card1 + merged id 1) << 32 | merged id 2, lsum, dsum), re-keyed to cluster
    ids with the exchange's maps."""
    t, c1, c2 = (np.asarray(final["times"], np.int64), np.asarray(final["c1"], np.int64),
                 np.asarray(final["c2"], np.int64))
    ls, ds = np.asarray(final["lsum"], np.int64), np.asarray(final["dsum"], np.float64)
    n = len(t)
    srt = True
    if n > 1:  # strictly increasing (time, id1, id2)
        gt = np.zeros(n - 1, bool)
        eq = np.ones(n - 1, bool)
        for c in (t, c1, c2):
            gt |= eq & (c[1:] > c[:-1])
            eq &= c[1:] == c[:-1]
        srt = bool(gt.all())
    org, per, b0, card1 = cpu_buckets
    key = np.asarray(cpu_groups["key"], np.uint64)
    m2 = (key & np.uint64(0xFFFFFFFF)).astype(np.int64)
    hi = (key >> np.uint64(32)).astype(np.int64)
    m1, b = hi % card1, hi // card1
    ct = (org + (b0 + b) * per) if per else np.full(len(key), universal, np.int64)
    k1, k2 = maps[0][m1].astype(np.int64), maps[1][m2].astype(np.int64)
    gs, cs_ = sample_mask(t, c1, c2), sample_mask(ct, k1, k2)
    return {
        "n_final": n, "lsum_final": int(ls.sum()), "dsum_final": float(ds.sum()), "sorted_final": srt,
        "first": [int(t[0]), int(c1[0]), int(c2[0])] if n else None,
        "last": [int(t[-1]), int(c1[-1]), int(c2[-1])] if n else None,
        "gpu_local_groups": int(gpu_local_groups), "cpu_local_groups": int(len(key)),
        "cpu_lsum": int(np.asarray(cpu_groups["lsum"], np.int64).sum()),
        "cpu_dsum": float(np.asarray(cpu_groups["dsum"], np.float64).sum()),
        "dicts_equal": [list(d) for d in cpu_dicts] == [list(d) for d in local_dicts],
        "gpu_sample": [a[gs] for a in (t, c1, c2, ls, ds)],
        "cpu_sample": [ct[cs_], k1[cs_], k2[cs_], np.asarray(cpu_groups["lsum"], np.int64)[cs_],
                       np.asarray(cpu_groups["dsum"], np.float64)[cs_]],
    }


def evaluate_dist_groupby(summaries):
    """rank 0: the exchanged result against the ranks' CPU results. Exact: the long-sum total, each
    rank's pre-exchange group count, the ranges (each strictly increasing, rank r's last key below rank
    r + 1's first), the sampled groups one by one (keys, long sums); the total group count lies between
    the largest rank's and the sum of the ranks' counts; double sums within 1e-9 relative."""
    S = summaries
    groups = sum(x["n_final"] for x in S)
    cpu_counts = [x["cpu_local_groups"] for x in S]
    out = {"groups": groups, "ranks": len(S)}
    out["local_counts_equal"] = all(x["gpu_local_groups"] == x["cpu_local_groups"] for x in S)
    out["dicts_equal"] = all(x["dicts_equal"] for x in S)
    out["group_count_in_bounds"] = max(cpu_counts) <= groups <= sum(cpu_counts)
    wrap = lambda v: int(np.array([v % (1 << 64)], np.uint64).view(np.int64)[0])  # noqa: E731 (int64 sums wrap)
    out["long_sum"] = wrap(sum(x["lsum_final"] for x in S))
    out["long_sum_equal"] = out["long_sum"] == wrap(sum(x["cpu_lsum"] for x in S))
    dg, dc = sum(x["dsum_final"] for x in S), sum(x["cpu_dsum"] for x in S)
    out["double_sum_rel_err"] = abs(dg - dc) / max(abs(dg), abs(dc), 1e-300)
    out["double_sum_within_1e-9"] = out["double_sum_rel_err"] <= 1e-9
    out["ranges_sorted"] = all(x["sorted_final"] for x in S)
    ne = [x for x in S if x["n_final"]]
    out["ranges_disjoint_ascending"] = all(_lex_lt(a["last"], b["first"]) for a, b in zip(ne, ne[1:]))
    # sampled groups: CPU records of every rank combined by key (sources in rank order, as dg_merge)
    cat = [np.concatenate([np.asarray(x["cpu_sample"][i]) for x in S]) for i in range(5)]
    order = np.lexsort((cat[2], cat[1], cat[0]))
    t, c1, c2, ls, ds = (a[order] for a in cat)
    if len(t):
        new = np.ones(len(t), bool)
        new[1:] = (t[1:] != t[:-1]) | (c1[1:] != c1[:-1]) | (c2[1:] != c2[:-1])
        starts = np.flatnonzero(new)
        t, c1, c2 = t[starts], c1[starts], c2[starts]
        ls = np.add.reduceat(ls, starts)
        ds = np.add.reduceat(ds, starts)
    g = [np.concatenate([np.asarray(x["gpu_sample"][i]) for x in S]) for i in range(5)]
    out["sample_groups"] = int(len(g[0]))
    same = len(g[0]) == len(t) and all(np.array_equal(a, b) for a, b in zip(g[:3], (t, c1, c2)))
    out["sample_keys_equal"] = bool(same)
    out["sample_long_sums_equal"] = bool(same and np.array_equal(g[3], ls))
    rel = 0.0
    if same and len(t):
        a, b = g[4].astype(np.float64), ds
        r = np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), 1e-300)
        r[a == b] = 0.0
        rel = float(r.max())
    out["sample_double_max_rel_err"] = rel
    out["sample_equal"] = bool(same and out["sample_long_sums_equal"] and rel <= 1e-9)
    out["all_equal"] = all(out[k] for k in ("local_counts_equal", "dicts_equal", "group_count_in_bounds",
                                             "long_sum_equal", "double_sum_within_1e-9", "ranges_sorted",
                                             "ranges_disjoint_ascending", "sample_equal"))
    return out


def pmc_traffic(args, kname):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes of this same bench
    command (bench_pmc/pmc_<config>.json, written by tools/prof_summary.py from separate FETCH_SIZE and
    WRITE_SIZE rocprofv3 runs). FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM: gfx950 tallies a
    wide streaming read's 128-B requests at 64 B; the decoders stage their blocks with 16-B loads);
    the raw value is kept beside it. (bench_pmc/ travels with the tree to the GPU box; profiles/ does not.)"""
    f = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_pmc", f"pmc_{args.config}.json")
    if not os.path.exists(f):
        return {}
    pm = json.load(open(f))
    ks = match_kernels(pm["kernels"], kname)
    if not ks:
        return {}
    # a spec of several kernels ("a+b", "prefix*") is one logical launch of each: per launch, the kernels'
    # bytes and times add up (every kernel of such a spec launches as often as the others)
    K = pm["kernels"]
    calls = max(K[k]["calls"] for k in ks)
    fetch = sum(K[k]["fetch_bytes"] for k in ks) / calls
    write = sum(K[k]["write_bytes"] for k in ks) / calls
    tcalls = max(K[k].get("trace_calls", K[k]["calls"]) for k in ks)
    avg_ns = sum(K[k]["avg_ns"] * K[k].get("trace_calls", K[k]["calls"]) for k in ks) / max(tcalls, 1)
    return {"traffic": 2 * fetch + write, "traffic_fetch_raw": fetch, "traffic_write": write,
            "rocprof_avg_launch_ms": avg_ns / 1e6, "rocprof_kernels": sorted(k.split("(")[0] for k in ks),
            "traffic_source": os.path.join("bench_pmc", os.path.basename(f)) + f" ({pm.get('label', '')})"}


def match_kernels(kernels, kname):
    """Profiled kernel names (demangled, e.g. "void dg::k_lz4_decode_flow<false>(...)") of a roofline
    kernel spec "a+b": each part is an exact kernel name (any template arguments), or a prefix when it
    ends in "*"."""
    out = []
    for k in kernels:
        base = k.split("(")[0].split("<")[0].split("::")[-1]
        for n in kname.split("+"):
            n = n.strip()
            if (n.endswith("*") and base.startswith(n[:-1])) or base == n:
                out.append(k)
                break
    return out


def device_probes(NAT, device, line):
    """What this GPU and its host link deliver to plain kernels and copies (dg_debug_probe, HIP events;
    after the timed region): a 2 GiB read + 2 GiB write stream copy (the measured HBM ceiling, SURVEY
    §8(d)), 1 GiB DMA copies each way and zero-copy kernel writes into pinned host memory (the groupBy
    fetch path), and for a groupBy line the reduce's memory floor — one ordered 8-byte word, one 16-byte
    record gathered at a pseudo-random row and four ordered 8-byte stores per element, for as many
    elements as the step's selected rows. The roofline line gets its kernel's fraction of the measured
    copy bandwidth next to the fraction of the 8 TB/s spec."""
    L = NAT.lib()

    def probe(kind, n, iters):
        ms = ctypes.c_double()
        NAT.check(L.dg_debug_probe(device, kind, int(n), iters, ctypes.byref(ms)))
        return ms.value

    out = {}
    gib = 1 << 30
    ms = probe(0, 2 * gib, 20)
    out["copy_gb_s"] = 2 * 2 * gib / (ms / 1e3) / 1e9  # bytes read + written
    for name, kind in (("d2h_gb_s", 1), ("h2d_gb_s", 2), ("zero_copy_write_gb_s", 4)):
        out[name] = gib / (probe(kind, gib, 5) / 1e3) / 1e9
    rf = line.get("roofline") or {}
    if rf.get("achieved"):
        rf["measured_copy_gb_s"] = out["copy_gb_s"]
        rf["frac_of_measured_copy"] = rf["achieved"] / out["copy_gb_s"]
    if line.get("groups_per_step"):
        n = int(line["selected_rows_per_step"] / max(line["n_gpus"], 1))
        if 0 < n < (1 << 32):
            g = probe(3, n, 5)
            red = line["phases_ms"].get("reduce_kernels")
            out["reduce_floor"] = {"elements": n, "gather_floor_ms": g, "reduce_kernels_ms": red,
                                   "reduce_over_floor": red / g if red else None,
                                   "floor": "per element: 8 B ordered read, 16 B record gathered at a pseudo-random "
                                            "row, 4 x 8 B ordered writes (k_gb_reduce's loads and stores alone)"}
    if line.get("pcie_fetch"):
        pf = line["pcie_fetch"]
        pf["link_d2h_gb_s"] = out["d2h_gb_s"]
        pf["link_zero_copy_write_gb_s"] = out["zero_copy_write_gb_s"]
    return out


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, argv, script=None) -> int:
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start N child processes of this
    script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), the way
    ChainedExecutionQueryRunner.java:89-180 fans segment runners out over the processing pool. The
    parent never touches the GPU and never execs: it waits for the ranks, rank 0 prints the JSON line
    (stdout is inherited), and the first failing rank stops the others and sets the exit code."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.2)
    return rc


def rank_env(args):
    """(world, rank, local_rank) of this process. Under a launcher (WORLD_SIZE set, e.g.
    torch.distributed.run) the world must be --gpus; without one, --gpus 1 is the single process."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus != 1:
            raise SystemExit("rank_env: --gpus > 1 needs the ranks started by launch_ranks")
        return 1, 0, 0
    if int(world) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    return int(world), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="groupby", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--segments", type=int, default=None)
    ap.add_argument("--compression", default="lz4", choices=["lz4", "lzf", "uncompressed", "none"])
    ap.add_argument("--bitmap", default="concise", choices=["concise", "roaring"])
    ap.add_argument("--lz4-mode", default="hc", choices=["hc", "fast"])
    ap.add_argument("--long-encoding", default="longs", choices=["longs", "auto"],
                    help="IndexSpec longEncoding of the written segments (auto: DELTA / TABLE / LONGS per column)")
    ap.add_argument("--data-dir", default=os.environ.get("DRUID_AMD_BENCH_DATA", "/tmp/druid_amd_bench"))
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-result-checks", action="store_true", help="N ranks: skip the CPU-engine result checks")
    ap.add_argument("--no-probes", action="store_true", help="skip the device copy / link / gather probes")
    ap.add_argument("--write-workers", type=int, default=8, help="processes writing the synthetic segments")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))  # before torch or the engine is imported
    world, rank, local_rank = rank_env(args)

    Q = importlib.import_module("incubator-druid_amd.query")
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")
    NAT = importlib.import_module("incubator-druid_amd._native")

    dist = None
    if world > 1:
        D = importlib.import_module("incubator-druid_amd.distributed")
        dist = D.init_from_env()

    rows_per, nseg, desc, cols = CONFIGS[args.config]
    rows_per = args.rows or rows_per
    nseg = args.segments or nseg
    paths = ensure_segments(args.data_dir, rank, nseg, rows_per, args.compression, args.bitmap, args.lz4_mode, cols,
                            partitioned=args.config in ("ts_hourly", "groupby_hourly"), workers=args.write_workers,
                            long_encoding=args.long_encoding)
    device = D.device_index() if world > 1 else local_rank
    segs = [S.GpuSegment(p, device=device) for p in paths]
    query = make_query(Q, args.config)

    gdict = None
    if dist is not None and args.config.startswith("topn"):
        gdict = D.GlobalDictionary.build(dist, [s.dictionary(query.dimension) for s in segs])
        translations = [gdict.translate(s.dictionary(query.dimension)) for s in segs]
    gmerge = None
    if dist is not None and isinstance(query, Q.GroupByQuery):
        gmerge = D.GroupByExchange(dist, query, segs)  # cluster-wide dictionaries + maps, built once

    ts_buckets = None  # cluster-wide bucket keys of a timeseries query (identical on every rank), once
    if dist is not None and isinstance(query, Q.TimeseriesQuery):
        local = R.merge_timeseries(query, R.timeseries_per_segment(segs, query, R.RunStats()))
        mine = sorted({0 if query.granularity.is_all else query.granularity.bucket_start(r.timestamp) for r in local})
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        ts_buckets = sorted({b for g in gathered for b in g})

    def step(stats):
        if isinstance(query, Q.TopNQuery):
            if dist is None:
                return R.run_topn(segs, query, stats)
            return D.gather_topn(dist, query, R.topn_raw(segs, query, stats), gdict, translations, segs)
        if isinstance(query, Q.TimeseriesQuery):
            if dist is None:
                # QueryRunnerFactory.mergeRunners: one engine call, the buckets folded natively
                # (dg_timeseries_merge) — not the per-segment lists merged in Python
                return R.run_query(query, segs, stats)
            per = R.timeseries_per_segment(segs, query, stats)
            res = R.merge_timeseries(query, per)
            return D.allreduce_timeseries(dist, query, res, ts_buckets)
        res = R.groupby_run(segs, query, stats)  # merged, ordered groups in HBM
        if dist is not None:
            merged = gmerge.exchange(res)  # this rank's key range of the cluster-wide result, in HBM
            res.release()
            res = merged
        n = res.groups
        res.release()
        return n

    import torch
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    first_ms = None
    for w in range(args.warmup):
        t_w = time.perf_counter()
        step(R.RunStats())
        if w == 0:  # the first call: cold caches, and a topN's one-time build of the dimension's bin index
            sync()
            first_ms = (time.perf_counter() - t_w) * 1e3
    # the timed steps carry no phase timestamps (dg_set_phase_timing: ~25 us of a configs[0] query);
    # the phase times come from PHASE_STEPS untimed steps after them
    NAT.lib().dg_set_phase_timing(0)
    stats = R.RunStats()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        result = step(stats)
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    NAT.lib().dg_set_phase_timing(1)
    pstats = R.RunStats()
    psteps = min(PHASE_STEPS, args.steps)
    for _ in range(psteps):
        step(pstats)
    sync()

    steps = args.steps
    calls = [c for c in stats.calls if c["segment_rows"] > 0]
    pcalls = [c for c in pstats.calls if c["segment_rows"] > 0]
    # counts and bytes from the timed steps; phase times (GPU timestamps) from the untimed phase steps
    per_step = lambda k: (sum(c[k] for c in pcalls) / psteps if k.endswith("_ms") and k != "total_ms"  # noqa: E731
                          else sum(c[k] for c in calls) / steps)
    selected_local = per_step("selected_rows")
    scanned_local = sum(s.num_rows for s in segs)
    selected_all, scanned_all = selected_local, scanned_local
    if dist is not None:  # the rows every rank actually aggregated (not this rank's count x world)
        t = torch.tensor([selected_local, float(scanned_local)], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t)
        selected_all, scanned_all = float(t[0].item()), float(t[1].item())
    value = selected_all * steps / elapsed
    phases = {"bitmap": per_step("bitmap_ms"), "decode": per_step("decode_ms"), "aggregate": per_step("aggregate_ms"),
              "query_wall": per_step("total_ms")}
    bytes_read = per_step("bytes_read")
    bytes_side = per_step("bytes_side")
    kernels = {}  # phase -> (kernel, algorithmic bytes per launch, launches per step, ms per step)
    dk = "k_lzf_decode" if args.compression == "lzf" else "k_lz4_light+k_lz4_decode"
    if phases["decode"] > 0:
        # LZ4: the light decoder (literal-heavy blocks) and the general one, both inside the phase
        kernels["decode"] = (dk if args.long_encoding == "longs" else dk + "+k_vsize_expand", bytes_read - bytes_side, 1,
                             phases["decode"])
    if per_step("decode_side_ms") > 0:
        # groupBy payload columns decoded in place on the side stream (overlapping keygen + sort)
        phases["decode_payload_side"] = per_step("decode_side_ms")
        kernels["decode_payload_side"] = (dk + " (payload, side stream)", bytes_side, 1, phases["decode_payload_side"])
    if per_step("lz4_general_ms") > 0:
        # the general LZ4 decoder alone (token-dense blocks of 8-byte value runs; main and side stream): its
        # own HIP-event span per stream, its blocks' stored bytes; a "launch" is one kernel launch, as
        # rocprofv3 counts
        # (the phase: the wall time it ran on either stream; the roofline below: per launch)
        phases["lz4_general"] = per_step("lz4_general_wall_ms")
        fb, gb = per_step("lz4_flow_blocks"), per_step("lz4_general_blocks")
        gname = "k_lz4_decode_flow" if fb >= gb else "k_lz4_decode" if fb == 0 else "k_lz4_decode+k_lz4_decode_flow"
        kernels["lz4_general"] = (gname, per_step("lz4_general_bytes"),
                                  max(per_step("lz4_general_launches"), 1.0), per_step("lz4_general_ms"))
    # LZ4 blocks per step by decoder (and those whose decode was fused with their aggregator)
    lz4_blocks = {"general": per_step("lz4_general_blocks"), "fused": per_step("lz4_fused_blocks")}
    if isinstance(query, Q.GroupByQuery):
        phases.update({"keygen": per_step("keygen_ms"), "sort": per_step("sort_ms"), "reduce": per_step("reduce_ms"),
                       "reduce_kernels": per_step("reduce_kernel_ms")})
        passes = max(1, int(round(per_step("sort_passes"))))
        n_sel = selected_local
        groups = per_step("groups")
        # the first pass's digit totals read every packed [key | row ref] word once (k_rs_hist0); every
        # one-sweep pass reads and writes it once (k_rs_scatter): 8 + 16 x passes B per selected row
        # the roofline kernel is one pass's scatter (passes launches per step); the first pass's digit totals
        # (k_rs_hist0, one read of the words) are inside the phase
        kernels["sort"] = ("k_rs_scatter", n_sel * 16.0 * passes, passes, phases["sort"])
        # keygen: the two 3-byte ids of the row in, its 8-byte sort word out
        kernels["keygen"] = ("k_gb_keygen", n_sel * (3 + 3 + 8), 1, phases["keygen"])
        # reduce (its kernels alone): the sorted words and the payload records in, per group its key and
        # (1 + aggregators) 8-byte slots out
        pw = len(query.aggregations)
        # (k_gb_carry / k_gb_open_finalize, a few us per step, are inside the phase but not the roofline kernel)
        kernels["reduce"] = ("k_gb_reduce", n_sel * (8.0 + 8.0 * pw) + groups * 8.0 * (2 + pw), 1, phases["reduce_kernels"])
    elif phases["aggregate"] > 0:
        if args.config.startswith("topn") and os.environ.get("DG_NO_TOPN_INDEX", "0") in ("", "0"):
            # topN by the dimension's bin index: per row its index entry (4-B row + 2-B id bits) and
            # its metric columns' 8-byte values (longSum + doubleSum; the dimension-ordered lines: longSum)
            kname, per_row = "k_topn_ix_reduce", 6 + (16 if args.config == "topn" else 8)
        elif args.config.startswith("topn"):  # (DG_NO_TOPN_INDEX=1: the per-call bins, the 3-byte id read)
            kname, per_row = "k_topn_bin_*", 3 + (16 if args.config == "topn" else 8)
        else:
            kname, per_row = "k_scan_agg", 8
        kernels["aggregate"] = (kname, scanned_local * per_row, 1, phases["aggregate"])
    if phases["bitmap"] > 0:
        # serialized bitmap bytes of the matched values + every row bitset written and read once
        kernels["bitmap"] = ("k_concise_or+k_filter_eval" if args.bitmap == "concise" else "k_roaring_or+k_filter_eval",
                             per_step("bitmap_bytes") or None, 1, phases["bitmap"])
    # the dominant kernel: the longest single-kernel span (phases that group several kernels, like the
    # decode phase or the side-stream payload decode, are reported in phases_ms)
    single = {k: v for k, v in kernels.items()
              if k in ("lz4_general", "aggregate", "bitmap", "sort", "keygen", "reduce")}

    def step_ms(k):
        # the kernel's own time per step: its rocprofv3 average x launches per step when the committed
        # profile of this command has it (a phase's HIP-event span also holds its helper kernels and
        # memsets: the sort phase holds k_rs_hist0), else the phase's HIP-event time
        kname, _, launches, kms = (single or kernels)[k]
        avg = pmc_traffic(args, kname).get("rocprof_avg_launch_ms")
        return avg * launches if avg else kms
    dom = max(single or kernels, key=step_ms) if kernels else None
    roofline = None
    if dom is not None:
        kname, kbytes, launches, kms = kernels[dom]
        per_launch_ms = kms / launches
        bpl = kbytes / launches if kbytes else None
        roofline = {"bound": "hbm", "kernel": kname, "phase": dom, "achieved": None, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": None, "traffic": None, "bytes_per_launch": bpl,
                    "hip_event_avg_launch_ms": per_launch_ms, "launches_per_step": launches,
                    "dominant_by": "kernel ms per step (rocprofv3 average x launches when profiled, else HIP events)",
                    "kernel_ms_per_step": {k: round(step_ms(k), 4) for k in (single or kernels)}}
        roofline.update(pmc_traffic(args, kname))
        # achieved = algorithmic bytes per launch / average launch time: the rocprofv3 average of the
        # committed profile of this command when there is one (bench_pmc/, the figure a reader recomputes
        # from profiles/), else this run's HIP-event span; both are reported
        prof_ms = roofline.get("rocprof_avg_launch_ms")
        avg_ms = prof_ms if prof_ms else per_launch_ms
        roofline["avg_launch_ms"] = avg_ms
        roofline["avg_launch_source"] = "rocprofv3 kernel trace (traffic_source)" if prof_ms else "HIP events, this run"
        if bpl:
            roofline["achieved"] = bpl / (avg_ms / 1e3) / 1e9
            roofline["frac"] = roofline["achieved"] / HBM_PEAK_GBS
            roofline["achieved_hip_events"] = bpl / (per_launch_ms / 1e3) / 1e9
            roofline["frac_hip_events"] = roofline["achieved_hip_events"] / HBM_PEAK_GBS
    line = {
        "metric": "filtered rows aggregated/sec",
        "value": value,
        "unit": "rows/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64/f64",
        "data": "synthetic (basic schema columns, seeded numpy generator, written as Druid v9 segments)",
        "config": {"workload": desc, "config": args.config, "rows_per_segment": rows_per, "segments_per_gpu": nseg,
                   "compression": args.compression, "lz4_mode": args.lz4_mode, "bitmap": args.bitmap,
                   "long_encoding": args.long_encoding,
                   "parallelism": f"segments sharded over {world} GPU(s)"},
        "roofline": roofline,
        "phases_ms": phases,
        "phases_source": f"{psteps} untimed steps after the timed ones, with phase timestamps (dg_set_phase_timing); "
                         "the timed steps run without them",
        "selected_rows_per_step": selected_all,
        "scanned_rows_per_s": scanned_all * steps / elapsed,
        "stored_bytes_per_step": bytes_read,
        "lz4_blocks_per_step": lz4_blocks,
        "rows_scanned_per_step": scanned_all,
        "first_step_ms": first_ms,
    }
    if args.config.startswith("topn") and kernels.get("aggregate", ("",))[0] == "k_topn_ix_reduce":
        line["topn_index"] = ("the dimension's rows grouped by dictionary-id bin (the row sets of Druid's per-value "
                              "bitmap index), built on the device by the first topN over the column (the first "
                              "warm-up step, first_step_ms) and kept with the segment; every step still decodes "
                              "and aggregates every metric input")
    if isinstance(query, Q.GroupByQuery):
        line["groups_per_step"] = per_step("groups")
    part = dicts = None
    if isinstance(query, Q.GroupByQuery) and dist is None:
        # the merged result, fetched to the host once (PCIe-inclusive; not part of `value`), and checked.
        # The destination is pinned host memory allocated once before the timing (the shim's direct
        # ByteBuffers, like the processing pool's startup allocation): the columns land by DMA.
        per_group = 4 * len(query.dimensions) + 8 * len(query.aggregations) + (0 if query.granularity.is_all else 8)
        pool = R.PinnedPool(int(line["groups_per_step"]) * per_group + (1 << 20))
        t1 = time.perf_counter()
        res = R.groupby_run(segs, query)
        t2 = time.perf_counter()
        dicts = [res.dictionary(d) for d in range(len(query.dimensions))]  # (host: the values as Python strings)
        res._dicts = dicts
        t2b = time.perf_counter()
        part = res.fetch(pool=pool)  # dg_result_fetch_groups: the pack kernel writes the pinned columns
        t3 = time.perf_counter()
        fetch_s = t3 - t1
        res.release()
        line["pcie_fetch"] = {"groups": len(part), "query_plus_fetch_ms": fetch_s * 1e3, "fetch_ms": (t3 - t2b) * 1e3,
                              "dictionary_ms": (t2b - t2) * 1e3,
                              "bytes_fetched": len(part) * per_group,
                              "fetch_gb_s": len(part) * per_group / max(t3 - t2b, 1e-9) / 1e9,
                              "rows_per_s_incl_fetch": scanned_local / fetch_s,
                              "destination": "pinned host memory (dg_host_alloc, allocated before the timing), "
                                             "written by the pack kernel over the link (zero-copy)",
                              "split": "fetch_ms = dg_result_fetch_groups (+ numpy views); dictionary_ms = the "
                                       "merged dictionaries' values materialised as host strings"}
        # result order: bucket time, then each dimension's merged id, strictly increasing
        gt = np.zeros(max(len(part) - 1, 0), dtype=bool)
        eq = np.ones(max(len(part) - 1, 0), dtype=bool)
        for c in [part.times] + list(part.codes):
            gt |= eq & (c[1:] > c[:-1])
            eq &= c[1:] == c[:-1]
        line["result_checks"] = {"groups": len(part),
                                 "long_sum": int(np.sum(np.asarray(part.aggs[0], dtype=np.int64))),
                                 "double_sum": float(np.sum(part.aggs[1], dtype=np.float64)),
                                 "sorted": bool(gt.all())}
        del gt, eq
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the CPU baseline on the box's usable cores, and the result of the benched query checked
        # against it (or against the oracle) after the timed loop
        threads = _cpu_threads()
        if isinstance(query, Q.GroupByQuery):
            cb = cpu_baseline_groupby(paths, query, threads, want_groups=part is not None)
            if part is not None:
                rc = line["result_checks"]
                rc.update(compare_groups(part, dicts, cb))
                rc["cpu_long_sum"] = int(np.sum(cb["_groups"]["lsum"]))
                rc["cpu_long_sum_equal"] = rc["cpu_long_sum"] == rc["long_sum"]
            for k in ("_groups", "_dicts", "_buckets"):
                cb.pop(k, None)
            line["cpu_baseline"] = cb
        elif isinstance(query, Q.TimeseriesQuery):
            gpu_res = step(R.RunStats())
            cb, cres = cpu_baseline_timeseries(paths, query, threads)
            line["cpu_baseline"] = cb
            line["result_checks"] = check_timeseries(gpu_res, cres, query)
        elif isinstance(query, Q.TopNQuery):
            gpu_res = step(R.RunStats())
            cb, cres = cpu_baseline_topn(paths, query, threads)
            line["cpu_baseline"] = cb
            line["result_checks"] = check_topn(gpu_res, cres, query)
    if dist is not None and not args.no_result_checks:
        # N ranks: the final result checked against every rank's CPU-engine result (after the timing; one
        # process per GPU, so the host cores are split between the node's ranks)
        threads = max(1, _cpu_threads() // int(os.environ.get("LOCAL_WORLD_SIZE", world)))
        t_chk = time.perf_counter()
        if isinstance(query, Q.GroupByQuery) and len(query.dimensions) == 2 and len(query.aggregations) == 2:
            res = R.groupby_run(segs, query)
            gpu_local = res.groups
            merged = gmerge.exchange(res)
            res.release()
            fp = merged.fetch()
            merged.release()
            final = {"times": np.broadcast_to(fp.times, (len(fp),)), "c1": fp.codes[0], "c2": fp.codes[1],
                     "lsum": fp.aggs[0], "dsum": fp.aggs[1]}
            cb = cpu_baseline_groupby(paths, query, threads, want_groups=True)
            summ = rank_groupby_summary(final, cb["_groups"], cb["_dicts"], cb["_buckets"], gmerge.maps, gmerge.local,
                                        query.interval[0], gpu_local)
            del fp, final, cb
            gathered = [None] * world
            dist.all_gather_object(gathered, summ)
            if rank == 0:
                line["result_checks"] = evaluate_dist_groupby(gathered)
            del gathered, summ
        elif isinstance(query, Q.TimeseriesQuery):
            gpu_res = step(R.RunStats())  # (all-reduced on every rank)
            _, cres = cpu_baseline_timeseries(paths, query, threads)
            local = [Q.Result(ts, {a.name: v for a, v in zip(query.aggregations, vals)}) for ts, (_, vals) in cres.items()]
            red = D.allreduce_timeseries(dist, query, local, ts_buckets)
            cdict = {r.timestamp: (0, [r.value[a.name] for a in query.aggregations]) for r in red}
            line["result_checks"] = dict(check_timeseries(gpu_res, cdict, query),
                                         against="every rank's CPU engine result, all-reduced")
        elif isinstance(query, Q.TopNQuery):
            allp = [None] * world
            dist.all_gather_object(allp, paths)
            gpu_res = step(R.RunStats())  # (rank 0 holds the folded result)
            if rank == 0:  # the CPU engine over every rank's segments (one node: their files are here)
                _, cres = cpu_baseline_topn([p for g in allp for p in g], query, _cpu_threads())
                line["result_checks"] = dict(check_topn(gpu_res, cres, query),
                                             against="the CPU engine over every rank's segments, rank-major")
        if rank == 0 and "result_checks" in line:
            line["result_checks"]["check_s"] = time.perf_counter() - t_chk
    del part
    if isinstance(query, Q.GroupByQuery) and dist is None:
        pool.close()
    if rank == 0 and not args.no_probes:
        line["device_probes"] = device_probes(NAT, device, line)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
