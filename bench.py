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
    """Every core this process may run on (sched_getaffinity), as SURVEY §8(d) asks for."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return max(1, os.cpu_count() or 1)


def _cpu_quota():
    """The cgroup CPU quota in cores (cpu.max), or None when unlimited / unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def cpu_baseline_groupby(paths, query, threads, want_groups=False):
    """oracle/libdruid_cpu.so: the reference's per-segment GroupByV2 loop (LZ4 decode, hash grouping,
    merge by value, ordered result) in C -O3 -march=native over row chunks of the segments on
    `threads` host threads, on the whole workload. Merged-dictionary maps are built before timing (the
    GPU engine caches them too). want_groups: also return every merged group (key = merged id 1 << 32
    | merged id 2, long sum, double sum) for the per-group comparison with the GPU result."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "libdruid_cpu.so"))
    lib.cpu_groupby2.restype = ctypes.c_int64
    vp = ctypes.c_void_p
    lib.cpu_groupby2.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p,
                                 ctypes.c_char_p, ctypes.c_char_p, vp, vp, ctypes.c_int32,
                                 ctypes.c_int, ctypes.POINTER(ctypes.c_double), vp, vp, vp, vp,
                                 ctypes.POINTER(ctypes.c_double)]
    segs = [O.OracleSegment(p) for p in paths]
    d1, d2 = query.dimensions
    maps, merged_dicts = [], []
    for dim in (d1, d2):
        dicts = [s.dictionary(dim) for s in segs]
        merged = sorted(set().union(*map(set, dicts)), key=lambda v: (v is not None, (v or "").encode("utf-16-be")))
        index = {v: i for i, v in enumerate(merged)}
        maps.append(([np.array([index[v] for v in dd], dtype=np.int32) for dd in dicts], len(merged)))
        merged_dicts.append(merged)
    (m1, card1), (m2, _) = maps
    ptr1 = (vp * len(segs))(*[a.ctypes.data for a in m1])
    ptr2 = (vp * len(segs))(*[a.ctypes.data for a in m2])
    lib.or_open.restype = vp
    lib.or_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    lib.or_close.argtypes = [vp]
    err = ctypes.create_string_buffer(512)
    hs = [lib.or_open(p.encode(), err, 512) for p in paths]  # the engine library's own segment readers
    if not all(hs):
        raise IOError(err.value.decode())
    handles = (vp * len(segs))(*hs)
    sums = (ctypes.c_double * 3)()
    rows = sum(s.num_rows for s in segs)
    out = None
    if want_groups:
        out = {"key": np.empty(rows, np.uint64), "lsum": np.empty(rows, np.int64), "dsum": np.empty(rows, np.float64)}
    ls, ds = query.aggregations[0].fieldName, query.aggregations[1].fieldName
    secs = ctypes.c_double()
    t0 = time.perf_counter()
    ng = lib.cpu_groupby2(handles, len(segs), d1.encode(), d2.encode(), ls.encode(), ds.encode(), ptr1, ptr2, card1,
                          threads, sums, out["key"].ctypes.data if out else None, None,
                          out["lsum"].ctypes.data if out else None, out["dsum"].ctypes.data if out else None,
                          ctypes.byref(secs))
    if ng < 0:
        raise RuntimeError("cpu_groupby2 failed")
    el = secs.value if secs.value > 0 else time.perf_counter() - t0
    for s, h in zip(segs, hs):
        s.close()
        lib.or_close(h)
    quota = _cpu_quota()
    res = {"value": rows / el, "unit": "rows/s", "cores": threads, "kind": "port",
           "sample": f"the whole step workload: {len(paths)} segments x {rows // len(paths)} rows, GroupByV2 "
                     f"{d1} x {d2} longSum+doubleSum -> {ng} merged groups in {el:.2f} s "
                     f"(oracle/cpu_engine.c + druid_oracle.c, C -O3 -march=native, {threads} threads over 1M-row "
                     f"chunks, LZ4 decoded per block inside the timing)",
           "cpu_model": _cpu_model(), "nproc": os.cpu_count(), "affinity_cores": threads,
           "cgroup_quota_cores": quota, "groups": int(ng)}
    if out is not None:
        for k in out:
            out[k] = out[k][:ng]
        res["_groups"] = out
        res["_dicts"] = merged_dicts
    return res


def compare_groups(part, dicts, cpu):
    """Per-group equality of the GPU's merged result with the CPU engine's, over every group: the same
    dimension values in the same order, long sums bit-exact, double sums within 1e-9 relative."""
    g = cpu["_groups"]
    n = len(part)
    out = {"groups_equal": n == len(g["key"]), "dicts_equal": dicts == cpu["_dicts"]}
    if not (out["groups_equal"] and out["dicts_equal"]):
        out["per_group_equal"] = False
        return out
    keys = (part.codes[0].astype(np.uint64) << np.uint64(32)) | part.codes[1].astype(np.uint64)
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
    # kernel names as "a+b", each a prefix of the demangled name (after the namespace) or "prefix*"
    names = [n.rstrip("*") for n in kname.split("+")]
    ks = [k for k in pm["kernels"] if any(k.startswith(n) or f"::{n}" in k for n in names)]
    if not ks:
        return {}
    calls = sum(pm["kernels"][k]["calls"] for k in ks)
    fetch = sum(pm["kernels"][k]["fetch_bytes"] for k in ks) / calls
    write = sum(pm["kernels"][k]["write_bytes"] for k in ks) / calls
    return {"traffic": 2 * fetch + write, "traffic_fetch_raw": fetch, "traffic_write": write,
            "traffic_source": os.path.join("bench_pmc", os.path.basename(f)) + f" ({pm.get('label', '')})"}


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
    ap.add_argument("--write-workers", type=int, default=8, help="processes writing the synthetic segments")
    args = ap.parse_args()

    Q = importlib.import_module("incubator-druid_amd.query")
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
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
    segs = [S.GpuSegment(p, device=local_rank) for p in paths]
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
            per = R.timeseries_per_segment(segs, query, stats)
            res = R.merge_timeseries(query, per)
            if dist is None:
                return res
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
    for _ in range(args.warmup):
        step(R.RunStats())
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

    steps = args.steps
    calls = [c for c in stats.calls if c["segment_rows"] > 0]
    per_step = lambda k: sum(c[k] for c in calls) / steps  # noqa: E731
    selected_local = per_step("selected_rows")
    scanned_local = sum(s.num_rows for s in segs)
    value = selected_local * world * steps / elapsed  # every rank holds the same shape of data (weak scaling)
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
        # the general LZ4 decoder alone (token-dense blocks; main and side stream): its own HIP-event span
        # per stream, its blocks' stored bytes; a "launch" here is one kernel launch, as rocprofv3 counts
        phases["lz4_general"] = per_step("lz4_general_ms")
        kernels["lz4_general"] = ("k_lz4_decode", per_step("lz4_general_bytes"),
                                  max(per_step("lz4_general_launches"), 1.0), phases["lz4_general"])
    if isinstance(query, Q.GroupByQuery):
        phases.update({"keygen": per_step("keygen_ms"), "sort": per_step("sort_ms"), "reduce": per_step("reduce_ms")})
        passes = max(1, int(round(per_step("sort_passes"))))
        n_sel = selected_local
        # one radix pass: the histogram reads every packed [key | row ref] word, the scatter reads and
        # writes it once: 3 x 8 B per selected row
        kernels["sort"] = ("k_rs_hist+k_rs_binscan+k_rs_scatter", 24.0 * n_sel, passes, phases["sort"])
        kernels["keygen"] = ("k_gb_count+k_gb_keygen", n_sel * (3 + 3 + 12), 1, phases["keygen"])
    elif phases["aggregate"] > 0:
        per_row = {"topn": 3 + 8 + 8}.get(args.config, 8)
        kernels["aggregate"] = ("k_topn_bin_*" if args.config.startswith("topn") else "k_scan_agg",
                                scanned_local * per_row, 1, phases["aggregate"])
    if phases["bitmap"] > 0:
        # serialized bitmap bytes of the matched values + every row bitset written and read once
        kernels["bitmap"] = ("k_concise_or+k_filter_eval" if args.bitmap == "concise" else "k_roaring_or+k_filter_eval",
                             per_step("bitmap_bytes") or None, 1, phases["bitmap"])
    # the dominant kernel: the longest single-kernel span (phases that group several kernels, like the
    # decode phase or the side-stream payload decode, are reported in phases_ms)
    single = {k: v for k, v in kernels.items() if k in ("lz4_general", "aggregate", "bitmap", "sort", "keygen")}
    dom = max(single or kernels, key=lambda k: (single or kernels)[k][3]) if kernels else None
    roofline = None
    if dom is not None:
        kname, kbytes, launches, kms = kernels[dom]
        per_launch_ms = kms / launches
        achieved = (kbytes / launches) / (per_launch_ms / 1e3) / 1e9 if kbytes else None
        roofline = {"bound": "hbm", "kernel": kname, "phase": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": None,
                    "bytes_per_launch": kbytes / launches if kbytes else None, "avg_launch_ms": per_launch_ms,
                    "launches_per_step": launches}
        roofline.update(pmc_traffic(args, kname))
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
        "stored_bytes_per_step": bytes_read,
        "rows_scanned_per_step": scanned_local * world,
    }
    if isinstance(query, Q.GroupByQuery):
        line["groups_per_step"] = per_step("groups")
    part = dicts = None
    if isinstance(query, Q.GroupByQuery) and dist is None:
        # the merged result, fetched to the host once (PCIe-inclusive; not part of `value`), and checked
        t1 = time.perf_counter()
        res = R.groupby_run(segs, query)
        part = res.fetch()
        fetch_s = time.perf_counter() - t1
        dicts = [res.dictionary(d) for d in range(len(query.dimensions))]
        res.release()
        line["pcie_fetch"] = {"groups": len(part), "query_plus_fetch_ms": fetch_s * 1e3,
                              "rows_per_s_incl_fetch": scanned_local / fetch_s}
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
        if args.config == "groupby":
            cb = cpu_baseline_groupby(paths, query, _cpu_threads(), want_groups=part is not None)
            if part is not None:
                rc = line["result_checks"]
                rc.update(compare_groups(part, dicts, cb))
                rc["cpu_long_sum"] = int(np.sum(cb["_groups"]["lsum"]))
                rc["cpu_long_sum_equal"] = rc["cpu_long_sum"] == rc["long_sum"]
            cb.pop("_groups", None)
            cb.pop("_dicts", None)
            line["cpu_baseline"] = cb
        else:
            line["cpu_baseline"] = cpu_baseline_oracle(query, paths[0], rows_per, args.cpu_seconds,
                                                       selected_local / scanned_local if scanned_local else 1.0)
    del part
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
