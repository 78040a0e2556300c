"""Benchmark: filtered rows aggregated per second (+ HBM GB/s vs the MI355X roofline).

Default workload = BASELINE.json configs[1]: TopNBenchmark 'basic' schema, topN over dimUniform
(threshold 10, metric sumFloatNormal, aggregators longSum(sumLongSequential) +
doubleSum(sumFloatNormal)), 4 segments x 750,000 rows per GPU, written with the reference's default
IndexSpec (Concise bitmaps, LZ4 blocks, LONGS encoding). A step = one topN query over all of this
rank's segments (one batched GPU call) + the cross-segment merge (TopNBinaryFn) + for N > 1 the
cross-rank all_gather / merge. Segments are resident in HBM before timing (attached once); every
step decodes the LZ4 blocks again, exactly as the reference decompresses blocks per query.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config topn|timeseries|groupby|filtered]
"""
import argparse
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

CONFIGS = {
    # name: (rows per segment, segments per GPU, description)
    "topn": (750_000, 4, "TopNBenchmark basic: topN dimUniform threshold=10, metric sumFloatNormal, 4 x 750k rows/GPU"),
    "topn_numeric": (750_000, 4, "TopNBenchmark basic.numericSort: topN dimUniform threshold=10, "
                                 "DimensionTopNMetricSpec(NUMERIC), longSum, 4 x 750k rows/GPU"),
    "topn_alphanumeric": (750_000, 4, "TopNBenchmark basic.alphanumericSort: topN dimUniform threshold=10, "
                                      "DimensionTopNMetricSpec(ALPHANUMERIC), longSum, 4 x 750k rows/GPU"),
    "timeseries": (750_000, 1, "TimeseriesBenchmark basic: timeseries ALL count+longSum+doubleSum, selector dimSequential=399"),
    # 1e9 rows in 64 time-partitioned segments over 30 days, 8 segments per GPU
    "ts_hourly": (15_625_000, 8, "1B-row dataset (64 x 15.625M rows, 30 days), 8 segments/GPU: timeseries HOUR "
                                 "count+longSum+doubleSum+longMax+doubleMin"),
    "groupby_hourly": (15_625_000, 8, "1B-row dataset (64 x 15.625M rows, 30 days), 8 segments/GPU: groupBy HOUR "
                                      "(dimZipf, dimSequential) longSum+doubleSum"),
    "groupby": (12_500_000, 1, "GroupByV2 dimUniform x dimHyperUnique + longSum/doubleSum"),
    "filtered": (12_500_000, 1, "compound AND/OR bound+selector+in filter, timeseries count"),
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
    p, rows, seed, bitmap, compression, lz4_mode, part, long_encoding = job
    if part is None:
        DG.write_basic_segment(p, rows, seed=seed, bitmap=bitmap, compression=compression, lz4_mode=lz4_mode,
                               long_encoding=long_encoding)
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


def ensure_segments(DG, root, rank, nseg, rows, compression, bitmap, lz4_mode, partitioned=False, workers=8,
                    long_encoding="longs"):
    """This rank's segments (seed 9999 + global segment index). partitioned: consecutive time chunks
    of the 1B-row dataset (rank r holds global chunks r*nseg ..); otherwise every segment spans the
    basic interval like the JMH benchmarks' segments. Written once, in parallel, and reused."""
    tag = ("p1b_" if partitioned else "") + ("auto_" if long_encoding == "auto" else "")
    d = os.path.join(root, f"{tag}r{rows}_s{nseg}_{compression}_{bitmap}_{lz4_mode}", f"rank{rank}")
    marker = os.path.join(d, "DONE")
    paths = [os.path.join(d, f"seg{i:04d}") for i in range(nseg)]
    if not os.path.exists(marker):
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d, exist_ok=True)
        jobs = [(p, rows, 9999 + rank * nseg + i, bitmap, compression, lz4_mode,
                 (rank * nseg + i) if partitioned else None, long_encoding) for i, p in enumerate(paths)]
        if len(jobs) > 1 and workers > 1:
            import multiprocessing as mp
            with mp.get_context("spawn").Pool(min(workers, len(jobs))) as pool:
                for p in pool.imap_unordered(_write_one, jobs):
                    print(f"[rank {rank}] wrote {p}", file=sys.stderr, flush=True)
        else:
            for j in jobs:
                print(f"[rank {rank}] wrote {_write_one(j)}", file=sys.stderr, flush=True)
        open(marker, "w").close()
    return paths


def cpu_baseline(Q, query, path, rows, seconds, codec="lz4", selected_fraction=1.0):
    """The oracle (scalar CPU restatement of the reference loops) on one segment, fresh decode each run.
    Reported in the metric's unit: selected (filtered) rows per second, i.e. the segment's rows times
    the query's selectivity measured on the GPU side."""
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
            "scanned_rows_per_s": rows * runs / el,
            "sample": f"{runs} run(s) of the query over 1 segment x {rows} rows (oracle/ C+numpy restatement, "
                      f"single thread, {codec.upper()} decode included), {el:.1f} s; value = scanned rows/s x "
                      f"selectivity {selected_fraction:.4g}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="topn", choices=sorted(CONFIGS))
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
    DG = importlib.import_module("incubator-druid_amd.datagen")
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        D = importlib.import_module("incubator-druid_amd.distributed")
        dist = D.init_from_env()

    rows_per, nseg, desc = CONFIGS[args.config]
    rows_per = args.rows or rows_per
    nseg = args.segments or nseg
    paths = ensure_segments(DG, args.data_dir, rank, nseg, rows_per, args.compression, args.bitmap, args.lz4_mode,
                            partitioned=args.config in ("ts_hourly", "groupby_hourly"), workers=args.write_workers,
                            long_encoding=args.long_encoding)
    segs = [S.GpuSegment(p, device=local_rank) for p in paths]
    query = make_query(Q, args.config)

    gdict = None
    if dist is not None and args.config.startswith("topn"):
        gdict = D.GlobalDictionary.build(dist, [s.dictionary(query.dimension) for s in segs])
        translations = [gdict.translate(s.dictionary(query.dimension)) for s in segs]
    gdicts = None
    if dist is not None and args.config.startswith("groupby"):
        gdicts = {d: D.GlobalDictionary.build(dist, [s.dictionary(d) for s in segs]) for d in query.dimensions}

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
        per = R.groupby_per_segment(segs, query, stats)
        if dist is None:
            return R.merge_groupby_columnar(query, per)
        merged = R.merge_groupby_columnar(query, per)
        part = R.GroupByPartial(merged[0], merged[1], merged[2])
        return D.gather_groupby(dist, query, part, gdicts)

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
    selected_local = stats.total("selected_rows") / steps
    scanned_local = sum(s.num_rows for s in segs)
    selected_all = selected_local * world  # every rank holds the same shape of data (weak scaling)
    value = selected_all * steps / elapsed
    # dominant kernel from the library's HIP-event timings (recorded on the context stream)
    decode_ms = stats.total("decode_ms") / steps
    agg_ms = stats.total("aggregate_ms") / steps
    bitmap_ms = stats.total("bitmap_ms") / steps
    bytes_read = stats.total("bytes_read") / steps
    uncompressed_equiv = None
    if args.config == "topn":
        uncompressed_equiv = scanned_local * (3 + 8 + 8)
    elif args.config.startswith("topn_"):
        uncompressed_equiv = scanned_local * (3 + 8)
    if decode_ms >= agg_ms and decode_ms > 0:
        kernel, k_ms, k_bytes = ("k_lzf_decode" if args.compression == "lzf" else "k_lz4_decode"), decode_ms, bytes_read
        if args.long_encoding == "auto":
            kernel = "k_lz4_decode+k_vsize_expand"  # the decode phase holds both launches
    else:
        # the aggregation kernel reads the decoded column bytes (ids + values) of every row
        kernel, k_ms = ("k_scan_agg" if args.config != "groupby" else "k_groupby"), agg_ms
        k_bytes = uncompressed_equiv if uncompressed_equiv else bytes_read
    achieved = (k_bytes / (k_ms / 1e3)) / 1e9 if k_ms > 0 else 0.0
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
        "data": "synthetic (basic schema, seeded numpy generator, written as Druid v9 segments)",
        "config": {"workload": desc, "config": args.config, "rows_per_segment": rows_per, "segments_per_gpu": nseg,
                   "compression": args.compression, "bitmap": args.bitmap, "long_encoding": args.long_encoding,
                   "parallelism": f"segments sharded over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "bytes_per_launch": k_bytes, "avg_launch_ms": k_ms},
        "phases_ms": {"bitmap": bitmap_ms, "decode": decode_ms, "aggregate": agg_ms,
                      "query_wall": stats.total("total_ms") / steps},
        "stored_bytes_per_step": bytes_read,
        "rows_scanned_per_step": scanned_local * world,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(Q, query, paths[0], rows_per, args.cpu_seconds, args.compression,
                                            selected_local / scanned_local if scanned_local else 1.0)
        line["cpu_baseline"]["cpu_model"] = _cpu_model()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _cpu_model():
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
