"""BASELINE configs[4] at its shape: the 1B-row dataset's time-partitioned LZ4 segments (bench.py
DATASET_1B: 64 consecutive time chunks of a 30-day interval, one segment per chunk, its interval =
its chunk), hourly timeseries (count, longSum, doubleSum, longMax, doubleMin) and hourly groupBy on
(dimZipf, dimSequential) with longSum + doubleSum, checked against the oracle, plus the two-rank
merge of those partials (the exchange the 8-GPU run does over RCCL) with two ranks as threads on
one GPU joined by a loopback stand-in for torch.distributed.

Segments here are the bench generator's chunks 0-3 at 1.5 M rows each (the bench writes 15.625 M
rows per chunk; the oracle is too slow for that), LZ4-HC like the reference's default IndexSpec,
spanning 45 hours — every segment holds ~12 hourly buckets and its first and last bucket are shared
with the neighbouring segments. Reference path: QueryableIndexStorageAdapter.makeCursors /
CursorSequenceBuilder.build (:367-456, one cursor per bucket, TimestampCheckingOffset), the
timeseries engine (TimeseriesQueryEngine.java:40-111) and GroupByQueryEngineV2.java:91-187 +
GroupByMergingQueryRunnerV2.java:170-290; cross-rank: TimeseriesBinaryFn.java:67-70 and the groupBy
merge by value."""
import importlib
import os

import numpy as np
import pytest

from compare import assert_results

pytestmark = pytest.mark.gpu

ROWS = 1_500_000
NSEG = 4


@pytest.fixture(scope="module")
def cfg5(tmp_path_factory):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    import bench as B
    base = str(tmp_path_factory.mktemp("cfg5"))
    jobs = [(os.path.join(base, f"seg{i}"), ROWS, 9999 + i, "concise", "lz4", "hc", i, "longs", B.BASIC)
            for i in range(NSEG)]
    import multiprocessing as mp
    with mp.get_context("spawn").Pool(NSEG) as pool:
        paths = pool.map(B._write_one, jobs)
    S = importlib.import_module("incubator-druid_amd.segment")
    import oracle as O
    return B, [S.GpuSegment(p) for p in paths], [O.OracleSegment(p) for p in paths]


@pytest.fixture(scope="module")
def R():
    return importlib.import_module("incubator-druid_amd.runners")


def test_segments_are_time_partitioned(cfg5):
    _, g, o = cfg5
    prev_end = None
    for gs, os_ in zip(g, o):
        t = os_.time()
        assert gs.num_rows == ROWS and gs.min_time == int(t[0]) and gs.max_time == int(t[-1])
        assert t[-1] - t[0] > 10 * 3_600_000  # ~11 hours per chunk
        if prev_end is not None:
            assert int(t[0]) >= prev_end
        prev_end = int(t[-1])


@pytest.mark.parametrize("interval", [None, ["1970-01-01T05:30:00/1970-01-02T20:00:00"]])
def test_hourly_timeseries(Q, O, R, cfg5, interval):
    B, g, o = cfg5
    q = B.make_query(Q, "ts_hourly")
    if interval:
        q = Q.TimeseriesQuery(intervals=interval, granularity="hour", aggregations=q.aggregations)
    exp = O.run(q, o)
    assert len(exp) >= 40 if interval is None else len(exp) == 39
    assert_results(q, R.run_query(q, g), exp)
    # per-segment runners merged by TimeseriesBinaryFn (QueryRunnerFactory.mergeRunners): one call per
    # segment, then the toolchest merge, equals the one batched call
    per = [R.run_query(q, [s]) for s in g]
    assert_results(q, R.merge_timeseries(q, [[r] for rs in per for r in rs]), exp)


@pytest.mark.parametrize("counted", ["0", "1"])
@pytest.mark.parametrize("interval", [None, ["1970-01-01T05:30:00/1970-01-02T20:00:00"]])
def test_hourly_groupby(Q, O, R, cfg5, interval, counted, monkeypatch):
    """configs[4]b's hourly groupBy over the whole interval (every row an element: the keygen runs
    without its count pass) and over an interval that cuts the segments (rows dropped by their time:
    counted), and with the count pass forced (DG_GB_COUNT=1)."""
    monkeypatch.setenv("DG_GB_COUNT", counted)
    B, g, o = cfg5
    q = B.make_query(Q, "groupby_hourly")
    if interval:
        q = Q.GroupByQuery(intervals=interval, granularity="hour", dimensions=q.dimensions,
                           aggregations=q.aggregations)
    exp = O.run(q, o)
    assert len(exp) > 1_000_000
    assert_results(q, R.run_query(q, g), exp)


class _ReduceOp:
    SUM, MIN, MAX = "sum", "min", "max"


def test_two_rank_merge(Q, O, R, cfg5):
    """Two ranks (threads) with two segments each: hourly groupBy through GroupByExchange (key
    ranges exchanged, merged on the receiving rank) and hourly timeseries through
    allreduce_timeseries (per-bucket sums / Math.min/max reductions)."""
    import threading
    import torch
    import test_merge_gpu as TM
    B, g, o = cfg5
    D = importlib.import_module("incubator-druid_amd.distributed")
    q = B.make_query(Q, "groupby_hourly")
    parts = TM._run_ranks(R, D, Q, [g[:2], g[2:]], q)
    assert all(len(p) > 300_000 for p in parts)
    assert_results(q, TM._rows(Q, q, parts), O.run(q, o))

    class Loop(TM.LoopbackDist):
        ReduceOp = _ReduceOp

        def all_reduce(self, t, op):
            got = self._exchange(t.clone())
            fn = {"sum": lambda a, b: a + b, "min": torch.minimum, "max": torch.maximum}[op]
            acc = got[0]
            for x in got[1:]:
                acc = fn(acc, x)
            t.copy_(acc)

    qt = B.make_query(Q, "ts_hourly")
    hub = TM._Hub(2)
    out, err = [None, None], []

    def work(rank):
        try:
            segs = g[:2] if rank == 0 else g[2:]
            local = R.merge_timeseries(qt, R.timeseries_per_segment(segs, qt, R.RunStats()))
            out[rank] = D.allreduce_timeseries(Loop(hub, rank), qt, local)
        except Exception as e:
            err.append(e)
            hub.barrier.abort()

    th = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise err[0]
    exp = O.run(qt, o)
    assert_results(qt, out[0], exp)
    assert_results(qt, out[1], exp)


@pytest.mark.parametrize("kind", ["timeseries", "groupby", "topn"])
def test_uniform_time_blocks_are_not_decoded(R, cfg5, kind, monkeypatch):
    """__time blocks whose rows share one hourly bucket (almost every block of these time-sorted
    segments) are not decoded: the scan reads fewer stored bytes than with every block decoded
    (DG_NO_TIME_SKIP=1), and the results are identical, also with an interval cutting blocks."""
    B, g, o = cfg5
    Q = importlib.import_module("incubator-druid_amd.query")
    lo, hi = g[0].min_time + 1_234_567, g[-1].max_time - 7_654_321
    for iv in (["1970-01-01/2020-01-01"], [(lo, hi)]):
        if kind == "timeseries":
            q = Q.TimeseriesQuery(intervals=iv, granularity="hour", aggregations=[Q.count("rows"),
                                                                                   Q.long_sum("sumLongSequential")])
        elif kind == "groupby":
            q = Q.GroupByQuery(intervals=iv, granularity="hour", dimensions=["dimZipf"],
                               aggregations=[Q.count("rows"), Q.double_sum("sumFloatNormal")])
        else:
            q = Q.TopNQuery(intervals=iv, granularity="hour", dimension="dimZipf", metric="rows", threshold=5,
                            aggregations=[Q.count("rows")])
        runs = {}
        for mode in ("skip", "decode"):
            if mode == "decode":
                monkeypatch.setenv("DG_NO_TIME_SKIP", "1")
            else:
                monkeypatch.delenv("DG_NO_TIME_SKIP", raising=False)
            stats = R.RunStats()
            runs[mode] = (R.run_query(q, g, stats), sum(c["bytes_read"] for c in stats.calls))
        monkeypatch.delenv("DG_NO_TIME_SKIP", raising=False)
        (a, bytes_skip), (b, bytes_all) = runs["skip"], runs["decode"]
        assert bytes_skip < bytes_all, (bytes_skip, bytes_all)
        assert_results(q, a, b)


@pytest.mark.parametrize("shape", ["hourly", "hourly_cut", "all", "day_desc", "pt6h_tz", "filtered", "filtered_all",
                                   "filtered_all_fagg"])
def test_fused_decode_aggregate(Q, O, R, cfg5, shape, monkeypatch):
    """Timeseries decode fused with aggregation: the LZ4 value blocks whose rows share one bucket are
    folded by the decoder into the bucket's slot (no decoded image written, the scan skips their
    rows). Results equal the unfused path (DG_NO_FUSE=1) and the oracle, for every aggregator kind of
    configs[4]a (longSum, doubleSum, longMax, doubleMin), an interval cutting blocks, ALL granularity
    (one bucket: every value block fused), a descending day query, calendar buckets in a +05:45 zone,
    and filtered queries (round 6: the decoders fold only the rows of the filter's bitset): hourly,
    ALL with a count (every aggregator folded or a plain count: no scan, the rows are the filter's
    count) and ALL with a FilteredAggregator count (the scan runs for it)."""
    B, g, o = cfg5
    base = B.make_query(Q, "ts_hourly")
    aggs = base.aggregations + [Q.long_min("lmin", "maxLongUniform"), Q.double_max("dmax", "sumFloatNormal")]
    lo, hi = g[0].min_time + 1_234_567, g[-1].max_time - 7_654_321
    iv = ["1970-01-01/2020-01-01"]
    kw = {}
    if shape == "hourly":
        q = Q.TimeseriesQuery(intervals=iv, granularity="hour", aggregations=aggs)
    elif shape == "hourly_cut":
        q = Q.TimeseriesQuery(intervals=[(lo, hi)], granularity="hour", aggregations=aggs)
    elif shape == "all":
        q = Q.TimeseriesQuery(intervals=iv, granularity="all", aggregations=aggs)
    elif shape == "day_desc":
        q = Q.TimeseriesQuery(intervals=[(lo, hi)], granularity="day", aggregations=aggs, descending=True)
    elif shape == "pt6h_tz":  # calendar buckets (caller-given bucket starts): a zone with a 45-minute offset
        q = Q.TimeseriesQuery(intervals=iv, aggregations=aggs,
                              granularity={"type": "period", "period": "PT6H", "timeZone": "Asia/Kathmandu"})
    elif shape == "filtered":
        q = Q.TimeseriesQuery(intervals=iv, granularity="hour", aggregations=aggs,
                              filter=Q.BoundDimFilter("dimSequential", "100", "500"))
    else:
        extra = [Q.count("n")]
        if shape == "filtered_all_fagg":
            extra.append(Q.filtered(Q.count("n7"), Q.SelectorDimFilter("dimSequential", "7")))
        q = Q.TimeseriesQuery(intervals=iv, granularity="all", aggregations=aggs + extra,
                              filter=Q.OrDimFilter([Q.BoundDimFilter("dimSequential", "100", "500"),
                                                    Q.SelectorDimFilter("dimZipf", "3")]))
    runs = {}
    for mode in ("fused", "plain"):
        if mode == "plain":
            monkeypatch.setenv("DG_NO_FUSE", "1")
        else:
            monkeypatch.delenv("DG_NO_FUSE", raising=False)
        stats = R.RunStats()
        runs[mode] = (R.run_query(q, g, stats), stats.total("lz4_fused_blocks"))
    monkeypatch.delenv("DG_NO_FUSE", raising=False)
    (a, nf), (b, n0) = runs["fused"], runs["plain"]
    assert n0 == 0
    if shape.startswith("filtered"):
        assert nf > 0.5 * 4 * NSEG * (ROWS // 8192), nf
    else:
        # configs[4]a's value columns: 4 columns x ~183 blocks per 1.5 M-row segment; only blocks at
        # bucket edges (and light blocks) are decoded
        assert nf > (0.97 if shape == "all" else 0.5) * 4 * NSEG * (ROWS // 8192), nf
    assert_results(q, a, b)
    assert_results(q, a, O.run(q, o))


@pytest.fixture(scope="module")
def signed_seg(tmp_path_factory, W):
    """One 600 k-row LZ4 segment of signed values: sequential longs running from -300 000 upwards (value
    runs through the sign change: run blocks), wide random longs, and doubles of both signs."""
    rng = np.random.default_rng(77)
    n = 600_000
    ts = np.arange(n, dtype=np.int64) * 3  # 30 minutes of rows
    spec = W.SegmentSpec(timestamps=ts, interval=(0, 3 * n),
                         dims={"d": W.encode_int_strings(rng.integers(0, 50, n))},
                         metrics={"seq": ("long", np.arange(n, dtype=np.int64) - 300_000),
                                  "wide": ("long", rng.integers(-(1 << 62), 1 << 62, n)),
                                  "dbl": ("double", rng.normal(-250.0, 1000.0, n))})
    p = W.write_segment(str(tmp_path_factory.mktemp("signed") / "seg"), spec)
    S = importlib.import_module("incubator-druid_amd.segment")
    import oracle as O
    return S.GpuSegment(p), O.OracleSegment(p)


@pytest.mark.parametrize("route", ["run", "no_run"])
def test_fused_folds_signed_and_cross_type(Q, O, R, signed_seg, route, monkeypatch):
    """Every fold of a fused decode over negative values: longMin / longMax / longSum (native int64),
    doubleSum, and the generic folds (doubleMax, doubleMin, longSum over a double column = Java's
    (long) cast, doubleSum over a long column), on the run decoder and on the general decoder
    (DG_NO_RUN_DECODE=1), against the unfused path and the oracle."""
    g, o = signed_seg
    if route == "no_run":
        monkeypatch.setenv("DG_NO_RUN_DECODE", "1")
    aggs = [Q.count("rows"), Q.long_min("smin", "seq"), Q.long_max("smax", "seq"), Q.long_sum("ssum", "seq"),
            Q.long_min("wmin", "wide"), Q.long_max("wmax", "wide"), Q.long_sum("wsum", "wide"),
            Q.double_sum("dsum", "dbl"), Q.double_max("dmax", "dbl"), Q.double_min("dmin", "dbl"),
            Q.long_sum("lsum_of_dbl", "dbl"), Q.double_sum("dsum_of_seq", "seq")]
    for gran in ("all", "minute"):
        q = Q.TimeseriesQuery(intervals=["1970-01-01/2020-01-01"], granularity=gran, aggregations=aggs)
        runs = {}
        for mode in ("fused", "plain"):
            if mode == "plain":
                monkeypatch.setenv("DG_NO_FUSE", "1")
            else:
                monkeypatch.delenv("DG_NO_FUSE", raising=False)
            stats = R.RunStats()
            runs[mode] = (R.run_query(q, [g], stats), stats.total("lz4_fused_blocks"))
        monkeypatch.delenv("DG_NO_FUSE", raising=False)
        (a, nf), (b, n0) = runs["fused"], runs["plain"]
        assert n0 == 0 and nf > 0, (nf, n0)
        assert_results(q, a, b)
        assert_results(q, a, O.run(q, [o]))


def test_time_skip_needs_no_row_order_inside_blocks(Q, R, W, tmp_path, monkeypatch):
    """The uniform-block skip bounds a __time block by its smallest and largest row time (recorded at
    attach), not by its neighbours' first rows, so rows shuffled inside their blocks still land in
    their own hour: the same per-hour counts and sums as decoding every block (DG_NO_TIME_SKIP=1)
    and as bucketing every row on the host."""
    rng = np.random.default_rng(5)
    nblk, per = 48, 8192
    span = 1_500_000  # ms per block: most blocks inside one hour, some across an hour boundary
    ts = np.concatenate([rng.permutation(np.arange(k * span, (k + 1) * span, span // per)[:per]) for k in range(nblk)])
    # the segment's first and last rows stay its min and max time (StorageAdapter.getMinTime / getMaxTime)
    i0, i1 = int(np.argmin(ts[:per])), len(ts) - per + int(np.argmax(ts[-per:]))
    ts[[0, i0]] = ts[[i0, 0]]
    ts[[-1, i1]] = ts[[i1, -1]]
    vals = rng.integers(-1000, 1000, len(ts))
    spec = W.SegmentSpec(timestamps=ts.astype(np.int64), interval=(0, nblk * span),
                         dims={"d": W.encode_int_strings(rng.integers(0, 5, len(ts)))},
                         metrics={"v": ("long", vals.astype(np.int64))})
    S = importlib.import_module("incubator-druid_amd.segment")
    seg = S.GpuSegment(W.write_segment(str(tmp_path / "seg"), spec, check_sorted=False))
    q = Q.TimeseriesQuery(intervals=["1970-01-01/2020-01-01"], granularity="hour",
                          aggregations=[Q.count("rows"), Q.long_sum("s", "v")])
    runs = {}
    for mode in ("skip", "decode"):
        if mode == "decode":
            monkeypatch.setenv("DG_NO_TIME_SKIP", "1")
        else:
            monkeypatch.delenv("DG_NO_TIME_SKIP", raising=False)
        stats = R.RunStats()
        runs[mode] = (R.run_query(q, [seg], stats), sum(c["bytes_read"] for c in stats.calls))
    monkeypatch.delenv("DG_NO_TIME_SKIP", raising=False)
    (a, bytes_skip), (b, bytes_all) = runs["skip"], runs["decode"]
    assert bytes_skip < bytes_all, (bytes_skip, bytes_all)
    assert_results(q, a, b)
    hour = ts // 3_600_000
    exp = {int(h) * 3_600_000: (int((hour == h).sum()), int(vals[hour == h].sum())) for h in np.unique(hour)}
    got = {r.timestamp: (r.value["rows"], r.value["s"]) for r in a if r.value["rows"]}
    assert got == exp
    seg.close()

