"""The library's own merge across devices of ONE process (QueryRunnerFactory.mergeRunners,
query/QueryRunnerFactory.java:62; a historical is one JVM driving every device):

- dg_groupby_merge_devices: the devices' dg_groupby_run results re-keyed into the union key space,
  cut into key ranges, moved between devices with peer copies and merged on the target
  (GroupByMergingQueryRunnerV2.java:170-290 semantics). On the one-GPU test box the "devices" are
  two contexts on device 0 (the copies are then device copies; on an 8-GPU node the same calls move
  the ranges over xGMI).
- dg_timeseries_merge: the TimeseriesBinaryFn fold (TimeseriesBinaryFn.java:67-70) of every
  segment's bucket list, host-side in the library; checked on CPU against the toolchest merge
  restated in Python (runners.merge_timeseries) on random lists with NaN / -0.0 min/max inputs."""
import ctypes
import importlib

import numpy as np
import pytest

from compare import TOL, assert_results

IV = ["1970-01-01/2020-01-01"]


def _ts_lists(Q, rng, n_lists, cap, period):
    aggs = [Q.count("rows"), Q.long_sum("ls", "l"), Q.double_sum("ds", "d"), Q.float_sum("fs", "d"),
            Q.AggregatorFactory("doubleMin", "dmin", "d"), Q.AggregatorFactory("doubleMax", "dmax", "d"),
            Q.AggregatorFactory("floatMin", "fmin", "d"), Q.AggregatorFactory("longMax", "lmax", "l")]
    specials = np.array([np.nan, -0.0, 0.0, 1.5, -2.25, np.inf, -np.inf, 3.0])
    per, lists = [], []
    for i in range(n_lists):
        k = int(rng.integers(0, cap + 1))
        starts = np.sort(rng.choice(np.arange(40), k, replace=False)) * period
        res = []
        for t in starts:
            d = float(rng.choice(specials)) if rng.random() < 0.5 else float(rng.normal())
            f = float(np.float32(d))
            rows = int(rng.integers(0, 3))
            ev = {"rows": rows, "ls": int(rng.integers(-2**62, 2**62)), "ds": d, "fs": f, "dmin": d, "dmax": d,
                  "fmin": f, "lmax": int(rng.integers(-5, 5))}
            res.append((int(t), rows, ev))
        lists.append(res)
        per.append([Q.Result(t, ev) for t, rows, ev in res])
    return aggs, lists, per


@pytest.mark.parametrize("gran", ["all", "hour"])
@pytest.mark.parametrize("skip", [False, True])
def test_timeseries_merge_matches_toolchest(Q, gran, skip):
    N = importlib.import_module("incubator-druid_amd._native")
    R = importlib.import_module("incubator-druid_amd.runners")
    rng = np.random.default_rng(7)
    period = 3_600_000
    for trial in range(20):
        n_lists, cap = int(rng.integers(1, 6)), 12
        aggs, lists, per = _ts_lists(Q, rng, n_lists, cap, period)
        ctx = {"skipEmptyBuckets": True} if skip else None
        q = Q.TimeseriesQuery(intervals=IV, granularity=gran, aggregations=aggs, context=ctx,
                              descending=bool(trial % 2))
        na = len(aggs)
        nb = np.array([len(l) for l in lists], dtype=np.int32)
        times = np.zeros(n_lists * cap, np.int64)
        rows = np.zeros(n_lists * cap, np.int64)
        vals = np.zeros(n_lists * cap * na, np.uint64)
        for i, l in enumerate(lists):
            for k, (t, r, ev) in enumerate(l):
                times[i * cap + k], rows[i * cap + k] = t, r
                for a_i, a in enumerate(aggs):
                    v = ev[a.name]
                    if a.output_type == "long":
                        vals[(i * cap + k) * na + a_i] = np.int64(v).view(np.uint64)
                    elif a.output_type == "double":
                        vals[(i * cap + k) * na + a_i] = np.float64(v).view(np.uint64)
                    else:
                        vals[(i * cap + k) * na + a_i] = np.uint64(np.float32(v).view(np.uint32))
        scan, keep = N.make_scan(q, Q, filters=False)
        on = ctypes.c_int32()
        out_cap = n_lists * cap
        o_t = np.zeros(max(out_cap, 1), np.int64)
        o_r = np.zeros(max(out_cap, 1), np.int64)
        o_v = np.zeros(max(out_cap, 1) * na, np.uint64)
        N.check(N.lib().dg_timeseries_merge(ctypes.byref(scan), n_lists, nb.ctypes.data, cap, times.ctypes.data,
                                            rows.ctypes.data, vals.ctypes.data, int(skip), out_cap, ctypes.byref(on),
                                            o_t.ctypes.data, o_r.ctypes.data, o_v.ctypes.data))
        if skip:  # skipEmptyBuckets drops a segment's empty buckets before the merge
            per = [[r for r, (_, rows_, _) in zip(p, l) if rows_ != 0] for p, l in zip(per, lists)]
        exp = R.merge_timeseries(q, per)
        cols = R._decode_slots(aggs, o_v.reshape(-1, na)[:on.value])
        got = [Q.Result(int(o_t[b]), {a.name: R._py(c[b], a.output_type) for a, c in zip(aggs, cols)})
               for b in range(on.value)]
        assert_results(q, got, exp)


@pytest.fixture(scope="module")
def two_contexts(tmp_path_factory, DG):
    """Config 3's shape at test size (dimUniform x dimHyperUnique, 3-byte ids, ~1 group per row), 4
    segments of 300k rows with different dictionaries, two on each of two contexts."""
    S = importlib.import_module("incubator-druid_amd.segment")
    import oracle as O
    base = tmp_path_factory.mktemp("merge_devices")
    paths = DG.write_basic_dataset(str(base), 4, 300_000, lz4_mode="fast", dims=["dimUniform", "dimHyperUnique"],
                                   metrics=["sumLongSequential", "sumFloatNormal", "minFloatZipf"])
    ca, cb = S.GpuContext(0), S.GpuContext(0)
    g = [S.GpuSegment(p, context=ca if i % 2 == 0 else cb) for i, p in enumerate(paths)]
    return (ca, cb), g, [O.OracleSegment(p) for p in paths]


@pytest.mark.gpu
def test_merge_devices_million_groups(Q, O, two_contexts):
    R = importlib.import_module("incubator-druid_amd.runners")
    (ca, cb), g, o = two_contexts
    aggs = [Q.count("rows"), Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal"),
            Q.float_sum("fs", "sumFloatNormal"), Q.AggregatorFactory("doubleMin", "dmin", "minFloatZipf")]
    q = Q.GroupByQuery(intervals=IV, dimensions=["dimUniform", "dimHyperUnique"], aggregations=aggs)
    exp = O.run(q, o)
    assert len(exp) > 1_000_000
    # the factory's mergeRunners over segments of two contexts: one dg_groupby_merge_devices call
    stats = R.RunStats()
    assert_results(q, R.run_query(q, g, stats), exp)
    assert len(stats.calls) == 3  # two dg_groupby_run + one dg_groupby_merge_devices
    # key ranges owned by both contexts: their concatenation is the merged result
    parts = R.groupby_merge_devices(g, q, targets=[ca, cb])
    try:
        assert all(p.groups > 300_000 for p in parts)
        got = [p.fetch() for p in parts]
    finally:
        for p in parts:
            p.release()
    keys = [tuple(r.event[d] for d in q.dimensions) for r in exp]
    assert [k for p in got for k in zip(*[list(c) for c in p.dims])] == keys
    for i, a in enumerate(aggs):
        col = np.concatenate([p.aggs[i] for p in got])
        e = np.array([r.event[a.name] for r in exp])
        if a.type in ("doubleSum", "floatSum"):
            assert np.allclose(col, e, rtol=TOL["double" if a.type == "doubleSum" else "float"], atol=0), a.name
        else:
            assert np.array_equal(col, e.astype(col.dtype)), a.name


@pytest.mark.gpu
def test_merge_devices_granularity_and_filters(Q, O, two_contexts):
    R = importlib.import_module("incubator-druid_amd.runners")
    _, g, o = two_contexts
    aggs = [Q.count("rows"), Q.long_sum("sumLongSequential"), Q.AggregatorFactory("doubleMax", "dmax", "minFloatZipf")]
    for q in (Q.GroupByQuery(intervals=IV, granularity="minute", dimensions=["dimUniform"], aggregations=aggs,
                             filter=Q.BoundDimFilter("dimHyperUnique", "100", "400")),
              Q.GroupByQuery(intervals=IV, granularity={"type": "period", "period": "P1M", "timeZone": "America/Los_Angeles"},
                             dimensions=["dimHyperUnique"], aggregations=aggs,
                             filter=Q.InDimFilter("dimUniform", ["5", "77", "1234"])),
              Q.GroupByQuery(intervals=IV, dimensions=["dimUniform"], aggregations=aggs,
                             limitSpec={"type": "default", "limit": 7,
                                        "columns": [{"dimension": "dimUniform", "direction": "descending"}]})):
        assert_results(q, R.run_query(q, g), O.run(q, o))
    # timeseries over both contexts: dg_timeseries_merge of every segment's buckets
    for gran in ("all", "minute"):
        q = Q.TimeseriesQuery(intervals=IV, granularity=gran, aggregations=aggs + [Q.float_sum("fs", "sumFloatNormal")],
                              filter=Q.NotDimFilter(Q.SelectorDimFilter("dimUniform", "3")))
        assert_results(q, R.run_query(q, g), O.run(q, o))


@pytest.mark.gpu
def test_merge_devices_runs_concurrently_and_spreads_targets(Q, O, two_contexts):
    """The in-process mergeRunners issues every context's dg_groupby_run at once (their host call spans
    overlap: the two calls were issued concurrently, each from its own thread; whether their kernels
    overlapped on the device is not measured here) and by default every participating context owns a
    key range of the merged result (nothing funnels into the first device)."""
    R = importlib.import_module("incubator-druid_amd.runners")
    (ca, cb), g, o = two_contexts
    aggs = [Q.count("rows"), Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")]
    q = Q.GroupByQuery(intervals=IV, dimensions=["dimUniform", "dimHyperUnique"], aggregations=aggs)
    exp = O.run(q, o)
    overlapped = False
    for _ in range(3):  # (thread start-up order can serialise one attempt)
        stats = R.RunStats()
        parts = R.groupby_merge_devices(g, q, stats)
        try:
            runs = [c for c in stats.calls if "t_start" in c]
            assert len(runs) == 2 and len(parts) == 2
            overlapped |= max(c["t_start"] for c in runs) < min(c["t_end"] for c in runs)
            assert all(p.groups > 300_000 for p in parts)
            got = [p.fetch() for p in parts]
        finally:
            for p in parts:
                p.release()
        keys = [tuple(r.event[d] for d in q.dimensions) for r in exp]
        assert [k for p in got for k in zip(*[list(c) for c in p.dims])] == keys
        for i, a in enumerate(aggs):
            col = np.concatenate([p.aggs[i] for p in got])
            e = np.array([r.event[a.name] for r in exp])
            if a.type == "doubleSum":
                assert np.allclose(col, e, rtol=TOL["double"], atol=0)
            else:
                assert np.array_equal(col, e.astype(col.dtype))
        if overlapped:
            break
    assert overlapped
