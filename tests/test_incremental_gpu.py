"""In-memory (realtime) segments: an IncrementalIndex's facts queried on the GPU
through dg_segment_from_rows (IncrementalIndexStorageAdapter: insertion-order dictionaries re-sorted,
no bitmap index — string filters are row predicates on the ids).

The reference's own strategy (QueryRunnerTestHelper.makeQueryRunners) runs every query over an
incremental index and over its persisted form and expects the same answer. Here: the index's rows are
persisted with the v9 writer (IndexMergerV9 layout); the oracle answers on the persisted segment, the
engine on the in-memory one (bit-exact floatSum included), and on the persisted one too. A realtime +
historical mix (one in-memory and one persisted segment of other rows in one call) checks the merged
dictionaries across both kinds. CPU: the index's rollup bookkeeping."""
import ctypes
import importlib

import numpy as np
import pytest

from compare import assert_results

METRICS = [("rows", "count", None), ("sumLong", "longSum", "l"), ("sumDouble", "doubleSum", "d"),
           ("sumFloat", "floatSum", "f"), ("minDouble", "doubleMin", "d"), ("maxFloat", "floatMax", "f")]


def _index(seed, n, rollup=True, gran="minute"):
    I = importlib.import_module("incubator-druid_amd.incremental")
    rng = np.random.default_rng(seed)
    idx = I.IncrementalIndex(["dimA", "dimB", "dimC", "tags"], METRICS, query_granularity=gran, rollup=rollup,
                             interval=(0, 6 * 3_600_000))
    a_vals = ["zeta", "alpha", "", "Beta", "béta", "gamma", "10", "9", "\U0001f600x", "～"]
    t = np.sort(rng.integers(0, 6 * 3_600_000, n))
    for i in range(n):
        ev = {"dimA": a_vals[min(int(rng.zipf(1.6)) - 1, len(a_vals) - 1)],
              "dimB": str(int(rng.integers(0, 400))),
              "l": int(rng.integers(-1000, 1000)), "d": float(rng.normal(100, 50)), "f": float(rng.normal(5000, 1))}
        if rng.random() < 0.6:
            ev["dimC"] = "c" + str(int(rng.integers(0, 30)))
        k = int(rng.integers(0, 4))  # multi-value: 0-3 tags (an empty list has no values)
        ev["tags"] = ["t" + str(int(x)) for x in rng.integers(0, 12, k)] if k != 1 or rng.random() < 0.5 else "t0"
        idx.add(int(t[i]), ev)
    return idx


def test_rollup_bookkeeping():
    I = importlib.import_module("incubator-druid_amd.incremental")
    idx = I.IncrementalIndex(["x"], [("rows", "count", None), ("s", "longSum", "v"), ("m", "floatMin", "w")],
                             query_granularity="hour")
    assert idx.add(10, {"x": "b", "v": 3, "w": 1.5}) == 1
    assert idx.add(3_599_999, {"x": "b", "v": 4, "w": -0.0}) == 1  # same hour, same value: rolled up
    assert idx.add(20, {"x": "", "v": 1, "w": 0.0}) == 2             # "" is null
    assert idx.add(30, {"v": 1, "w": 0.0}) == 2                      # missing is null too
    assert idx.add(3_600_000, {"x": "a", "v": 5, "w": 2.0}) == 3
    spec = idx.to_spec()
    assert spec.timestamps.tolist() == [0, 0, 3_600_000]
    dct, ids = spec.dims["x"]
    assert dct == ["", "a", "b"] and ids.tolist() == [0, 2, 1]  # null first, then "b" (same hour)
    assert spec.metrics["rows"][1].tolist() == [2, 2, 1]
    assert spec.metrics["s"][1].tolist() == [2, 7, 5]
    assert np.signbit(spec.metrics["m"][1][1]) and spec.metrics["m"][1][0] == 0.0
    mv = I.IncrementalIndex(["t"], [("rows", "count", None)])
    mv.add(0, {"t": ["b", "a"]})
    mv.add(0, {"t": []})
    mv.add(0, {"t": "a"})
    mv.add(0, {"t": ["a", "b"]})  # the same sorted row as the first: rolled up
    sp = mv.to_spec()
    dct, rows = sp.dims["t"]
    assert dct == ["", "a", "b"] and [r.tolist() for r in rows] == [[], [1], [1, 2]]  # by value count, then values
    assert sp.metrics["rows"][1].tolist() == [1, 1, 2]
    no = I.IncrementalIndex(["x"], [("rows", "count", None)], rollup=False)
    for _ in range(3):
        no.add(5, {"x": "a"})
    assert len(no) == 3


@pytest.fixture(scope="module")
def indexes():
    return {"rollup": _index(5, 40_000), "plain": _index(6, 6_000, rollup=False, gran="none"),
            "other": _index(7, 20_000)}


@pytest.fixture(scope="module")
def persisted(indexes, W, tmp_path_factory):
    base = tmp_path_factory.mktemp("incremental")
    return {k: W.write_segment(str(base / k), v.to_spec(), lz4_mode="fast") for k, v in indexes.items()}


def _queries(Q):
    aggs = [Q.long_sum("rows", "rows"), Q.long_sum("sumLong", "sumLong"), Q.double_sum("sumDouble", "sumDouble"),
            Q.float_sum("sumFloat", "sumFloat"), Q.double_min("minDouble", "minDouble"),
            Q.float_max("maxFloat", "maxFloat")]
    iv = ["1970-01-01T00:00:00Z/1970-01-01T05:30:00Z"]
    filters = [None, Q.SelectorDimFilter("dimA", "alpha"), Q.SelectorDimFilter("dimC", None),
               Q.InDimFilter("dimC", ["c1", "c7", None]),
               Q.BoundDimFilter("dimB", "50", "200", upperStrict=True, ordering="numeric"),
               Q.BoundDimFilter("dimA", "b", "z"),
               Q.AndDimFilter([Q.NotDimFilter(Q.SelectorDimFilter("dimA", "zeta")),
                               Q.OrDimFilter([Q.SelectorDimFilter("dimC", "c3"), Q.BoundDimFilter("dimB", None, "20", ordering="numeric")])])]
    out = []
    for f in filters:
        out.append(Q.TimeseriesQuery(intervals=iv, granularity="hour", filter=f, aggregations=aggs))
    out.append(Q.TimeseriesQuery(intervals=iv, granularity="all", filter=filters[4], aggregations=aggs, descending=True))
    out.append(Q.TopNQuery(intervals=iv, granularity="all", dimension="dimA", metric="sumLong", threshold=5,
                           aggregations=aggs, filter=filters[3]))
    out.append(Q.TopNQuery(intervals=iv, granularity="all", dimension="dimB", metric={"type": "dimension", "ordering": "numeric"},
                           threshold=20, aggregations=aggs))
    out.append(Q.GroupByQuery(intervals=iv, granularity="hour", dimensions=["dimA", "dimC"], aggregations=aggs,
                              filter=filters[6]))
    out.append(Q.GroupByQuery(intervals=iv, granularity="all", dimensions=["dimB", "dimA"], aggregations=aggs,
                              limitSpec={"type": "default", "columns": ["dimA"], "limit": 30}))
    # the multi-value dimension: grouped (a row under each of its values, an empty row as null),
    # topN per value, and filtered (a row matches when one of its values does)
    out.append(Q.GroupByQuery(intervals=iv, granularity="hour", dimensions=["tags", "dimC"], aggregations=aggs))
    out.append(Q.TopNQuery(intervals=iv, granularity="all", dimension="tags", metric="sumDouble", threshold=6,
                           aggregations=aggs, filter=filters[2]))
    for f in (Q.SelectorDimFilter("tags", "t3"), Q.SelectorDimFilter("tags", None), Q.InDimFilter("tags", ["t1", "t11", None]),
              Q.NotDimFilter(Q.BoundDimFilter("tags", "t2", "t5"))):
        out.append(Q.TimeseriesQuery(intervals=iv, granularity="hour", filter=f, aggregations=aggs))
        out.append(Q.GroupByQuery(intervals=iv, granularity="all", dimensions=["dimA"], aggregations=aggs, filter=f))
    return out


def _exact_floats(q, got, exp):
    name = "sumFloat"
    for g, e in zip(got, exp):
        if hasattr(g, "event"):
            assert np.float32(g.event[name]) == np.float32(e.event[name])
        elif isinstance(g.value, dict):
            assert np.float32(g.value[name]) == np.float32(e.value[name])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["rollup", "plain"])
def test_in_memory_segment_matches_persisted(Q, O, indexes, persisted, kind):
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")
    mem = indexes[kind].to_segment()
    disk = S.GpuSegment(persisted[kind])
    osg = O.OracleSegment(persisted[kind])
    assert mem.num_rows == disk.num_rows == len(indexes[kind])
    assert (mem.min_time, mem.max_time) == (disk.min_time, disk.max_time)
    for q in _queries(Q):
        exp = O.run(q, [osg])
        got = R.run_query(q, [mem])
        assert_results(q, got, exp)
        assert_results(q, got, R.run_query(q, [disk]))
        _exact_floats(q, got, exp)


@pytest.mark.gpu
def test_realtime_plus_historical(Q, O, indexes, persisted):
    """One call over an in-memory segment and a persisted segment of other rows (a realtime node's
    index next to historical segments): dictionaries merge across both kinds."""
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")
    segs = [indexes["rollup"].to_segment(), S.GpuSegment(persisted["other"])]
    osegs = [O.OracleSegment(persisted["rollup"]), O.OracleSegment(persisted["other"])]
    for q in _queries(Q):
        assert_results(q, R.run_query(q, segs), O.run(q, osegs))


@pytest.mark.gpu
def test_from_rows_argument_errors():
    N = importlib.import_module("incubator-druid_amd._native")
    S = importlib.import_module("incubator-druid_amd.segment")
    ctx = S.GpuContext.get(0)
    L = N.lib()

    def call(ts, cols):
        ts = np.asarray(ts, np.int64)
        arr = (N.dg_row_column * max(len(cols), 1))(*cols)
        h = ctypes.c_void_p()
        rc = L.dg_segment_from_rows(ctx.handle, len(ts), ts.ctypes.data, 0, 100, ctypes.cast(arr, ctypes.c_void_p),
                                    len(cols), ctypes.byref(h))
        if rc == 0:
            L.dg_segment_release(h)
        return rc

    vals = (ctypes.c_char_p * 2)(b"a", b"b")
    ids = np.array([0, 1, 1], np.int32)
    good = N.dg_row_column(b"d", 4, 2, ctypes.cast(vals, ctypes.c_void_p), ids.ctypes.data, None)
    assert call([1, 2, 3], [good]) == 0
    assert call([3, 2, 1], [good]) == 6                      # timestamps must ascend
    dup = (ctypes.c_char_p * 2)(b"a", b"a")
    assert call([1, 2, 3], [N.dg_row_column(b"d", 4, 2, ctypes.cast(dup, ctypes.c_void_p), ids.ctypes.data, None)]) == 6
    bad = np.array([0, 2, 1], np.int32)
    assert call([1, 2, 3], [N.dg_row_column(b"d", 4, 2, ctypes.cast(vals, ctypes.c_void_p), bad.ctypes.data, None)]) == 6
    assert call([1, 2, 3], [good, good]) == 6                # repeated name
    assert call([1, 2, 3], [N.dg_row_column(b"__time", 1, 0, None, None, ids.ctypes.data)]) == 6
