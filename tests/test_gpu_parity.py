"""GPU parity suite (MI355X): the HIP path through the C-ABI against the CPU oracle and the
reference's known-answer tests. Integer work (row selections, counts, long sums, min/max) must be
bit-exact; doubleSum within 1e-9 and floatSum within 1e-5 relative (tests/compare.py)."""
import importlib

import numpy as np
import pytest

from compare import assert_kat, assert_results

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R():
    return importlib.import_module("incubator-druid_amd.runners")


@pytest.fixture(scope="module")
def S():
    return importlib.import_module("incubator-druid_amd.segment")


@pytest.fixture(scope="module")
def gpu_sample(S, sample_dirs):
    return {k: S.GpuSegment(p) for k, p in sample_dirs.items()}


@pytest.fixture(scope="module")
def gpu_basic(S, basic_dirs):
    return {k: [S.GpuSegment(p) for p in ps] for k, ps in basic_dirs.items()}


@pytest.fixture(scope="module")
def oracle_basic(O, basic_dirs):
    return {k: [O.OracleSegment(p) for p in ps] for k, ps in basic_dirs.items()}


def test_segment_attach_facts(S, O, sample_dirs, v8_dir, kats):
    g = S.GpuSegment(v8_dir)
    assert g.num_rows == 6
    assert (g.min_time, g.max_time) == (kats["v8_segment"]["time"][0], kats["v8_segment"]["time"][-1])
    assert g.dictionary("dim1") == [None, "dim10"]
    for p in sample_dirs.values():
        gs, os_ = S.GpuSegment(p), O.OracleSegment(p)
        assert gs.num_rows == os_.num_rows
        assert gs.min_time == int(os_.time()[0]) and gs.max_time == int(os_.time()[-1])
        assert gs.dictionary("quality") == os_.dictionary("quality")


def test_engine_kats_on_gpu(R, Q, engine_kats, gpu_sample):
    for layout, seg in gpu_sample.items():
        for case in engine_kats["cases"]:
            q = Q.query_from_json(case["query"])
            got = R.run_query(q, [seg])
            if "expected_rows" in case:
                exp = case["expected_rows"]
                assert len(got) == len(exp), (layout, case["name"])
                for row, (day, val, rows, idx, dsum) in zip(got, exp):
                    assert row.timestamp == Q.parse_time(day)
                    assert row.event["quality"] == val
                    assert row.event["rows"] == rows and row.event["idx"] == idx
                    assert abs(row.event["idxDouble"] - dsum) <= 1e-6 * dsum
                    assert abs(row.event["idxFloat"] - dsum) <= 1e-5 * dsum
            else:
                assert_kat(q, got, case["expected"])


def _filters(Q):
    return [
        None,
        Q.SelectorDimFilter("dimSequential", "399"),
        Q.SelectorDimFilter("dimSequentialHalfNull", None),
        Q.SelectorDimFilter("dimNull", None),
        Q.SelectorDimFilter("missingDim", None),
        Q.SelectorDimFilter("missingDim", "x"),
        Q.SelectorDimFilter("dimUniform", "no-such-value"),
        Q.InDimFilter("dimZipf", ["1", "2", "3", "77"]),
        Q.BoundDimFilter("dimSequential", "100", "200", False, True),
        Q.BoundDimFilter("dimUniform", "0", "100", True, True),
        Q.BoundDimFilter("dimSequential", "100", "200", False, True, "numeric"),
        Q.BoundDimFilter("dimZipf", None, "5", False, False, "numeric"),
        Q.NotDimFilter(Q.SelectorDimFilter("dimZipf", "7")),
        Q.OrDimFilter([Q.AndDimFilter([Q.BoundDimFilter("dimSequential", "100", "200"),
                                       Q.InDimFilter("dimZipf", ["1", "2", "3"])]),
                       Q.SelectorDimFilter("dimUniform", "199"),
                       Q.NotDimFilter(Q.SelectorDimFilter("dimZipf", "7"))]),
        Q.AndDimFilter([Q.NotDimFilter(Q.InDimFilter("dimZipf", ["1", "2"])),
                        Q.OrDimFilter([Q.SelectorDimFilter("dimSequentialHalfNull", None),
                                       Q.BoundDimFilter("dimHyperUnique", "5", "6")])]),
    ]


ALL_AGGS = [
    ("count", "rows", None), ("longSum", "ls", "sumLongSequential"), ("doubleSum", "ds", "sumFloatNormal"),
    ("floatSum", "fs", "sumFloatNormal"), ("longMin", "lmin", "maxLongUniform"), ("longMax", "lmax", "maxLongUniform"),
    ("doubleMin", "dmin", "minFloatZipf"), ("doubleMax", "dmax", "sumFloatNormal"), ("floatMin", "fmin", "sumFloatNormal"),
    ("floatMax", "fmax", "minFloatZipf"),
]


def _aggs(Q, which=None):
    out = []
    for t, n, f in ALL_AGGS:
        if which is None or n in which:
            out.append(Q.AggregatorFactory(t, n, f))
    return out


LAYOUTS = [("concise", "lz4"), ("roaring", "lz4"), ("concise", "uncompressed"), ("roaring", "none")]


@pytest.mark.parametrize("layout", LAYOUTS)
def test_filter_bitmaps_match_oracle(Q, O, gpu_basic, oracle_basic, layout):
    for gs, os_ in zip(gpu_basic[layout], oracle_basic[layout]):
        for f in _filters(Q):
            if f is None:
                continue
            words, cnt = gs.filter_bitmap(f.optimize(), Q)
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:gs.num_rows].astype(bool)
            exp = O.filter_mask(os_, f.optimize())
            assert cnt == int(exp.sum()), f
            assert np.array_equal(bits, exp), f


@pytest.mark.parametrize("layout", LAYOUTS)
def test_timeseries_matches_oracle(R, Q, O, gpu_basic, oracle_basic, layout):
    for f in _filters(Q):
        q = Q.TimeseriesQuery(intervals=["1970-01-01/2020-01-01"], aggregations=_aggs(Q), filter=f)
        assert_results(q, R.run_query(q, gpu_basic[layout]), O.run(q, oracle_basic[layout]))


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("gran,interval,skip", [
    ("minute", "1970-01-01T00:00:00/1970-01-01T00:20:00", False),
    ("minute", "1970-01-01T00:02:30/1970-01-01T00:09:10", True),
    ({"type": "duration", "duration": 7777, "origin": "1970-01-01T00:00:00.123Z"}, "1970-01-01T00:00:01/1970-01-01T00:03:00", False),
    ("all", "1970-01-01T00:05:00/1970-01-01T00:06:00", False),
    ("second", "1970-01-01T00:00:10/1970-01-01T00:01:10", True),
    ("all", "2000-01-01/2001-01-01", False),
])
def test_timeseries_granularity_and_intervals(R, Q, O, gpu_basic, oracle_basic, layout, gran, interval, skip):
    for f in (None, Q.InDimFilter("dimZipf", ["1", "2"]), Q.SelectorDimFilter("dimSequential", "7")):
        q = Q.TimeseriesQuery(intervals=[interval], granularity=gran, aggregations=_aggs(Q), filter=f,
                              context={"skipEmptyBuckets": skip})
        assert_results(q, R.run_query(q, gpu_basic[layout]), O.run(q, oracle_basic[layout]))


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("dim,metric,inverted,threshold", [
    ("dimUniform", "ds", False, 10), ("dimUniform", "ls", False, 10), ("dimZipf", "rows", False, 5),
    ("dimSequential", "lmax", False, 3), ("dimSequential", "dmin", True, 7), ("dimZipf", "fs", False, 200),
    ("dimSequentialHalfNull", "ls", True, 4), ("missingDim", "rows", False, 3), ("dimUniform", "fmax", False, 1001),
])
def test_topn_matches_oracle(R, Q, O, gpu_basic, oracle_basic, layout, dim, metric, inverted, threshold):
    spec = {"type": "inverted", "metric": {"type": "numeric", "metric": metric}} if inverted else metric
    for f in (None, Q.BoundDimFilter("dimSequential", "100", "200")):
        q = Q.TopNQuery(intervals=["1970-01-01/2020-01-01"], dimension=dim, metric=spec, threshold=threshold,
                        aggregations=_aggs(Q), filter=f)
        assert_results(q, R.run_query(q, gpu_basic[layout]), O.run(q, oracle_basic[layout]))


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("dims,gran", [
    (["dimZipf"], "all"), (["dimZipf", "dimSequential"], "all"), (["dimUniform", "dimHyperUnique"], "all"),
    (["dimSequentialHalfNull"], "minute"), (["dimZipf", "missingDim"], "all"), ([], "minute"),
])
def test_groupby_matches_oracle(R, Q, O, gpu_basic, oracle_basic, layout, dims, gran):
    for f in (None, Q.NotDimFilter(Q.SelectorDimFilter("dimZipf", "1"))):
        q = Q.GroupByQuery(intervals=["1970-01-01/2020-01-01"], granularity=gran, dimensions=dims,
                           aggregations=_aggs(Q), filter=f)
        assert_results(q, R.run_query(q, gpu_basic[layout]), O.run(q, oracle_basic[layout]))


def test_integer_results_deterministic(R, Q, gpu_basic):
    q = Q.TopNQuery(intervals=["1970-01-01/2020-01-01"], dimension="dimUniform", metric="ls", threshold=50,
                    aggregations=_aggs(Q, {"rows", "ls", "lmin", "lmax"}))
    a = R.run_query(q, gpu_basic[("concise", "lz4")])
    b = R.run_query(q, gpu_basic[("concise", "lz4")])
    assert a[0].value == b[0].value


def test_per_segment_runner_and_merge(R, Q, O, gpu_basic, oracle_basic):
    """createRunner per segment + toolchest merge == mergeRunners batched call."""
    q = Q.TimeseriesQuery(intervals=["1970-01-01/2020-01-01"], granularity="minute", aggregations=_aggs(Q))
    f = R.TimeseriesQueryRunnerFactory()
    per = [f.createRunner(s).run(q) for s in gpu_basic[("concise", "lz4")]]
    merged = R.merge_timeseries(q, per)
    assert_results(q, merged, O.run(q, oracle_basic[("concise", "lz4")]))


def _pattern_columns(n, rng):
    """Long/double columns that stress every LZ4 token shape (long literal runs, offset-1 runs,
    short periodic matches, token-dense sequences, incompressible data, mixtures)."""
    seq = np.arange(n, dtype=np.int64)
    spikes = np.zeros(n, dtype=np.int64)
    spikes[rng.integers(0, n, n // 500)] = rng.integers(1, 1 << 40, n // 500)
    mixed = np.where((seq // 3000) % 2 == 0, rng.integers(-(1 << 62), 1 << 62, n), seq % 7)
    return {
        "zeros": ("long", np.zeros(n, dtype=np.int64)),
        "const": ("long", np.full(n, 0x0102030405060708, dtype=np.int64)),
        "seq": ("long", seq % 10000),
        "period3": ("long", seq % 3),
        "random": ("long", rng.integers(-(1 << 62), 1 << 62, n)),
        "spikes": ("long", spikes),
        "mixed": ("long", mixed),
        "dbl": ("double", rng.normal(5000.0, 1.0, n)),
        "dblround": ("double", np.round(rng.normal(100.0, 10.0, n), 1)),
    }


@pytest.mark.parametrize("mode", ["hc", "fast"])
def test_lz4_every_value_round_trips(R, Q, O, S, W, tmp_path, mode):
    """Per-row buckets (1 ms granularity) make every decoded value visible: bit-exact vs the oracle."""
    rng = np.random.default_rng(7)
    n = 70_000  # > 8 blocks of longs, partial last block
    metrics = _pattern_columns(n, rng)
    spec = W.SegmentSpec(timestamps=np.arange(n, dtype=np.int64),
                         dims={"d": W.encode_int_strings(rng.integers(0, 300, n))}, metrics=metrics)
    p = W.write_segment(str(tmp_path / f"pat_{mode}"), spec, compression="lz4", lz4_mode=mode)
    g, o = S.GpuSegment(p), O.OracleSegment(p)
    aggs = [Q.long_sum(k, k) for k, (t, _) in metrics.items() if t == "long"] + \
           [Q.double_max(k, k) for k, (t, _) in metrics.items() if t == "double"]
    for chunk in range(0, len(aggs), 8):
        q = Q.TimeseriesQuery(intervals=[(0, n)], granularity={"type": "duration", "duration": 1},
                              aggregations=aggs[chunk:chunk + 8])
        got, exp = R.run_query(q, [g]), O.run(q, [o])
        assert len(got) == n
        assert_results(q, got, exp)
    q = Q.GroupByQuery(intervals=[(0, n)], dimensions=["d"], aggregations=[Q.count("rows"), Q.long_sum("seq")])
    assert_results(q, R.run_query(q, [g]), O.run(q, [o]))
