"""FilteredAggregatorFactory (per-aggregator row matchers) and the predicate filters resolved over
dictionaries (regex, search, like, alphanumeric / strlen bounds) on the GPU, against the oracle, in
all three engines. Integer aggregates bit-exact, doubleSum 1e-9, floatSum 1e-5 (tests/compare.py)."""
import importlib

import pytest

from compare import assert_results

pytestmark = pytest.mark.gpu

ALL = ["1970-01-01/2020-01-01"]
LAYOUTS = [("concise", "lz4"), ("roaring", "none"), ("concise", "uncompressed")]


@pytest.fixture(scope="module")
def R():
    return importlib.import_module("incubator-druid_amd.runners")


@pytest.fixture(scope="module")
def S():
    return importlib.import_module("incubator-druid_amd.segment")


@pytest.fixture(scope="module")
def basic(S, O, basic_dirs):
    return {k: ([S.GpuSegment(p) for p in basic_dirs[k]], [O.OracleSegment(p) for p in basic_dirs[k]]) for k in LAYOUTS}


def _filters(Q):
    return [
        Q.SelectorDimFilter("dimZipf", "3"),
        Q.NotDimFilter(Q.SelectorDimFilter("dimSequential", "7")),
        Q.SelectorDimFilter("missingDim", None),
        Q.SelectorDimFilter("missingDim", "x"),
        Q.InDimFilter("dimZipf", ["1", "2", "nope"]),
        Q.BoundDimFilter("dimSequential", "100", "200", True, False),
        Q.BoundDimFilter("dimUniform", "50", "5000", False, True, "numeric"),
        Q.BoundDimFilter("dimSequential", "5", "50", False, True, "alphanumeric"),
        Q.BoundDimFilter("dimZipf", None, "2", False, False, "strlen"),
        Q.RegexDimFilter("dimSequential", "^1.?5$"),
        Q.SearchQueryDimFilter("dimUniform", {"type": "contains", "value": "777"}),
        Q.SearchQueryDimFilter("dimSequentialHalfNull", {"type": "fragment", "values": ["1", "2"]}),
        Q.LikeDimFilter("dimSequential", "9%"),
        Q.LikeDimFilter("dimSequentialHalfNull", "_0"),
        Q.OrDimFilter([Q.RegexDimFilter("dimZipf", "^9"), Q.LikeDimFilter("missingDim", "%")]),
    ]


def _aggs(Q, flt):
    return [Q.count("rows"),
            Q.filtered(Q.count("frows"), flt),
            Q.filtered(Q.long_sum("fls", "sumLongSequential"), flt),
            Q.filtered(Q.double_sum("fds", "sumFloatNormal"), flt),
            Q.filtered(Q.float_sum("ffs", "sumFloatNormal"), flt),
            Q.filtered(Q.long_max("flmax", "maxLongUniform"), flt),
            Q.filtered(Q.double_min("fdmin", "minFloatZipf"), flt),
            Q.double_sum("ds", "sumFloatNormal")]


@pytest.mark.parametrize("layout", LAYOUTS)
def test_filtered_aggregators_timeseries(R, Q, O, basic, layout):
    g, o = basic[layout]
    for i, flt in enumerate(_filters(Q)):
        for gran in (("all", "minute") if i % 5 == 0 else ("all",)):
            q = Q.TimeseriesQuery(intervals=ALL, granularity=gran, aggregations=_aggs(Q, flt),
                                  filter=Q.NotDimFilter(Q.SelectorDimFilter("dimZipf", "5")))
            assert_results(q, R.run_query(q, g), O.run(q, o))


@pytest.mark.parametrize("layout", LAYOUTS[:2])
def test_filtered_aggregators_topn_groupby(R, Q, O, basic, layout):
    g, o = basic[layout]
    for flt in _filters(Q)[::3]:
        q = Q.TopNQuery(intervals=ALL, dimension="dimZipf", metric="fds", threshold=7, aggregations=_aggs(Q, flt))
        assert_results(q, R.run_query(q, g), O.run(q, o))
        q = Q.TopNQuery(intervals=ALL, dimension="dimUniform", metric="frows", threshold=5, aggregations=_aggs(Q, flt))
        assert_results(q, R.run_query(q, g), O.run(q, o))
        q = Q.GroupByQuery(intervals=ALL, dimensions=["dimZipf"], aggregations=_aggs(Q, flt))
        assert_results(q, R.run_query(q, g), O.run(q, o))


@pytest.mark.parametrize("layout", LAYOUTS)
def test_predicate_filters_as_query_filters(R, Q, O, basic, layout):
    g, o = basic[layout]
    aggs = [Q.count("rows"), Q.long_sum("ls", "sumLongSequential"), Q.double_sum("ds", "sumFloatNormal")]
    for flt in _filters(Q)[7:]:
        q = Q.TimeseriesQuery(intervals=ALL, aggregations=aggs, filter=flt)
        assert_results(q, R.run_query(q, g), O.run(q, o))
        words, cnt = g[0].filter_bitmap(flt, Q)
        mask = O.filter_mask(o[0], flt)
        assert cnt == int(mask.sum())
        q = Q.GroupByQuery(intervals=ALL, dimensions=["dimZipf"], aggregations=aggs, filter=flt)
        assert_results(q, R.run_query(q, g), O.run(q, o))


def test_filtered_aggregator_benchmark_shape(R, Q, O, basic):
    """FilteredAggregatorBenchmark's filter (benchmarks/.../FilteredAggregatorBenchmark.java:163-178)
    minus its JavaScript leg: OR(alphanumeric bound, regex, search contains, in) around a count."""
    g, o = basic[("concise", "lz4")]
    flt = Q.OrDimFilter([
        Q.BoundDimFilter("dimSequential", "-1", "-1", True, True, "alphanumeric"),
        Q.RegexDimFilter("dimSequential", "X"),
        Q.SearchQueryDimFilter("dimSequential", {"type": "contains", "value": "X", "caseSensitive": False}),
        Q.InDimFilter("dimSequential", ["X"]),
    ])
    q = Q.TimeseriesQuery(intervals=ALL, aggregations=[Q.filtered(Q.count("rows"), flt)])
    got = R.run_query(q, g)
    assert_results(q, got, O.run(q, o))
    assert got[0].value["rows"] == 0
