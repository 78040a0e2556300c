"""CPU: the multi-threaded C engine timed as bench.py's cpu_baseline (oracle/cpu_engine.c) against the
oracle's restatement, on small basic-schema segments (so the result checks that compare the GPU with
it rest on a checked reference): timeseries with bitmap filter programs and granularity buckets, topN
(PooledTopNAlgorithm per segment + TopNBinaryFn fold), groupBy with time buckets."""
import importlib
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


@pytest.fixture(scope="module")
def B():
    return importlib.import_module("bench")


def _segs(basic_dirs):
    return basic_dirs[("concise", "lz4")] + basic_dirs[("roaring", "lz4")][:1]


FILTERS = {
    "none": lambda Q: None,
    "selector": lambda Q: Q.SelectorDimFilter("dimSequential", "399"),
    "compound": lambda Q: Q.OrDimFilter([Q.AndDimFilter([Q.BoundDimFilter("dimSequential", "100", "200"),
                                                         Q.InDimFilter("dimZipf", ["1", "2", "3"])]),
                                         Q.SelectorDimFilter("dimUniform", "199"),
                                         Q.NotDimFilter(Q.SelectorDimFilter("dimZipf", "7"))]),
}


@pytest.mark.parametrize("flt", sorted(FILTERS))
@pytest.mark.parametrize("gran", ["all", "minute"])
def test_cpu_timeseries_matches_oracle(B, O, Q, basic_dirs, flt, gran):
    paths = _segs(basic_dirs)
    query = Q.TimeseriesQuery(intervals=["1970-01-01/2020-01-01"], granularity=gran, filter=FILTERS[flt](Q),
                              aggregations=[Q.count("rows"), Q.long_sum("sumLongSequential"),
                                            Q.double_sum("sumFloatNormal"), Q.long_max("maxLongUniform"),
                                            Q.double_min("minFloatZipf")])
    _, cres = B.cpu_baseline_timeseries(paths, query, 3)
    osegs = [O.OracleSegment(p) for p in paths]
    exp = O.run(query, osegs)
    for s in osegs:
        s.close()
    checks = B.check_timeseries(exp, cres, query)
    assert checks["per_bucket_equal"], checks


def test_cpu_topn_matches_oracle(B, O, Q, basic_dirs):
    paths = _segs(basic_dirs)
    query = Q.TopNQuery(intervals=["1970-01-01/2020-01-01"], dimension="dimUniform", metric="sumFloatNormal",
                        threshold=10, aggregations=[Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")])
    _, cres = B.cpu_baseline_topn(paths, query, 2)
    osegs = [O.OracleSegment(p) for p in paths]
    exp = O.run(query, osegs)
    for s in osegs:
        s.close()
    checks = B.check_topn(exp, cres, query)
    assert checks["per_entry_equal"] and checks["entries"] == 10, checks


@pytest.mark.parametrize("ordering", ["lexicographic", "alphanumeric", "numeric", "inverted_numeric"])
def test_cpu_topn_dimension_orders_match_oracle(B, O, Q, basic_dirs, ordering):
    """DimensionTopNMetricSpec orderings (TopNBenchmark's numericSort / alphanumericSort shapes, the
    LEXICOGRAPHIC optimizer's id cut, an InvertedTopNMetricSpec around NUMERIC) on the C engine vs the
    oracle."""
    paths = _segs(basic_dirs)
    spec = {"type": "dimension", "ordering": ordering.split("_")[-1], "previousStop": None}
    if ordering.startswith("inverted"):
        spec = {"type": "inverted", "metric": spec}
    query = Q.TopNQuery(intervals=["1970-01-01/2020-01-01"], dimension="dimUniform", metric=spec, threshold=10,
                        aggregations=[Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")])
    _, cres = B.cpu_baseline_topn(paths, query, 2)
    osegs = [O.OracleSegment(p) for p in paths]
    exp = O.run(query, osegs)
    for s in osegs:
        s.close()
    checks = B.check_topn(exp, cres, query)
    assert checks["per_entry_equal"] and checks["entries"] == 10, checks


@pytest.mark.parametrize("gran", ["all", "minute"])
def test_cpu_groupby_matches_oracle(B, O, Q, basic_dirs, gran):
    paths = _segs(basic_dirs)
    query = Q.GroupByQuery(intervals=["1970-01-01/2020-01-01"], granularity=gran, dimensions=["dimZipf", "dimSequential"],
                           aggregations=[Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")])
    cb = B.cpu_baseline_groupby(paths, query, 3, want_groups=True)
    g = cb["_groups"]
    osegs = [O.OracleSegment(p) for p in paths]
    exp = O.run(query, osegs)
    for s in osegs:
        s.close()
    org, per, b0, card1 = cb["_buckets"]
    m1 = {v: i for i, v in enumerate(cb["_dicts"][0])}
    m2 = {v: i for i, v in enumerate(cb["_dicts"][1])}
    keys, lsum, dsum = [], [], []
    for row in exp:
        b = (row.timestamp - org) // per - b0 if per else 0
        keys.append(((b * card1 + m1[row.event["dimZipf"]]) << 32) | m2[row.event["dimSequential"]])
        lsum.append(row.event["sumLongSequential"])
        dsum.append(row.event["sumFloatNormal"])
    assert list(g["key"]) == keys  # the same groups in the same (time, value) order
    assert list(g["lsum"]) == lsum
    np.testing.assert_allclose(g["dsum"], dsum, rtol=1e-9)
