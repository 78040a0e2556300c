"""groupBy limit push-down: GroupByQuery.isApplyLimitPushDown
(query/groupby/GroupByQuery.java:377-416) and LimitedBufferHashGrouper's outcome — the first `limit`
groups in the push-down row order (getRowOrderingForPushDown :423-528) — applied on the device by
dg_result_limit (re-packed keys, radix sort, gather of the first `limit` groups).

GPU: engine queries whose limit is pushed down against the oracle (its groupBy merge followed by its
own DefaultLimitSpec restatement, oracle.groupby_post_process), with the device result checked to hold
exactly min(limit, groups) groups; the same through the two-rank exchange (each rank keeps its key
range's first `limit`). CPU: the push-down decision table."""
import ctypes
import importlib

import numpy as np
import pytest

from compare import assert_results


def _aggs(Q):
    return [Q.count("rows"), Q.long_sum("ls", "sumLongSequential"), Q.AggregatorFactory("doubleSum", "ds", "sumFloatNormal"),
            Q.float_sum("fs", "sumFloatNormal")]


SPECS = [
    {"type": "default", "columns": ["dimZipf"], "limit": 7},
    {"type": "default", "limit": 13},
    {"type": "default", "columns": [{"dimension": "dimSequential", "direction": "descending", "dimensionOrder": "numeric"}],
     "limit": 25},
    {"type": "default", "columns": [{"dimension": "dimSequentialHalfNull", "direction": "descending"},
                                    {"dimension": "dimZipf", "dimensionOrder": "strlen"}], "limit": 40},
    {"type": "default", "columns": [{"dimension": "dimZipf", "dimensionOrder": "alphanumeric", "direction": "descending"},
                                    {"dimension": "dimSequential", "direction": "ascending"}], "limit": 1_000_000},
]
GRANS = [("all", False), ({"type": "period", "period": "PT1M"}, False), ({"type": "period", "period": "PT1M"}, True)]


def _query(Q, spec, gran, by_dims_first, dims=("dimZipf", "dimSequential", "dimSequentialHalfNull"), ctx=None):
    c = dict(ctx or {})
    if by_dims_first:
        c["sortByDimsFirst"] = True
    return Q.GroupByQuery(intervals=[(0, 1 << 42)], granularity=gran, dimensions=list(dims), aggregations=_aggs(Q),
                          limitSpec=spec, context=c,
                          filter=Q.BoundDimFilter("dimSequential", "0", "3000", ordering="numeric"))


def test_push_down_decision(Q):
    """determineApplyLimitPushDown / validateAndGetForceLimitPushDown (GroupByQuery.java:352-416)."""
    mk = lambda ls, having=None, ctx=None: Q.GroupByQuery(intervals=[(0, 1)], dimensions=["a", "b"],
                                                          aggregations=[Q.count("rows")], limitSpec=ls, having=having,
                                                          context=ctx or {})
    assert mk({"type": "default", "limit": 3}).apply_limit_push_down()
    assert mk({"type": "default", "columns": ["b", {"dimension": "a", "direction": "desc"}], "limit": 3}).apply_limit_push_down()
    assert not mk({"type": "default", "columns": ["a"]}).apply_limit_push_down()  # no limit
    assert not mk(None).apply_limit_push_down()
    assert not mk({"type": "default", "columns": ["rows"], "limit": 3}).apply_limit_push_down()  # aggregator ordering
    assert not mk({"type": "default", "limit": 3}, having={"type": "always"}).apply_limit_push_down()
    assert not mk({"type": "default", "limit": 3}, ctx={"applyLimitPushDown": False}).apply_limit_push_down()
    assert not mk({"type": "default", "limit": 3}, ctx={"applyLimitPushDown": "false"}).apply_limit_push_down()
    assert mk({"type": "default", "limit": 3}, ctx={"applyLimitPushDown": False, "forceLimitPushDown": True}).apply_limit_push_down()
    with pytest.raises(ValueError):
        mk({"type": "default", "columns": ["a"]}, ctx={"forceLimitPushDown": True}).apply_limit_push_down()
    with pytest.raises(ValueError):
        mk({"type": "default", "limit": 2}, having={"type": "always"}, ctx={"forceLimitPushDown": True}).apply_limit_push_down()


@pytest.fixture(scope="module")
def segs(basic_dirs):
    S = importlib.import_module("incubator-druid_amd.segment")
    return [S.GpuSegment(p) for p in basic_dirs[("concise", "lz4")]]


@pytest.fixture(scope="module")
def osegs(basic_dirs, O):
    return [O.OracleSegment(p) for p in basic_dirs[("concise", "lz4")]]


def _full_groups(R, Q, segs, gran):
    r = R.groupby_run(segs, _query(Q, None, gran, False))
    try:
        return r.groups
    finally:
        r.release()


@pytest.mark.gpu
@pytest.mark.parametrize("gran,by_dims_first", GRANS, ids=["all", "PT1M", "PT1M-dims-first"])
def test_limit_push_down_matches_oracle(Q, O, segs, osegs, gran, by_dims_first):
    R = importlib.import_module("incubator-druid_amd.runners")
    total = None
    for spec in SPECS:
        q = _query(Q, spec, gran, by_dims_first)
        assert q.apply_limit_push_down()
        res = R.groupby_run(segs, q, limit_push_down=True)
        try:
            if total is None:
                total = _full_groups(R, Q, segs, gran)
            assert res.groups == min(spec["limit"], total)
        finally:
            res.release()
        got, exp = R.run_query(q, segs), O.run(q, osegs)
        assert len(got) == min(spec["limit"], total)
        assert [(r.timestamp, tuple(r.event[d] for d in q.dimensions)) for r in got] == \
               [(r.timestamp, tuple(r.event[d] for d in q.dimensions)) for r in exp], spec
        assert_results(q, got, exp)
        # switched off in the context: all groups through the host post-processing. The same rows
        # where the push-down order refines the final one (time first); with sortByDimsFirst the
        # reference's two paths differ (the push-down cut is taken over dimensions, then time)
        q_off = _query(Q, spec, gran, by_dims_first, ctx={"applyLimitPushDown": False})
        assert not q_off.apply_limit_push_down()
        exp_off = O.run(q_off, osegs)
        assert_results(q_off, R.run_query(q_off, segs), exp_off)
        if not by_dims_first:
            assert_results(q_off, exp_off, exp)


@pytest.mark.gpu
def test_limit_push_down_two_rank_exchange(Q, O, segs, osegs):
    """Each rank's key range after the exchange holds whole groups; its first `limit` are kept, and the
    cluster's first `limit` are among them."""
    import test_merge_gpu as TM
    R = importlib.import_module("incubator-druid_amd.runners")
    D = importlib.import_module("incubator-druid_amd.distributed")
    for spec in SPECS[:4]:
        q = _query(Q, spec, {"type": "period", "period": "PT1M"}, False)
        parts = TM._run_ranks(R, D, Q, [segs[:1], segs[1:]], q)
        assert all(len(p) <= spec["limit"] for p in parts)
        got = R.merge_groupby(q, parts)
        exp = O.run(q, osegs)
        assert [tuple(r.event[d] for d in q.dimensions) for r in got] == [tuple(r.event[d] for d in q.dimensions) for r in exp]
        assert_results(q, got, exp)


@pytest.mark.gpu
def test_limit_abi_errors(Q, segs):
    R = importlib.import_module("incubator-druid_amd.runners")
    N = importlib.import_module("incubator-druid_amd._native")
    q = _query(Q, None, "all", False)
    res = R.groupby_run(segs, q)
    try:
        card = int(N.lib().dg_result_dim_cardinality(res.handle, 0))
        bad = np.full(card, card, np.int32)  # ranks must lie in [0, card)
        col = (N.dg_order_column * 1)(N.dg_order_column(0, 0, bad.ctypes.data))
        lim = N.dg_limit(ctypes.cast(col, ctypes.c_void_p), 1, 5, 0)
        assert N.lib().dg_result_limit(res.handle, ctypes.byref(lim)) == 6  # DG_ERR_ARG
        col = (N.dg_order_column * 1)(N.dg_order_column(7, 0, None))
        lim = N.dg_limit(ctypes.cast(col, ctypes.c_void_p), 1, 5, 0)
        assert N.lib().dg_result_limit(res.handle, ctypes.byref(lim)) == 6
        lim = N.dg_limit(None, 0, 0, 0)
        assert N.lib().dg_result_limit(res.handle, ctypes.byref(lim)) == 6  # limit must be > 0
        lim = N.dg_limit(None, 0, 5, 0)
        assert N.lib().dg_result_limit(res.handle, ctypes.byref(lim)) == 0
        assert N.lib().dg_result_groups(res.handle) == 5
        # a limited result is no longer in key order: the exchange's export refuses it
        ks = N.dg_keyspace()
        assert N.lib().dg_result_export(res.handle, ctypes.byref(ks), None, None, None) == 6
    finally:
        res.release()
