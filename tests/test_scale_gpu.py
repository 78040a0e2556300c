"""Parity at the BASELINE shapes (the benchmarks' own data, not 40k-row toys):

* config 2: topN over dimUniform (~100k values -> 3-byte dictionary ids, 16,384 rows per block,
  CompressedVSizeColumnarIntsSupplier.java:82-101) on 4 x 750k-row LZ4-HC segments;
* config 3: groupBy dimUniform x dimHyperUnique, both 3-byte ids, ~1 group per row, merged over
  segments with different dictionaries (GroupByMergingQueryRunnerV2 merge by value);
* floatSum at 750k rows per segment, where the reference's own float32 row-order recurrence
  (FloatSumAggregator.java:47-59) has drifted ~1e-2 from the exact sum: the engine must follow the
  recurrence (bitwise equal here), not a more accurate tree sum;
* config 4: compound AND/OR/NOT filters on >= 200k-row Roaring segments (multi-container bitmaps,
  run containers) and Concise, bit-exact row selections.

Every comparison is against the CPU oracle on the same segment bytes; integer results and row
selections bit-exact, doubleSum 1e-9 relative, floatSum bitwise (tests/compare.py tolerances)."""
import importlib
import math

import numpy as np
import pytest

from compare import TOL, assert_results

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R():
    return importlib.import_module("incubator-druid_amd.runners")


@pytest.fixture(scope="module")
def S():
    return importlib.import_module("incubator-druid_amd.segment")


@pytest.fixture(scope="module")
def cfg2(tmp_path_factory, DG, S, O):
    """TopNBenchmark 'basic': 4 segments x 750,000 rows, seeds 9999 + i, LZ4-HC, Concise."""
    paths = DG.write_basic_dataset(str(tmp_path_factory.mktemp("cfg2")), 4, 750_000, lz4_mode="hc")
    return [S.GpuSegment(p) for p in paths], [O.OracleSegment(p) for p in paths]


IV = ["1970-01-01/2020-01-01"]


def test_cfg2_ids_are_three_bytes(W, cfg2):
    g, o = cfg2
    for s in o:
        card = s.cardinality("dimUniform")
        assert card > 65_535
        assert W.num_bytes_for_max(card - 1) == 3  # VSizeColumnarInts.getNumBytesForMax


@pytest.mark.parametrize("name", ["topn", "topn_numeric", "topn_alphanumeric", "topn_floatsum"])
def test_cfg2_topn_matches_oracle(R, Q, O, cfg2, name):
    g, o = cfg2
    aggs = [Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")]
    if name == "topn":
        q = Q.TopNQuery(intervals=IV, dimension="dimUniform", metric="sumFloatNormal", threshold=10, aggregations=aggs)
    elif name == "topn_floatsum":
        q = Q.TopNQuery(intervals=IV, dimension="dimUniform", metric="fsum", threshold=25,
                        aggregations=aggs + [Q.float_sum("fsum", "sumFloatNormal")])
    else:
        q = Q.TopNQuery(intervals=IV, dimension="dimUniform", threshold=10, aggregations=aggs[:1],
                        metric={"type": "dimension", "ordering": name.split("_")[1], "previousStop": None})
    assert_results(q, R.run_query(q, g), O.run(q, o))


@pytest.mark.parametrize("no_index", ["0", "1"])
def test_cfg2_topn_bin_index(R, Q, O, S, cfg2, no_index, monkeypatch):
    """topN by the dimension's cached bin index (the first call over fresh segments builds it from the
    decoded ids, the later ones reuse it without decoding the ids) and by the per-call bins
    (DG_NO_TOPN_INDEX=1): numeric, inverted and dimension-ordered metrics, a filter, an interval that
    cuts the segments, a segment listed twice, a topN over a second dimension — against the oracle."""
    monkeypatch.setenv("DG_NO_TOPN_INDEX", no_index)
    g0, o = cfg2
    g = [S.GpuSegment(s.path) for s in g0]  # fresh segments: no index yet
    aggs = [Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal"), Q.count("rows")]
    qs = [Q.TopNQuery(intervals=IV, dimension="dimUniform", metric="sumFloatNormal", threshold=10, aggregations=aggs),
          Q.TopNQuery(intervals=IV, dimension="dimUniform", metric="sumLongSequential", threshold=10, aggregations=aggs),
          Q.TopNQuery(intervals=IV, dimension="dimUniform", threshold=7, aggregations=aggs,
                      metric={"type": "inverted", "metric": {"type": "numeric", "metric": "rows"}}),
          Q.TopNQuery(intervals=IV, dimension="dimUniform", threshold=10, aggregations=aggs[:1],
                      metric={"type": "dimension", "ordering": "numeric", "previousStop": None}),
          Q.TopNQuery(intervals=IV, dimension="dimUniform", metric="sumFloatNormal", threshold=10, aggregations=aggs,
                      filter=Q.BoundDimFilter("dimSequential", "100", "500")),
          Q.TopNQuery(intervals=["1970-01-01T00:02/1970-01-01T00:09"], dimension="dimUniform", metric="rows",
                      threshold=10, aggregations=aggs),
          Q.TopNQuery(intervals=IV, dimension="dimZipf", metric="sumFloatNormal", threshold=10, aggregations=aggs)]
    before = [s.device_bytes() for s in g]
    try:
        for rnd in range(2):  # build, then reuse
            for q in qs:
                assert_results(q, R.run_query(q, g), O.run(q, o))
        # the indexes (dimUniform, dimZipf: 6 B per row + the bin starts each) count toward the footprint
        for s, b in zip(g, before):
            grown = s.device_bytes() - b
            assert grown == 0 if no_index == "1" else 2 * 6 * s.num_rows <= grown <= 2 * 6 * s.num_rows + (1 << 20)
        q = qs[0]
        assert_results(q, R.run_query(q, [g[0], g[1], g[0]]), O.run(q, [o[0], o[1], o[0]]))
    finally:
        for s in g:
            s.close()


def test_cfg2_floatsum_follows_the_reference_recurrence(R, Q, O, cfg2):
    """750k rows of N(5000, 1) per segment: the float32 row-order sum is off the exact sum by
    ~1e-2, far outside 1e-5 — the engine matches the reference's recurrence bit for bit."""
    g, o = cfg2
    q = Q.TimeseriesQuery(intervals=IV, aggregations=[Q.float_sum("fsum", "sumFloatNormal"),
                                                       Q.double_sum("dsum", "sumFloatNormal"), Q.count("rows")])
    got, exp = R.run_query(q, g), O.run(q, o)
    assert np.float32(got[0].value["fsum"]) == np.float32(exp[0].value["fsum"])
    exact = math.fsum(float(x) for s in o for x in s.numeric("sumFloatNormal", "double").astype(np.float32))
    drift = abs(exp[0].value["fsum"] - exact) / exact
    assert drift > 100 * TOL["float"], drift  # the reason a tree sum would fail parity here
    assert_results(q, got, exp)
    # per-segment runners (one cursor each) and groupBy / topN cells of the same column
    for s_g, s_o in zip(g, o):
        a, b = R.run_query(q, [s_g]), O.run(q, [s_o])
        assert np.float32(a[0].value["fsum"]) == np.float32(b[0].value["fsum"])
    qg = Q.GroupByQuery(intervals=IV, dimensions=["dimZipf"],
                        aggregations=[Q.float_sum("fsum", "sumFloatNormal"), Q.count("rows")])
    got_g, exp_g = R.run_query(qg, g), O.run(qg, o)
    assert len(got_g) == len(exp_g)
    for a, b in zip(got_g, exp_g):
        assert a.event["dimZipf"] == b.event["dimZipf"] and a.event["rows"] == b.event["rows"]
        assert np.float32(a.event["fsum"]) == np.float32(b.event["fsum"]), a.event
    qt = Q.TopNQuery(intervals=IV, dimension="dimZipf", metric="fsum", threshold=20,
                     aggregations=[Q.float_sum("fsum", "sumFloatNormal"), Q.count("rows")])
    got_t, exp_t = R.run_query(qt, g), O.run(qt, o)
    assert [e["dimZipf"] for e in got_t[0].value] == [e["dimZipf"] for e in exp_t[0].value]
    for a, b in zip(got_t[0].value, exp_t[0].value):
        assert np.float32(a["fsum"]) == np.float32(b["fsum"])


@pytest.fixture(scope="module")
def cfg3(tmp_path_factory, DG, S, O):
    """Two 600k-row segments: dimUniform (~100k values) x dimHyperUnique (row % 100000), both 3-byte
    ids; different seeds give different dimUniform dictionaries (the merge remaps ids)."""
    base = tmp_path_factory.mktemp("cfg3")
    paths = DG.write_basic_dataset(str(base), 2, 600_000, lz4_mode="hc")
    return [S.GpuSegment(p) for p in paths], [O.OracleSegment(p) for p in paths]


def _columns(rows, dims, aggs):
    t = np.array([r.timestamp for r in rows], dtype=np.int64)
    keys = [tuple(r.event[d] for d in dims) for r in rows]
    vals = {a.name: np.array([r.event[a.name] for r in rows]) for a in aggs}
    return t, keys, vals


@pytest.mark.parametrize("status", ["narrow", "wide"])
def test_cfg3_groupby_high_cardinality_matches_oracle(R, Q, O, cfg3, status, monkeypatch):
    """1.2 M groups vs the oracle, with the radix look-back status in 32-bit words (the default below
    2^30 elements) and in 64-bit words (DG_SORT_WIDE_STATUS=1, the path of larger calls)."""
    if status == "wide":
        monkeypatch.setenv("DG_SORT_WIDE_STATUS", "1")
    else:
        monkeypatch.delenv("DG_SORT_WIDE_STATUS", raising=False)
    g, o = cfg3
    assert g[0].dictionary("dimUniform") != g[1].dictionary("dimUniform")
    aggs = [Q.count("rows"), Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal"),
            Q.float_sum("fsum", "sumFloatNormal"), Q.AggregatorFactory("longMax", "lmax", "maxLongUniform"),
            Q.AggregatorFactory("doubleMin", "dmin", "minFloatZipf")]
    q = Q.GroupByQuery(intervals=IV, dimensions=["dimUniform", "dimHyperUnique"], aggregations=aggs)
    part = R.groupby_per_device(g, q)[0]
    exp = O.run(q, o)
    assert len(part) == len(exp) > 1_000_000
    t, keys, vals = _columns(exp, q.dimensions, aggs)
    assert np.array_equal(part.times, t)
    got_keys = list(zip(*[list(c) for c in part.dims]))
    assert got_keys == keys
    for a, col in zip(aggs, part.aggs):
        e = vals[a.name]
        if a.type == "doubleSum":
            assert np.allclose(col, e, rtol=TOL["double"], atol=0)
        elif a.type == "floatSum":
            assert np.array_equal(col.astype(np.float32), e.astype(np.float32))
        else:
            assert np.array_equal(col, e.astype(col.dtype)), a.name


@pytest.mark.parametrize("bitmap", ["roaring", "concise"])
def test_cfg4_compound_filters_on_large_segments(R, Q, O, S, DG, tmp_path_factory, bitmap):
    """>= 200k rows: every Roaring bitmap spans several 65,536-row containers; dimNull's and
    dimSequentialHalfNull's bitmaps are long runs (run containers / Concise fills)."""
    base = tmp_path_factory.mktemp(f"cfg4_{bitmap}")
    paths = DG.write_basic_dataset(str(base), 2, 230_000, bitmap=bitmap, lz4_mode="fast")
    g, o = [S.GpuSegment(p) for p in paths], [O.OracleSegment(p) for p in paths]
    filters = [
        Q.OrDimFilter([Q.AndDimFilter([Q.BoundDimFilter("dimSequential", "100", "200"),
                                       Q.InDimFilter("dimZipf", ["1", "2", "3"])]),
                       Q.SelectorDimFilter("dimUniform", "199"),
                       Q.NotDimFilter(Q.SelectorDimFilter("dimZipf", "7"))]),
        Q.AndDimFilter([Q.SelectorDimFilter("dimNull", None), Q.BoundDimFilter("dimUniform", "0", "100", True, True)]),
        Q.NotDimFilter(Q.SelectorDimFilter("dimSequentialHalfNull", None)),
        Q.OrDimFilter([Q.InDimFilter("dimUniform", [str(v) for v in range(1, 5000, 7)]),
                       Q.BoundDimFilter("dimHyperUnique", "99990", None)]),
    ]
    for gs, os_ in zip(g, o):
        for f in filters:
            words, cnt = gs.filter_bitmap(f.optimize(), Q)
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:gs.num_rows].astype(bool)
            exp = O.filter_mask(os_, f.optimize())
            assert cnt == int(exp.sum()) and np.array_equal(bits, exp), (bitmap, f)
    for f in filters:
        q = Q.TimeseriesQuery(intervals=IV, aggregations=[Q.count("rows"), Q.long_sum("sumLongSequential")], filter=f)
        assert_results(q, R.run_query(q, g), O.run(q, o))


@pytest.mark.parametrize("mode", ["inplace", "agg_filter", "interval", "phase_off", "no_side", "fetch_pinned",
                                  "fetch_staged", "flow_wgs_7", "per_block_run_first", "rows_elems",
                                  "rows_elems_counted"])
def test_cfg3_groupby_sort_paths(R, Q, O, cfg3, mode, monkeypatch):
    """The headline's shape through the keygen paths: longSum / doubleSum of plain LZ4 columns decoded
    straight into the payload records (row-ref mode) next to a floatSum the keygen writes; a
    FilteredAggregator (its column goes through the keygen, the other in place) with a row filter
    (sparse rows: references stay row indices); and an interval cutting the segments (the per-row
    time check path). Then the engine's run-time switches on the in-place path: phase timing off (the
    bench's timed steps: the side-stream payload decode must still be joined before the reduce), the
    payload decoded on the main stream (DG_NO_SIDE=1), the side stream's persistent flow decoder with
    7 workgroups (DG_FLOW_WGS=7: every workgroup decodes many blocks) or one workgroup per block after
    the run decoder (DG_FLOW_WGS=0, DG_GEN_FIRST=0: the round-5 placement), and the groups fetched into
    pinned host memory by the pack kernel (zero-copy) or through the staged DMA copy (DG_FETCH_ZC=0);
    without the floatSum every row is an element and the keygen runs without its count pass (and with
    it, DG_GB_COUNT=1)."""
    N = importlib.import_module("incubator-druid_amd._native")
    if mode == "no_side":
        monkeypatch.setenv("DG_NO_SIDE", "1")
    if mode == "fetch_staged":
        monkeypatch.setenv("DG_FETCH_ZC", "0")
    if mode == "flow_wgs_7":
        monkeypatch.setenv("DG_FLOW_WGS", "7")
    if mode == "per_block_run_first":
        monkeypatch.setenv("DG_FLOW_WGS", "0")
        monkeypatch.setenv("DG_GEN_FIRST", "0")
    if mode == "rows_elems_counted":
        monkeypatch.setenv("DG_GB_COUNT", "1")
    g, o = cfg3
    aggs = [Q.count("rows"), Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal"),
            Q.float_sum("fsum", "sumFloatNormal")]
    if mode.startswith("rows_elems"):  # (no floatSum: every row an element, the keygen's count pass skipped)
        aggs = aggs[:3]
    iv, flt = IV, None
    if mode == "agg_filter":
        aggs[1] = Q.filtered(Q.long_sum("sumLongSequential"), Q.BoundDimFilter("dimHyperUnique", "2", "7"))
        flt = Q.NotDimFilter(Q.BoundDimFilter("dimUniform", "50000", "60000"))
    elif mode == "interval":
        ts = np.concatenate([s.time() for s in o])
        lo, hi = int(np.quantile(ts, 0.2)), int(np.quantile(ts, 0.7))
        iv = [(lo, hi)]
    q = Q.GroupByQuery(intervals=iv, dimensions=["dimUniform", "dimHyperUnique"], aggregations=aggs, filter=flt)
    pool = None
    if mode == "phase_off":
        N.lib().dg_set_phase_timing(0)
        try:
            for _ in range(2):  # (a second call: the first call's events are stale, not unrecorded)
                part = R.groupby_per_device(g, q)[0]
        finally:
            N.lib().dg_set_phase_timing(1)
    elif mode.startswith("fetch_"):
        pool = R.PinnedPool(len(o[0].time()) * 2 * (4 * 2 + 8 * len(aggs)) + (1 << 20))
        res = R.groupby_run(g, q)
        part = res.fetch(pool=pool)
        res.release()
    else:
        part = R.groupby_per_device(g, q)[0]
    exp = O.run(q, o)
    assert len(part) == len(exp) > 200_000
    t, keys, vals = _columns(exp, q.dimensions, aggs)
    assert np.array_equal(part.times, t)
    assert list(zip(*[list(c) for c in part.dims])) == keys
    for a, col in zip(aggs, part.aggs):
        e = vals[a.name]
        if a.type == "doubleSum":
            assert np.allclose(col, e, rtol=TOL["double"], atol=0)
        elif a.type == "floatSum":
            assert np.array_equal(col.astype(np.float32), e.astype(np.float32))
        else:
            assert np.array_equal(col, e.astype(col.dtype)), a.name
    if pool is not None:
        with pytest.raises(RuntimeError, match="still in use"):
            pool.close()  # the partial's arrays are views of the pool
        del part, col
        pool.close()


@pytest.mark.parametrize("switch", [("DG_NO_OVERLAP", "1"), ("DG_LIGHT_MAIN", "0"), ("DG_LIGHT_MAIN", "1"),
                                    ("DG_FLOW_WGS", "5"), ("DG_GEN_FIRST", "1")])
def test_cfg2_decoder_stream_switches(R, Q, O, cfg2, switch, monkeypatch):
    """The decoder stream placements of a timeseries / topN call: every decoder on the call's stream
    (DG_NO_OVERLAP=1), and the light blocks beside the run decoder on the side stream (DG_LIGHT_MAIN=0)
    or after the general decoder on the call's stream (=1, the default), the flow decoder as 5
    persistent workgroups (DG_FLOW_WGS=5) and launched before the run decoder (DG_GEN_FIRST=1), against
    the oracle."""
    monkeypatch.setenv(*switch)
    g, o = cfg2
    aggs = [Q.count("rows"), Q.long_sum("sumLongSequential"), Q.double_sum("sumFloatNormal")]
    for q in (Q.TopNQuery(intervals=IV, dimension="dimUniform", metric="sumFloatNormal", threshold=10,
                          aggregations=aggs[1:]),
              Q.TimeseriesQuery(intervals=IV, filter=Q.SelectorDimFilter("dimSequential", "399"), aggregations=aggs),
              Q.TimeseriesQuery(intervals=IV, granularity="minute", aggregations=aggs)):
        assert_results(q, R.run_query(q, g), O.run(q, o))


def test_cfg1_selector_timeseries_on_lz4_hc_segments(R, Q, O, cfg2):
    """BASELINE configs[0]'s exact query (TimeseriesBenchmark basic: SelectorDimFilter dimSequential =
    '399', count + longSum(sumLongSequential) + doubleSum(sumFloatNormal), ALL granularity) on the
    750k-row LZ4-HC segments of config 2, one by one and merged."""
    g, o = cfg2
    q = Q.TimeseriesQuery(intervals=IV, filter=Q.SelectorDimFilter("dimSequential", "399"),
                          aggregations=[Q.count("rows"), Q.long_sum("sumLongSequential"),
                                        Q.double_sum("sumFloatNormal")])
    for s_g, s_o in zip(g, o):
        got, exp = R.run_query(q, [s_g]), O.run(q, [s_o])
        assert exp[0].value["rows"] == 750  # every 1,000th row
        assert_results(q, got, exp)
    assert_results(q, R.run_query(q, g), O.run(q, o))


@pytest.mark.parametrize("bitmap", ["concise", "roaring"])
def test_cfg4_compound_filter_on_a_full_size_segment(R, Q, O, S, DG, tmp_path_factory, bitmap):
    """BASELINE configs[3]'s compound filter on one GPU's full 12.5M-row share (one segment, the
    filter's dimensions), bit-exact against the oracle's row selection, and its timeseries count."""
    base = tmp_path_factory.mktemp(f"cfg4full_{bitmap}")
    p = DG.write_basic_segment(str(base / "seg"), 12_500_000, seed=9999, bitmap=bitmap, lz4_mode="hc",
                               dims=["dimSequential", "dimZipf", "dimUniform"], metrics=["rows"])
    gs, os_ = S.GpuSegment(p), O.OracleSegment(p)
    f = Q.OrDimFilter([Q.AndDimFilter([Q.BoundDimFilter("dimSequential", "100", "200"),
                                       Q.InDimFilter("dimZipf", ["1", "2", "3"])]),
                       Q.SelectorDimFilter("dimUniform", "199"),
                       Q.NotDimFilter(Q.SelectorDimFilter("dimZipf", "7"))])
    words, cnt = gs.filter_bitmap(f.optimize(), Q)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:gs.num_rows].astype(bool)
    exp = O.filter_mask(os_, f.optimize())
    assert cnt == int(exp.sum()) and np.array_equal(bits, exp)
    q = Q.TimeseriesQuery(intervals=IV, aggregations=[Q.count("rows")], filter=f)
    assert_results(q, R.run_query(q, [gs]), O.run(q, [os_]))
