"""Dictionary-id widths: CompressedVSizeColumnarIntsSupplier reads 1/2/3-byte ids
through its VSize path and numBytes == Integer.BYTES through the full-int specialization
(data/CompressedVSizeColumnarIntsSupplier.java:108-122: 4-byte ids, 16384 per block, :254-353), and
VSizeColumnarInts the same widths big-endian (VSizeColumnarInts.java:124-127). The Java writer picks
numBytes from the cardinality (getNumBytesForMax), so a 4-byte column needs > 16.7 M values; the
format is the same for a small dictionary, which the writer here emits on request (id_bytes).

CPU: the oracle's restatement reads every width back to the ids written.
GPU: filters (bitmap + the id predicate of topN/groupBy keys), timeseries, topN and groupBy on
columns of every width through the C-ABI, equal to the oracle."""
import importlib

import numpy as np
import pytest

from compare import assert_results

WIDTHS = [None, 3, 4]  # None: numBytes by cardinality (2 bytes for a, 1 byte for b)


def _spec(W, n, seed):
    rng = np.random.default_rng(seed)
    ts = np.sort(rng.integers(0, 6 * 3_600_000, n)).astype(np.int64)
    a = rng.integers(0, 300, n)          # 300 values: numBytes 2 by cardinality
    b = rng.zipf(1.3, n) % 50            # skewed, 50 values
    return W.SegmentSpec(timestamps=ts,
                         dims={"a": W.encode_int_strings(a), "b": W.encode_int_strings(b)},
                         metrics={"m": ("long", rng.integers(-1000, 1000, n)), "x": ("double", rng.normal(3, 1, n))})


def _write(W, path, width, comp, seed, n=70_000):
    return W.write_segment(path, _spec(W, n, seed), bitmap="concise" if seed % 2 else "roaring",
                           compression=comp, lz4_mode="fast", id_bytes=width)


@pytest.mark.parametrize("comp", ["lz4", "uncompressed"])
@pytest.mark.parametrize("width", WIDTHS)
def test_oracle_reads_every_id_width(O, W, tmp_path, width, comp):
    spec = _spec(W, 70_000, 5)
    p = W.write_segment(str(tmp_path / "s"), spec, compression=comp, lz4_mode="fast", id_bytes=width)
    o = O.OracleSegment(p)
    for d in ("a", "b"):
        assert np.array_equal(o.ids(d), spec.dims[d][1]), (d, width)
        assert o.dictionary(d) == spec.dims[d][0]


@pytest.mark.gpu
@pytest.mark.parametrize("comp", ["lz4", "uncompressed"])
@pytest.mark.parametrize("width", WIDTHS)
def test_gpu_id_widths(Q, O, W, tmp_path, width, comp):
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")
    paths = [_write(W, str(tmp_path / f"s{i}"), width, comp, seed=11 + i) for i in range(2)]
    g = [S.GpuSegment(p) for p in paths]
    o = [O.OracleSegment(p) for p in paths]
    aggs = [Q.count("rows"), Q.long_sum("m", "m"), Q.AggregatorFactory("doubleSum", "x", "x"),
            Q.AggregatorFactory("longMax", "mx", "m")]
    iv = [(0, 1 << 40)]
    filters = [None, Q.SelectorDimFilter("a", "17"), Q.InDimFilter("b", ["1", "2", "40"]),
               Q.BoundDimFilter("a", "100", "200", False, True),
               Q.OrDimFilter([Q.SelectorDimFilter("b", "3"), Q.NotDimFilter(Q.BoundDimFilter("a", "1", "5"))])]
    for f in filters:
        if f is not None:
            for gs, os_ in zip(g, o):
                words, cnt = gs.filter_bitmap(f.optimize(), Q)
                bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:gs.num_rows].astype(bool)
                exp = O.filter_mask(os_, f.optimize())
                assert cnt == int(exp.sum()) and np.array_equal(bits, exp), (f, width)
        for q in (Q.TimeseriesQuery(intervals=iv, granularity="hour", aggregations=aggs, filter=f),
                  Q.TopNQuery(intervals=iv, dimension="a", metric="x", threshold=7, aggregations=aggs, filter=f),
                  Q.TopNQuery(intervals=iv, dimension="b", metric={"type": "dimension", "ordering": "numeric"},
                              threshold=5, aggregations=aggs, filter=f),
                  Q.GroupByQuery(intervals=iv, dimensions=["a", "b"], aggregations=aggs, filter=f),
                  Q.GroupByQuery(intervals=iv, dimensions=["b"], granularity="hour", aggregations=aggs, filter=f)):
            assert_results(q, R.run_query(q, g), O.run(q, o))
            assert_results(q, R.run_query(q, g[:1]), O.run(q, o[:1]))
