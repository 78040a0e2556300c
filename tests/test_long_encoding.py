"""DELTA / TABLE long encodings (IndexSpec longEncoding=auto).

CPU part: the oracle's VSizeLongSerde restatement against the reference's own known answers
(VSizeLongSerdeTest.java: getBitsForMax table, the serde value vectors over every supported size),
a hand-checked packed byte string, and writer -> oracle round trips for every codec.
GPU part: the HIP expansion (k_vsize_expand after the LZ4 / uncompressed / NONE block read) against
the oracle and the written values, bit-exact, every packed width 1..64 exercised."""
import importlib

import numpy as np
import pytest

from compare import assert_results

# VSizeLongSerdeTest.testGetBitsForMax (processing/src/test/.../VSizeLongSerdeTest.java:57-68)
BITS_FOR_MAX = [(1, 1), (2, 1), (3, 2), (16, 4), (200, 8), (999, 12), (12345678, 24), (2 ** 31 - 1, 32),
                (2 ** 63 - 1, 64)]
# VSizeLongSerdeTest values0..values6 and the minimum size each is serialized at (:34-41, :71-95)
SERDE_VALUES = [
    ([0, 1, 1, 0, 1, 1, 1, 1, 0, 0, 1, 1], 1),
    ([12, 5, 2, 9, 3, 2, 5, 1, 0, 6, 13, 10, 15], 4),
    ([1, 1, 1, 1, 1, 11, 11, 11, 11], 4),
    ([200, 200, 200, 401, 200, 301, 200, 200, 200, 404, 200, 200, 200, 200], 9),
    ([123, 632, 12, 39, 536, 0, 1023, 52, 777, 526, 214, 562, 823, 346], 10),
    ([1000000, 1000001, 1000002, 1000003, 1000004, 1000005, 1000006, 1000007, 1000008], 20),
]
CODECS = ["lz4", "uncompressed", "none"]


def test_bits_for_max_kats(O, W):
    for value, bits in BITS_FOR_MAX:
        assert O.bits_for_max(value) == bits
        assert W.bits_for_max(value) == bits


def test_vsize_serde_kats(O, W):
    for bits in W.VSIZE_SUPPORTED:
        for values, min_bits in SERDE_VALUES:
            if bits < min_bits:
                continue
            packed = W.vsize_pack(np.array(values, dtype=np.int64), bits)
            assert len(packed) == W.vsize_serialized_size(bits, len(values))
            assert list(O.vsize_unpack(packed, bits, len(values))) == values, bits
        if bits >= 8:  # testSerdeIncLoop(i, 0, 256) / (0, 50000) for i >= 16
            n = 50000 if bits >= 16 else 256
            packed = W.vsize_pack(np.arange(n, dtype=np.int64), bits)
            got = O.vsize_unpack(packed, bits, n)
            assert np.array_equal(got, np.arange(n))
    # Size1Ser by hand: 0110 1111 | 0011 (zero-filled) then the 4 closing bytes
    assert W.vsize_pack(np.array(SERDE_VALUES[0][0]), 1).hex() == "6f3000000000"
    # values per 64 KiB block (getNumValuesPerBlock): the 4 closing bytes push 64-bit to 4096, 1-bit -> 2^18
    assert W.vsize_values_per_block(64) == 4096 and W.vsize_values_per_block(1) == 262144


def _encoded_columns(n, rng):
    """One column per packed width: TABLE for 1/2/4/8 bits (table sizes 2, 4, 16, 256 plus a
    single-value table), DELTA for 12..64 bits (ranges just above each smaller width)."""
    cols = {}
    for size in (1, 2, 4, 16, 256):
        vals = rng.integers(-(1 << 62), 1 << 62, size)
        cols[f"table{size}"] = ("long", vals[rng.integers(0, size, n)])
    for bits, prev in ((12, 8), (16, 12), (20, 16), (24, 20), (32, 24), (40, 32), (48, 40), (56, 48)):
        lo = int(rng.integers(-(1 << 60), 1 << 60))
        span = (1 << prev) + int(rng.integers(1, (1 << bits) - (1 << prev) - 1))
        vals = lo + rng.integers(0, span, n)
        vals[0], vals[1] = lo, lo + span - 1
        cols[f"delta{bits}"] = ("long", vals.astype(np.int64))
    full = rng.integers(-(1 << 62), 1 << 62, n)  # delta + 1 > 2^56 -> 64-bit DELTA
    full[0], full[1] = -(1 << 62), (1 << 62) - 2  # delta = Long.MAX_VALUE - 1 (MAX_VALUE itself -> LONGS)
    cols["delta64"] = ("long", full.astype(np.int64))
    cols["longs"] = ("long", rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64))  # overflow -> LONGS
    return cols


def test_writer_picks_reference_formats(W):
    rng = np.random.default_rng(3)
    cols = _encoded_columns(5000, rng)
    for name, (_, vals) in cols.items():
        fmt, meta = W.choose_long_encoding(vals)
        want = "table" if name.startswith("table") else ("longs" if name == "longs" else "delta")
        assert fmt == want, name
        if fmt == "delta":
            assert meta[2] == int(name[5:]), name


@pytest.mark.parametrize("codec", CODECS)
def test_oracle_reads_auto_encoded_columns(O, W, tmp_path, codec):
    rng = np.random.default_rng(5)
    n = 70_000
    cols = _encoded_columns(n, rng)
    ts = np.arange(n, dtype=np.int64)
    spec = W.SegmentSpec(timestamps=ts, dims={}, metrics=cols)
    p = W.write_segment(str(tmp_path / codec), spec, compression=codec, long_encoding="auto", lz4_mode="fast")
    o = O.OracleSegment(p)
    assert np.array_equal(o.time(), ts)
    for name, (_, vals) in cols.items():
        assert np.array_equal(o.numeric(name, "long"), vals), name
        assert np.array_equal(o.numeric(name, "double"), vals.astype(np.float64)), name


# ---------------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("codec", CODECS)
def test_gpu_expands_every_width(Q, O, W, tmp_path, codec):
    """Per-row buckets (1 ms granularity) expose every expanded value: bit-exact vs the oracle and
    vs the written values; plus a filtered groupBy, min/max and double coercions."""
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")
    rng = np.random.default_rng(11)
    n = 70_000  # several blocks at 12+ bits, one partial block at 1 bit; partial last blocks everywhere
    cols = _encoded_columns(n, rng)
    spec = W.SegmentSpec(timestamps=np.arange(n, dtype=np.int64) + 1_000,
                         dims={"d": W.encode_int_strings(rng.integers(0, 50, n))}, metrics=cols)
    p = W.write_segment(str(tmp_path / codec), spec, compression=codec, long_encoding="auto", lz4_mode="fast")
    g, o = S.GpuSegment(p), O.OracleSegment(p)
    assert (g.min_time, g.max_time) == (1_000, n - 1 + 1_000)
    names = list(cols)
    for chunk in range(0, len(names), 8):
        aggs = [Q.long_sum(k, k) for k in names[chunk:chunk + 8]]
        q = Q.TimeseriesQuery(intervals=[(1_000, n + 1_000)], granularity={"type": "duration", "duration": 1},
                              aggregations=aggs)
        got = R.run_query(q, [g])
        assert len(got) == n
        assert_results(q, got, O.run(q, [o]))
        for k in names[chunk:chunk + 8]:
            assert np.array_equal(np.array([row.value[k] for row in got], dtype=np.int64), cols[k][1]), k
    aggs = [Q.AggregatorFactory("longMin", "mn_" + k, k) for k in names[:6]] + \
           [Q.AggregatorFactory("longMax", "mx_" + k, k) for k in names[6:12]] + \
           [Q.AggregatorFactory("doubleSum", "ds_" + k, k) for k in names[12:]]
    q = Q.GroupByQuery(intervals=[(0, 1 << 40)], dimensions=["d"], aggregations=[Q.count("rows")] + aggs,
                       filter=Q.BoundDimFilter("d", "10", "30", False, True, ordering="numeric"))
    assert_results(q, R.run_query(q, [g]), O.run(q, [o]))


@pytest.mark.gpu
def test_gpu_table_encoded_time(Q, O, W, tmp_path):
    """A __time column with <= 256 distinct values is TABLE-encoded: time bounds and hourly buckets."""
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")
    rng = np.random.default_rng(13)
    n = 40_000
    ts = np.sort(rng.integers(0, 24, n)) * 3_600_000 + 1_500_000_000_000
    spec = W.SegmentSpec(timestamps=ts.astype(np.int64), dims={"d": W.encode_int_strings(rng.integers(0, 9, n))},
                         metrics={"m": ("long", rng.integers(0, 5, n))})
    p = W.write_segment(str(tmp_path / "t"), spec, compression="lz4", long_encoding="auto")
    g, o = S.GpuSegment(p), O.OracleSegment(p)
    assert (g.min_time, g.max_time) == (int(ts[0]), int(ts[-1]))
    q = Q.TimeseriesQuery(intervals=[(0, 1 << 42)], granularity="hour",
                          aggregations=[Q.count("rows"), Q.long_sum("m", "m")])
    assert_results(q, R.run_query(q, [g]), O.run(q, [o]))
