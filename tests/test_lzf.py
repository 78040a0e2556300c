"""LZF blocks (CompressionStrategy.LZF id 0x00, and LZF_VERSION 0x01 numeric columns of older
segments). The codec is compress-lzf 1.0.4 (a pom dependency, not vendored): the oracle restates
its published chunk format ("ZV" chunks, liblzf tokens) and is pinned by hand-assembled known-answer
chunks below plus round trips through the writer's encoder; the GPU decoder (k_lzf_decode) is checked
bit-exact against the oracle on per-row buckets."""
import importlib

import numpy as np
import pytest

from compare import assert_results

# "ZV" type 1: literal run of one 'a' (ctrl 0x00), back-reference ctrl 0xE0 + ext 0 (length 9) at
# distance 0 + 1 = 1 -> ten 'a'; then a type-0 chunk "xyz"
KAT = (bytes.fromhex("5a5601000500" "0a" "0061e00000") + bytes.fromhex("5a56000003") + b"xyz", b"a" * 10 + b"xyz")
# long literal run (32 bytes, ctrl 31) then a 3-byte reference at distance 16 (ctrl 0x20 | 0, offset 15)
_LIT = bytes(range(32))
KAT2 = (bytes.fromhex("5a560100") + bytes([35, 0, 35]) + bytes([31]) + _LIT + bytes([0x20, 15]),
        _LIT + _LIT[16:19])


def test_lzf_known_answers(O):
    for enc, dec in (KAT, KAT2):
        assert O.lzf_decompress(enc) == dec
    with pytest.raises(ValueError):
        O.lzf_decompress(b"ZX\x00\x00\x01a")  # bad magic
    with pytest.raises(ValueError):
        O.lzf_decompress(bytes.fromhex("5a5601000300" "05" "20ff00"))  # reference before the output start


def test_lzf_writer_round_trips(O):
    T = importlib.import_module("incubator-druid_amd._tools")
    rng = np.random.default_rng(0)
    cases = [np.arange(8192, dtype="<i8").tobytes(), rng.bytes(65536), bytes(65536),
             (b"abc" * 30000)[:65536], rng.integers(0, 3, 65536, dtype=np.uint8).tobytes(), b"x",
             np.round(rng.normal(100, 10, 8192), 1).astype("<f8").tobytes()]
    for d in cases:
        assert O.lzf_decompress(T.lzf_compress(d)) == d


def _metrics(n, rng):
    seq = np.arange(n, dtype=np.int64)
    return {"seq": ("long", seq % 10000), "rnd": ("long", rng.integers(-(1 << 62), 1 << 62, n)),
            "zeros": ("long", np.zeros(n, dtype=np.int64)), "dbl": ("double", rng.normal(5000.0, 1.0, n)),
            "flt": ("float", rng.normal(3.0, 1.0, n).astype(np.float32))}


@pytest.mark.parametrize("comp", ["lzf", "lzf_v1"])
def test_oracle_reads_lzf_segments(O, W, tmp_path, comp):
    rng = np.random.default_rng(4)
    n = 40_000
    m = _metrics(n, rng)
    spec = W.SegmentSpec(timestamps=np.arange(n, dtype=np.int64), dims={"d": W.encode_int_strings(rng.integers(0, 300, n))},
                         metrics=m)
    o = O.OracleSegment(W.write_segment(str(tmp_path / comp), spec, compression=comp))
    assert np.array_equal(o.time(), np.arange(n))
    for k, (kind, v) in m.items():
        got = o.numeric(k, kind)
        assert np.array_equal(got, v), k


@pytest.mark.gpu
@pytest.mark.parametrize("comp", ["lzf", "lzf_v1"])
def test_gpu_lzf_every_value(Q, O, W, tmp_path, comp):
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")
    rng = np.random.default_rng(8)
    n = 50_000
    m = _metrics(n, rng)
    spec = W.SegmentSpec(timestamps=np.arange(n, dtype=np.int64) + 7,
                         dims={"d": W.encode_int_strings(rng.integers(0, 300, n))}, metrics=m)
    p = W.write_segment(str(tmp_path / comp), spec, compression=comp)
    g, o = S.GpuSegment(p), O.OracleSegment(p)
    assert (g.min_time, g.max_time) == (7, n - 1 + 7)
    aggs = [Q.long_sum("seq", "seq"), Q.long_sum("rnd", "rnd"), Q.long_sum("zeros", "zeros"),
            Q.AggregatorFactory("doubleMax", "dbl", "dbl"), Q.AggregatorFactory("floatMax", "flt", "flt")]
    q = Q.TimeseriesQuery(intervals=[(0, n + 7)], granularity={"type": "duration", "duration": 1}, aggregations=aggs)
    got = R.run_query(q, [g])
    assert len(got) == n
    assert_results(q, got, O.run(q, [o]))
    assert np.array_equal(np.array([r.value["rnd"] for r in got], dtype=np.int64), m["rnd"][1])
    q = Q.TopNQuery(intervals=[(0, 1 << 40)], dimension="d", metric="seq", threshold=7, aggregations=aggs,
                    filter=Q.BoundDimFilter("d", "10", "200", False, True, ordering="numeric"))
    assert_results(q, R.run_query(q, [g]), O.run(q, [o]))
    q = Q.GroupByQuery(intervals=[(0, 1 << 40)], dimensions=["d"], aggregations=[Q.count("rows")] + aggs)
    assert_results(q, R.run_query(q, [g]), O.run(q, [o]))
