"""Literal-only LZ4 blocks (incompressible data: LZ4 writes one sequence of literals, e.g. sequential
3-byte ids like dimHyperUnique, or random doubles) are their own decoded image: the attach places
their literal bytes 16-byte aligned in HBM and every view points at them, no decoder runs. Results over
such columns (dimension ids, aggregator inputs, groupBy keys + payload via the keygen, topN) equal the
oracle's. The segment's `hu` (3-byte sequential ids) and `noise` (random 63-bit longs) blocks are
literal-only; `seq` and `rnd` are not."""
import importlib

import numpy as np
import pytest

from compare import assert_results

ROWS = 300_000


def _literal_only(block: bytes) -> bool:
    """lz4_literal_start's rule: one sequence of literals (no match length) ending the block."""
    if len(block) < 2 or block[0] & 15:
        return False
    q, L = 1, block[0] >> 4
    if L == 15:
        while True:
            b = block[q]
            q += 1
            L += b
            if b != 255:
                break
    return L > 0 and q + L == len(block)


@pytest.fixture(scope="module")
def seg(tmp_path_factory, W):
    rng = np.random.default_rng(41)
    ts = np.arange(ROWS, dtype=np.int64) * 12  # one hour
    spec = W.SegmentSpec(timestamps=ts, interval=(0, 12 * ROWS),
                         dims={"hu": W.encode_int_strings(np.arange(ROWS) % 100000),
                               "z": W.encode_int_strings(rng.integers(0, 7, ROWS))},
                         metrics={"rnd": ("double", rng.random(ROWS)),
                                  "seq": ("long", np.arange(ROWS, dtype=np.int64)),
                                  "noise": ("long", rng.integers(-(1 << 62), 1 << 62, ROWS))})
    p = W.write_segment(str(tmp_path_factory.mktemp("lit") / "seg"), spec)
    return p


def test_columns_hold_literal_only_blocks(W):
    """CPU: the data above compresses to literal-only LZ4 blocks (what the engine's attach detects)."""
    rng = np.random.default_rng(41)
    ids = ((np.arange(16384) + 16384) % 100000).astype("<u4").view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
    assert _literal_only(W.lz4_compress(ids, "hc"))
    assert _literal_only(W.lz4_compress(rng.integers(0, 1 << 63, 8192).astype("<i8").tobytes(), "hc"))
    assert not _literal_only(W.lz4_compress(np.arange(8192, dtype="<i8").tobytes(), "hc"))


@pytest.mark.gpu
def test_literal_blocks_match_oracle(Q, O, seg):
    R = importlib.import_module("incubator-druid_amd.runners")
    S = importlib.import_module("incubator-druid_amd.segment")
    g, o = S.GpuSegment(seg), O.OracleSegment(seg)
    iv = ["1970-01-01/2020-01-01"]
    aggs = [Q.count("rows"), Q.double_sum("rnd"), Q.long_sum("seq"), Q.long_max("noise"), Q.double_min("rnd_min", "rnd")]
    qs = [Q.TimeseriesQuery(intervals=iv, granularity="all", aggregations=aggs),
          Q.TimeseriesQuery(intervals=iv, granularity="minute", aggregations=aggs),
          Q.TimeseriesQuery(intervals=iv, granularity="all", aggregations=aggs,
                            filter=Q.BoundDimFilter("hu", "100", "20000")),
          Q.GroupByQuery(intervals=iv, dimensions=["hu"], aggregations=[Q.double_sum("rnd"), Q.long_sum("noise")]),
          Q.GroupByQuery(intervals=iv, dimensions=["z", "hu"], granularity="minute",
                         aggregations=[Q.count("rows"), Q.double_sum("rnd")]),
          Q.TopNQuery(intervals=iv, dimension="hu", metric="rnd", threshold=7,
                      aggregations=[Q.double_sum("rnd"), Q.long_sum("seq")])]
    for q in qs:
        assert_results(q, R.run_query(q, [g]), O.run(q, [o]))
    g.close()
    o.close()
