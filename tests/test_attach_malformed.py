"""Attach-time validation of segment bytes (GenericIndexed offsets, truncated column parts): a corrupt
segment is rejected with DG_ERR_FORMAT (the reference throws IAE / ISE from GenericIndexed.java:131-149
when a header does not fit its buffer) instead of reading outside the mapped file."""
import ctypes
import importlib
import os
import shutil
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _columns(path):
    with open(os.path.join(path, "meta.smoosh")) as f:
        return {ln.split(",")[0]: (int(ln.split(",")[2]), int(ln.split(",")[3])) for ln in f.read().split("\n")[1:] if ln}


def _patch(src, dst, fn):
    shutil.copytree(src, dst)
    p = os.path.join(dst, "00000.smoosh")
    data = bytearray(open(p, "rb").read())
    fn(data, _columns(dst))
    open(p, "wb").write(bytes(data))
    return dst


def _dict_offsets_at(data, col):
    """Byte position of the dictionary GenericIndexed's first offset of a string column part:
    [i32 descriptor length][descriptor][u8 version][i32 flags][0x01][sorted][i32 used][i32 n][offsets]"""
    start, _ = col
    jl = struct.unpack(">i", bytes(data[start:start + 4]))[0]
    return start + 4 + jl + 1 + 4 + 2 + 4 + 4


def test_corrupt_segments_rejected(tmp_path, DG):
    N = importlib.import_module("incubator-druid_amd._native")
    S = importlib.import_module("incubator-druid_amd.segment")
    good = DG.write_basic_segment(str(tmp_path / "good"), 5000, seed=3, lz4_mode="fast")
    ctx = S.GpuContext.get(0)

    def huge_offset(data, cols):  # first dictionary value ends far outside the values region
        o = _dict_offsets_at(data, cols["dimZipf"])
        data[o:o + 4] = struct.pack(">i", 0x7FFFFFF0)

    def negative_length(data, cols):  # second value ends before it starts
        o = _dict_offsets_at(data, cols["dimZipf"])
        data[o + 4:o + 8] = struct.pack(">i", 0)
        data[o:o + 4] = struct.pack(">i", 40)

    def huge_count(data, cols):  # element count larger than the header region
        o = _dict_offsets_at(data, cols["dimUniform"])
        data[o - 4:o] = struct.pack(">i", 0x3FFFFFFF)

    def truncated_part(data, cols):  # a numeric column's header claims more blocks than it holds
        start, end = cols["sumLongSequential"]
        jl = struct.unpack(">i", bytes(data[start:start + 4]))[0]
        p = start + 4 + jl  # [u8 version 2][i32 total][i32 sizePer][u8 codec]...
        data[p + 1:p + 5] = struct.pack(">i", 0x7FFFFFF)

    for i, fn in enumerate((huge_offset, negative_length, huge_count, truncated_part)):
        bad = _patch(good, str(tmp_path / f"bad{i}"), fn)
        h = ctypes.c_void_p()
        rc = N.lib().dg_segment_attach(ctx.handle, bad.encode(), ctypes.byref(h))
        assert rc == 1, (fn.__name__, rc, N.lib().dg_last_error())
    h = ctypes.c_void_p()
    assert N.lib().dg_segment_attach(ctx.handle, good.encode(), ctypes.byref(h)) == 0
    N.lib().dg_segment_release(h)


def test_short_literal_only_block_rejected(tmp_path, W):
    """A literal-only LZ4 block is read in place (no decoder runs, so nothing checks its decoded length
    on the device): when its literals do not cover its rows the attach fails with DG_ERR_FORMAT instead
    of letting the views read past the block. Random longs compress to literal-only blocks; the
    column's row total is raised by 100 so its last block (1,808 rows written) claims 1,908."""
    N = importlib.import_module("incubator-druid_amd._native")
    S = importlib.import_module("incubator-druid_amd.segment")
    n = 10_000
    rng = np.random.default_rng(5)
    spec = W.SegmentSpec(timestamps=np.arange(n, dtype=np.int64), interval=(0, n),
                         dims={"d": W.encode_int_strings(np.arange(n) % 7)},
                         metrics={"noise": ("long", rng.integers(-(1 << 62), 1 << 62, n))})
    good = W.write_segment(str(tmp_path / "good"), spec)
    ctx = S.GpuContext.get(0)
    h = ctypes.c_void_p()
    assert N.lib().dg_segment_attach(ctx.handle, good.encode(), ctypes.byref(h)) == 0
    N.lib().dg_segment_release(h)

    def longer_total(data, cols):
        start, _ = cols["noise"]
        jl = struct.unpack(">i", bytes(data[start:start + 4]))[0]
        p = start + 4 + jl  # [u8 version 2][i32 total][i32 sizePer][u8 codec]...
        assert struct.unpack(">i", bytes(data[p + 1:p + 5]))[0] == n
        data[p + 1:p + 5] = struct.pack(">i", n + 100)

    bad = _patch(good, str(tmp_path / "short"), longer_total)
    h = ctypes.c_void_p()
    rc = N.lib().dg_segment_attach(ctx.handle, bad.encode(), ctypes.byref(h))
    assert rc == 1 and "literal-only block" in N.lib().dg_last_error().decode(), (rc, N.lib().dg_last_error())


def test_corrupt_multi_value_row_lists(tmp_path, Q, W):
    """Multi-value row lists are validated on the device once decoded (offsets start at 0, never
    decrease and stay within the values; every value id is below the dictionary size) before any
    kernel follows them: a corrupt list fails the query with DG_ERR_FORMAT instead of sending the
    explode / topN / filter kernels outside their buffers. Legacy compressed form with UNCOMPRESSED
    blocks, so the offsets (1 byte: 0, 2, 4, ..., 200) and ids can be patched in place."""
    N = importlib.import_module("incubator-druid_amd._native")
    S = importlib.import_module("incubator-druid_amd.segment")
    R = importlib.import_module("incubator-druid_amd.runners")
    n = 100
    rows = [["x", "y"]] * n
    dic, ids = W.encode_multi_strings(rows)
    spec = W.SegmentSpec(timestamps=np.arange(n, dtype=np.int64) * 1000, dims={"tags": (dic, ids)},
                         metrics={"m": ("long", np.arange(n))})
    good = W.write_segment(str(tmp_path / "good"), spec, compression="uncompressed", legacy_multi_value=True)
    offsets = bytes(range(0, 2 * n + 1, 2))
    ids_block = bytes([0, 1] * n)

    def find(data, pat):
        i = bytes(data).find(pat)
        assert i >= 0 and bytes(data).find(pat, i + 1) < 0
        return i

    def decreasing(data, cols):
        o = find(data, offsets)
        data[o + 50] = 1

    def past_values(data, cols):
        o = find(data, offsets)
        data[o + n] = 250

    def bad_id(data, cols):
        o = find(data, ids_block)
        data[o + 7] = 0x7F

    q = Q.GroupByQuery(intervals=[(0, 1 << 40)], dimensions=["tags"], aggregations=[Q.count("rows")])
    assert [r.event["rows"] for r in R.run_query(q, [S.GpuSegment(good)])] == [n, n]
    for i, fn in enumerate((decreasing, past_values, bad_id)):
        bad = _patch(good, str(tmp_path / f"mv{i}"), fn)
        g = S.GpuSegment(bad)  # attach reads headers only; the lists are checked per query
        for qq in (q, Q.TopNQuery(intervals=[(0, 1 << 40)], dimension="tags", metric="rows", threshold=3,
                                  aggregations=[Q.count("rows")])):
            with pytest.raises(N.DruidGpuError, match="corrupt multi-value row lists"):
                R.run_query(qq, [g])
