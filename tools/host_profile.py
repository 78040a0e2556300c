"""Wall-time split of one bench step (topN config) between the engine call, the engine-side merge and
the Python result building (diagnostic; runs on a GPU box after bench.py has written the segments)."""
import importlib
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

Q = importlib.import_module("incubator-druid_amd.query")
R = importlib.import_module("incubator-druid_amd.runners")
S = importlib.import_module("incubator-druid_amd.segment")
DG = importlib.import_module("incubator-druid_amd.datagen")


def main():
    rows, nseg = 750_000, 4
    paths = bench.ensure_segments(DG, "/tmp/druid_amd_bench", 0, nseg, rows, "lz4", "concise", "hc")
    segs = [S.GpuSegment(p, device=0) for p in paths]
    q = bench.make_query(Q, "topn")
    for _ in range(3):
        R.run_topn(segs, q)
    acc = {"topn_raw": 0.0, "merge": 0.0, "build": 0.0, "engine_total_ms": 0.0, "decode_ms": 0.0,
           "aggregate_ms": 0.0, "bitmap_ms": 0.0}
    n = 30
    for _ in range(n):
        st = R.RunStats()
        t0 = time.perf_counter()
        raw = R.topn_raw(segs, q, st)
        t1 = time.perf_counter()
        res = R.topn_merge_raw(q, raw.cnt, raw.ids, raw.vals, raw.K, raw.ts, [s.handle for s in segs])
        t2 = time.perf_counter()
        ts, lists, keys, slots = res
        values = [segs[int(l)].dim_value(q.dimension, int(k)) for l, k in zip(lists, keys)]
        out = [Q.Result(ts, R._topn_entries(q, values, slots))]
        t3 = time.perf_counter()
        acc["topn_raw"] += t1 - t0
        acc["merge"] += t2 - t1
        acc["build"] += t3 - t2
        acc["engine_total_ms"] += st.total("total_ms") / 1e3
        acc["decode_ms"] += st.total("decode_ms") / 1e3
        acc["aggregate_ms"] += st.total("aggregate_ms") / 1e3
        acc["bitmap_ms"] += st.total("bitmap_ms") / 1e3
    for k, v in acc.items():
        print(f"{k:16s} {v / n * 1e3:8.3f} ms")
    assert out


if __name__ == "__main__":
    main()
