"""Where a small query's step goes (diagnostic, GPU box): per bench step of the timeseries (configs[0])
and topN (configs[1]) lines, the wall time of the Python plan build (make_scan), of the engine call and
of the rest (result building, merge), averaged over 50 steps after warm-up; the engine's own host
stamps with DG_HOST_TRACE=1 (stderr). Run after bench.py has written the segments:
    python tools/small_profile.py [timeseries|topn ...]"""
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
N = importlib.import_module("incubator-druid_amd._native")


def main():
    for cfg in sys.argv[1:] or ["timeseries", "topn"]:
        rows, nseg, _, cols = bench.CONFIGS[cfg]
        paths = bench.ensure_segments("/tmp/druid_amd_bench", 0, nseg, rows, "lz4", "concise", "hc", cols)
        segs = [S.GpuSegment(p, device=0) for p in paths]
        q = bench.make_query(Q, cfg)
        run = (lambda st: R.run_topn(segs, q, st)) if cfg.startswith("topn") else \
            (lambda st: R.run_query(q, segs, st))
        for _ in range(10):
            run(R.RunStats())
        n = 50
        t_scan = 0.0
        for _ in range(n):
            t0 = time.perf_counter()
            N.make_scan(q, Q, segments=segs)
            t_scan += time.perf_counter() - t0
        st = R.RunStats()
        t0 = time.perf_counter()
        for _ in range(n):
            run(st)
        wall = (time.perf_counter() - t0) / n
        eng = sum(c["total_ms"] for c in st.calls) / n
        dev = {k: sum(c[k] for c in st.calls) / n for k in ("bitmap_ms", "decode_ms", "aggregate_ms")}
        print(f"{cfg}: step {wall * 1e3:.3f} ms | make_scan {t_scan / n * 1e3:.3f} ms | engine call {eng:.3f} ms | "
              f"rest {wall * 1e3 - eng:.3f} ms | device phases {dev}", flush=True)
        os.environ["DG_HOST_TRACE"] = "1"
        for _ in range(3):
            run(R.RunStats())
        os.environ.pop("DG_HOST_TRACE")
        for s in segs:
            s.close()


if __name__ == "__main__":
    main()
