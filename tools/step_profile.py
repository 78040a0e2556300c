"""Host-side split of one small bench step (diagnostic, GPU box): wall time per step with the phase
timestamps off, the engine's own total_ms (query_wall), and a cProfile of the Python around it.
usage: python tools/step_profile.py timeseries|filtered|topn|topn_numeric [steps]"""
import cProfile
import importlib
import os
import pstats
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
    name = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    rows, nseg, _, cols = bench.CONFIGS[name]
    paths = bench.ensure_segments("/tmp/druid_amd_bench", 0, nseg, rows, "lz4", "concise", "hc", cols)
    segs = [S.GpuSegment(p, device=0) for p in paths]
    q = bench.make_query(Q, name)

    def step(st):
        if isinstance(q, Q.TopNQuery):
            return R.run_topn(segs, q, st)
        return R.run_query(q, segs, st)  # (as bench.py's single-rank step)

    for _ in range(20):
        step(R.RunStats())
    N.lib().dg_set_phase_timing(0)
    st = R.RunStats()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(st)
    wall = (time.perf_counter() - t0) / steps * 1e3
    print(f"{name}: step {wall:.4f} ms, engine total_ms {st.total('total_ms') / steps:.4f} ms "
          f"({len(st.calls) / steps:.0f} engine calls per step)")
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(steps):
        step(R.RunStats())
    prof.disable()
    pstats.Stats(prof).sort_stats("tottime").print_stats(25)
    pstats.Stats(prof).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
