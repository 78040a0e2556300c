"""Per-phase cycles of the light LZ4 decoder (k_lz4_light) on the literal-heavy block kinds of
tools/lz4_profile.py (diagnostic; runs on a GPU box): stage, parse, table, output."""
import sys

import numpy as np

import lz4_profile as P


def main():
    ctx = P.S.GpuContext.get(0)
    rng = np.random.default_rng(1)
    pays = P.payloads(rng, 92)
    for k in sys.argv[1:] or ["uniform3", "hyper3"]:
        blocks = [P.W.lz4_compress(x, "hc") for x in pays[k]]
        ms, p = P.run(ctx, blocks)
        d = np.diff(p[:, :5], axis=1)
        print(f"{k:10s} kernel={ms:.3f} ms cps={p[:, 11].mean():.1f} cycles: " +
              " ".join(f"{nm}={v:.0f}" for nm, v in zip(["stage", "parse", "table", "output"], d.mean(axis=0))))


if __name__ == "__main__":
    main()
