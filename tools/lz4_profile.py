"""Per-phase cycle breakdown of the LZ4 decoder (diagnostic; runs on a GPU box).

Blocks are the bench segments' column kinds (basic schema, LZ4-HC): sequential longs, __time,
normal doubles, 3-byte dimUniform ids. Prints, per kind and for the bench's mix, the kernel time
and the mean s_memtime cycles of each phase (stage, parse, fill, coop, jump, output).
"""
import ctypes
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
N = importlib.import_module("incubator-druid_amd._native")
S = importlib.import_module("incubator-druid_amd.segment")
W = importlib.import_module("incubator-druid_amd.writer")
BLOCK = 65536
PHASES = ["stage", "parse+scan", "jobs+read", "fill+write", "resolve", "output"]
KINDS = {-1: "malformed", 0: "general", 1: "general-wide", 2: "light", 3: "run", 4: "flow"}


def classify(block):
    k = ctypes.c_int32()
    N.check(N.lib().dg_debug_lz4_classify(block, len(block), ctypes.byref(k)))
    return KINDS[k.value]


def payloads(rng, k):
    n8 = BLOCK // 8
    out = {"seqlong": [], "time": [], "normal": [], "uniform3": [], "hyper3": [], "ulong500": [], "zipfdbl": []}
    for i in range(k):
        seq = np.arange(i * n8, (i + 1) * n8, dtype=np.int64)
        out["seqlong"].append((seq % 10000).astype("<i8").tobytes())
        out["time"].append(np.round(seq * 1.3333).astype("<i8").tobytes())
        out["normal"].append(rng.normal(5000, 1, n8).astype("<f8").tobytes())
        out["ulong500"].append(rng.integers(0, 501, n8).astype("<i8").tobytes())
        zk = np.arange(1, 1001, dtype=np.float64)
        zp = 1.0 / zk
        out["zipfdbl"].append(rng.choice(zk - 1, size=n8, p=zp / zp.sum()).astype("<f8").tobytes())
        ids = rng.integers(1, 100001, BLOCK // 3 + 1).astype("<u4").view(np.uint8).reshape(-1, 4)[:, :3]
        out["uniform3"].append(ids.tobytes()[:3 * 16384])
        hyp = (np.arange(i * 16384, (i + 1) * 16384) % 100000).astype("<u4").view(np.uint8).reshape(-1, 4)[:, :3]
        out["hyper3"].append(hyp.tobytes())
    return out


def run(ctx, blocks):
    n = len(blocks)
    bufs = [np.frombuffer(b, dtype=np.uint8).copy() for b in blocks]
    ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    lens = (ctypes.c_int32 * n)(*[len(b) for b in blocks])
    out = np.zeros(n * BLOCK, dtype=np.uint8)
    out_lens = (ctypes.c_int32 * n)()
    ms = ctypes.c_double()
    prof = np.zeros(n * 32, dtype=np.uint64)
    for _ in range(2):
        N.check(N.lib().dg_debug_lz4_decode(ctx.handle, ptrs, lens, n, out.ctypes.data, out_lens, ctypes.byref(ms),
                                            prof.ctypes.data))
    p = prof.reshape(n, 32).astype(np.int64)
    return ms.value, p


def report(name, ms, p, decoder=""):
    d = np.diff(p[:, :7], axis=1)
    print(f"{name:10s} [{decoder}] blocks={len(p):4d} kernel={ms:7.3f} ms  in_bytes(avg)={p[:, 9].mean():7.0f} "
          f"jump_rounds(avg/max)={p[:, 8].mean():5.1f}/{p[:, 8].max():3d} coop_jobs={p[:, 10].mean():6.1f} "
          f"cps={p[:, 11].mean():6.1f} listed={p[:, 7].mean():7.0f}")
    print("   cycles/phase (mean): " + "  ".join(f"{nm}={v:8.0f}" for nm, v in zip(PHASES, d.mean(axis=0))))
    if "flow" in decoder:
        sub = {"literals": p[:, 13] - p[:, 2], "job_scan": p[:, 14] - p[:, 13], "job_copy": p[:, 15] - p[:, 14],
               "own": p[:, 3] - p[:, 15]}
        print("   literal phase (wave 0, mean): " + "  ".join(f"{nm}={v.mean():8.0f}" for nm, v in sub.items()))
        busy = p[:, 16:32]
        print(f"   levels: busy cycles per wave (mean over blocks) max={busy.max(axis=1).mean():8.0f} "
              f"mean={busy.mean():8.0f}; wave 0 barrier wait={p[:, 12].mean():8.0f}")
    if decoder != "general":
        return
    sub = {"scan1": p[:, 12] - p[:, 4], "scan2": p[:, 13] - p[:, 12], "rounds": p[:, 5] - p[:, 13]}
    print("   resolve (mean): " + "  ".join(f"{nm}={v.mean():8.0f}" for nm, v in sub.items()))
    base = int(os.environ.get("LZ4_WAVE_BASE", "3"))  # the phase start of the build's DG_LZ_WAVE_STAMP point
    fw = p[:, 16:32] - p[:, base:base + 1]  # each wave's own end of the phase, from the phase start
    print(f"   phase end per wave (mean over blocks): first={fw.min(axis=1).mean():8.0f} last={fw.max(axis=1).mean():8.0f}")
    print(f"   fill_general cycles in the last interval's wave: {p[:, 14].mean():8.0f}")
    print("   phase end by wave index: " + " ".join(f"{v:.0f}" for v in fw.mean(axis=0)))


def main():
    ctx = S.GpuContext.get(0)
    rng = np.random.default_rng(1)
    # 1024 blocks of a kind: four per CU, so most blocks run with the decoder's code already in the
    # instruction cache (92 blocks = one cold block per CU)
    pays = payloads(rng, int(os.environ.get("LZ4_PROFILE_BLOCKS", "1024")))
    comp = {k: [W.lz4_compress(x, "hc") for x in v] for k, v in pays.items()}
    kinds = sys.argv[1:] or list(comp)
    for k, blocks in comp.items():
        if k not in kinds:
            continue
        ms, p = run(ctx, blocks)
        report(k, ms, p, "/".join(sorted({classify(b) for b in blocks})))
    if sys.argv[1:] and "mix" not in kinds:
        return
    mix = []
    for s in range(4):
        mix += comp["uniform3"][:46] + comp["seqlong"] + comp["normal"]
    ms, p = run(ctx, mix)
    report("bench-mix", ms, p)


if __name__ == "__main__":
    main()
