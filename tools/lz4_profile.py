"""Per-phase cycle breakdown of the LZ4 decoder on the bench segments (diagnostic)."""
import ctypes, importlib, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
N = importlib.import_module("incubator-druid_amd._native")
S = importlib.import_module("incubator-druid_amd.segment")
DG = importlib.import_module("incubator-druid_amd.datagen")
path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/druid_amd_bench/lz4prof/seg"
if not os.path.exists(os.path.join(path, "version.bin")):
    DG.write_basic_segment(path, 750_000, seed=9999)
seg = S.GpuSegment(path)
L = N.lib()
L.dg_debug_lz4_profile.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int32,
                                   ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)]
names = ["stage", "spec_walk", "fixpoint", "resolve", "count+scan", "literals+table", "pointer_jump"]
for col in ["sumLongSequential", "sumFloatNormal", "dimUniform", "__time", "dimSequential"]:
    for rep in range(2):
        buf = np.zeros(200 * 12, dtype=np.uint64)
        nb, ms = ctypes.c_int32(), ctypes.c_double()
        N.check(L.dg_debug_lz4_profile(seg.handle, col.encode(), buf.ctypes.data, 200, ctypes.byref(nb), ctypes.byref(ms)))
    p = buf.reshape(-1, 12)[:min(nb.value, 200)].astype(np.int64)
    d = np.diff(p[:, :8], axis=1)
    print(f"{col:20s} blocks={nb.value:4d} kernel={ms.value:8.3f} ms  n(avg)={p[:,9].mean():7.0f} jump_rounds(avg/max)={p[:,8].mean():6.1f}/{p[:,8].max():4d} slow={p[:,10].mean():6.1f} fix_rounds={p[:,11].mean():4.1f}")
    print("   cycles/phase (mean): " + "  ".join(f"{nm}={v:8.0f}" for nm, v in zip(names, d.mean(axis=0))))
