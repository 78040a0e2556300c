"""The groupBy sort alone (dg_debug_probe DG_PROBE_SORT): N packed words of the headline's key shape,
sorted by the engine's radix passes and checked ascending; prints ms per sort and the HBM rate of the
passes' algorithmic bytes (first-pass histogram read + per pass 8 B read + 8 B written per word).
usage: python tools/sort_probe.py [N] [ITERS]   (DRUID_AMD_LIB selects a variant build)"""
import ctypes
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
NAT = importlib.import_module("incubator-druid_amd._native")

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
L = NAT.lib()
ms = ctypes.c_double()
NAT.check(L.dg_debug_probe(0, 5, n, iters, ctypes.byref(ms)))
passes = 5
gb = n * (8 + 16 * passes) / 1e9
print(f"sort {n} words: {ms.value:.3f} ms  ({gb / (ms.value / 1e3):.0f} GB/s of {gb:.2f} GB algorithmic)",
      os.environ.get("DRUID_AMD_LIB", "default"))
