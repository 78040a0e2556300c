"""Per-launch cost of a chain of small dependent kernels on one stream, launched one by one
(DG_PROBE_CHAIN) and replayed from a captured hipGraph (DG_PROBE_CHAIN_GRAPH): what graph capture
could take off the small queries' chains of 4-50 us kernels (diagnostic, GPU box).
and the host-side cost of the enqueue calls a small query makes (launch, staged upload, stream join).
usage: python tools/launch_probe.py [ITERS]"""
import ctypes
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
NAT = importlib.import_module("incubator-druid_amd._native")

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
L = NAT.lib()
ms = ctypes.c_double()
for n in (1, 8, 32, 128):
    row = []
    for kind, name in ((6, "stream"), (7, "graph")):
        NAT.check(L.dg_debug_probe(0, kind, n, iters, ctypes.byref(ms)))
        row.append(f"{name} {ms.value * 1e3:8.1f} us/chain {ms.value * 1e3 / n:6.2f} us/launch")
    print(f"chain of {n:4d}: " + " | ".join(row))
for kind, name, n in ((8, "host: kernel launch", 16), (9, "host: H2D hipMemcpyAsync of 16 KiB", 16384),
                      (9, "host: H2D hipMemcpyAsync of 256 B", 256), (10, "host: event record + stream wait", 1)):
    NAT.check(L.dg_debug_probe(0, kind, n, iters, ctypes.byref(ms)))
    print(f"{name}: {ms.value * 1e3:.2f} us per call")
