"""Summarise a tools/gpu_profile.sh run: per-kernel duration stats (kernel trace) and per-launch HBM
bytes from the separate FETCH_SIZE / WRITE_SIZE PMC passes, with the gfx950 corrections of
MI355X_MICROARCH.md (HBM section): FETCH_SIZE is in KiB and reports half of the bytes of wide
streaming reads (x2), WRITE_SIZE in KiB is exact for 16-byte stores.

    python tools/summarize_profile.py gpurun_out OUT_PREFIX

writes OUT_PREFIX_rocprof_summary.txt and OUT_PREFIX_pmc_traffic.json (per-kernel mean bytes per
launch over the launches of the bench's own grid size, i.e. excluding segment-attach decodes)."""
import collections
import csv
import json
import os
import sys


def main(src, prefix):
    stats = list(csv.DictReader(open(os.path.join(src, "prof_trace", "trace_kernel_stats.csv"))))
    trace = list(csv.DictReader(open(os.path.join(src, "prof_trace", "trace_kernel_trace.csv"))))
    lines = ["kernel stats (rocprofv3 --kernel-trace --stats):",
             f"{'kernel':70s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'pct':>6s}"]
    for r in stats:
        lines.append(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:10.1f} "
                     f"{float(r['MinNs'])/1e3:10.1f} {float(r['MaxNs'])/1e3:10.1f} {float(r['Percentage']):6.2f}")
    # the bench launches of each kernel = the most frequent grid size among its dispatches
    dur = collections.defaultdict(list)
    for r in trace:
        name = r["Kernel_Name"].split("(")[0]
        if "Grid_Size" in r:
            grid = int(r["Grid_Size"])
        else:
            grid = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
        dur[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for tag, fname, counter in (("fetch", "fetch_counter_collection.csv", "FETCH_SIZE"),
                                ("write", "write_counter_collection.csv", "WRITE_SIZE")):
        path = os.path.join(src, f"prof_{tag}", fname)
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            pmc[(name, int(r["Grid_Size"]))][counter].append(float(r["Counter_Value"]))
    lines.append("")
    lines.append("per launch, grouped by (kernel, grid size): duration from the trace pass, HBM bytes from the PMC passes")
    lines.append(f"{'kernel':40s} {'grid':>9s} {'n':>4s} {'avg_us':>9s} {'FETCH_KiB':>11s} {'WRITE_KiB':>11s} {'hbm_MB(corr)':>13s}")
    out = {}
    for (name, grid), ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        f = pmc[(name, grid)].get("FETCH_SIZE", [])
        w = pmc[(name, grid)].get("WRITE_SIZE", [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        corr = None
        if fk is not None and wk is not None:
            corr = (2 * fk + wk) * 1024
        lines.append(f"{name[:40]:40s} {grid:9d} {len(ds):4d} {sum(ds)/len(ds):9.1f} "
                     f"{fk if fk is not None else float('nan'):11.1f} {wk if wk is not None else float('nan'):11.1f} "
                     f"{corr/1e6 if corr else float('nan'):13.2f}")
        key = name.replace("dg::", "")
        if key not in out or len(ds) > out[key]["launches"]:
            out[key] = {"grid": grid, "launches": len(ds), "avg_us": sum(ds) / len(ds),
                        "fetch_kib": fk, "write_kib": wk, "hbm_bytes_corrected": corr}
    open(prefix + "_rocprof_summary.txt", "w").write("\n".join(lines) + "\n")
    json.dump(out, open(prefix + "_pmc_traffic.json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
