"""Summarise a tools/gpu_profile.sh run: bench line, per-kernel time (trace pass) and HBM bytes per
launch from the separate FETCH_SIZE / WRITE_SIZE passes. The table shows FETCH_SIZE raw and doubled
(MI355X_MICROARCH.md: gfx950's correction, valid for wide streaming reads only; random gathers are
left raw). With a second argument it also writes the per-kernel totals as JSON (bench.py reads
bench_pmc/pmc_<config>.json for its roofline.traffic).

usage: prof_summary.py [gpurun_out dir] [out.json] [label]"""
import collections
import csv
import json
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
line = [l for l in open(f"{d}/prof_trace.log") if l.startswith('{"metric"')]
if line:
    b = json.loads(line[-1])
    print("bench:", round(b["ms_per_step"], 3), "ms/step", round(b["value"] / 1e9, 3), "G rows/s", b["phases_ms"])
rows = list(csv.DictReader(open(f"{d}/prof_trace/trace_kernel_stats.csv")))
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for f, c in ((f"{d}/prof_fetch/fetch_counter_collection.csv", "FETCH_SIZE"),
             (f"{d}/prof_write/write_counter_collection.csv", "WRITE_SIZE")):
    for r in csv.DictReader(open(f)):
        # launches of more than 2 workgroups: the query's; attach reads each segment's time bounds
        # with a 2-block decode (read_time_bounds), which would skew a per-launch figure
        if int(r["Grid_Size"]) > 2 * int(r["Workgroup_Size"]):
            cnt[r["Kernel_Name"]][c].append(float(r["Counter_Value"]))
dur = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/prof_trace/trace_kernel_trace.csv")):
    if int(r["Grid_Size_X"]) > 2 * int(r["Workgroup_Size_X"]):
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print("per-launch columns over launches of more than 2 workgroups (q_calls, q_avg_us, fetch, write); calls / avg_us / % = all launches")
print(f"{'kernel':60s} {'calls':>5s} {'avg_us':>9s} {'%':>6s} {'q_calls':>7s} {'q_avg_us':>9s} {'fetchMB':>9s} {'fetchMBx2':>9s} {'writeMB':>9s}")
out = {"label": sys.argv[3] if len(sys.argv) > 3 else "", "kernels": {}}
if line:
    out["bench"] = {k: b.get(k) for k in ("ms_per_step", "value", "steps", "warmup", "phases_ms", "config")}
for r in rows:
    k = r["Name"]
    fe = cnt[k]["FETCH_SIZE"]
    wr = cnt[k]["WRITE_SIZE"]
    fmb = sum(fe) / len(fe) / 1e3 if fe else float("nan")
    wmb = sum(wr) / len(wr) / 1e3 if wr else float("nan")
    q = dur.get(k, [])
    qavg = sum(q) / len(q) / 1e3 if q else float("nan")
    print(f"{k[:60]:60s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.1f} {float(r['Percentage']):6.2f} {len(q):7d} {qavg:9.1f} "
          f"{fmb:9.1f} {2 * fmb:9.1f} {wmb:9.1f}")
    if fe and wr:  # FETCH_SIZE / WRITE_SIZE are in KiB
        out["kernels"][k] = {"calls": len(fe), "avg_ns": sum(q) / len(q) if q else float(r["AverageNs"]),
                             "trace_calls": len(q), "fetch_bytes": sum(fe) * 1024, "write_bytes": sum(wr) * 1024}
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
