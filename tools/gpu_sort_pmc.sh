#!/bin/bash
# SQ counters of the radix scatter on the sort probe (tools/sort_probe.py): wave cycles split into
# issue / stalled, instruction mix, LDS bank conflicts; two passes of 8 SQ counters, each bounded.
# Summary (per dispatch of k_rs_scatter / k_rs_hist0) in gpurun_out/sort_sq_<tag>.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-sq}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P2="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  rm -rf gpurun_out/ssq_$i
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -f csv -d gpurun_out/ssq_$i -o sq -- python3 tools/sort_probe.py ${N:-100000000} 2 > gpurun_out/ssq_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/ssq_$i.log; exit 5; }
done
python3 - > gpurun_out/sort_sq_$TAG.txt <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for i in (1, 2):
    for f in glob.glob(f"gpurun_out/ssq_{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:40]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if i == 1 and r["Counter_Name"] == "SQ_WAVES":
                n[k] += 1
for k, c in acc.items():
    if "rs_" not in k:
        continue
    print(k, "dispatches", n[k])
    for name in sorted(c):
        print(f"   {name:24s} {c[name] / max(n[k], 1):16.0f}")
PY
cat gpurun_out/sort_sq_$TAG.txt
