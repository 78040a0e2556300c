#!/bin/bash
# SQ counters of the LZ4 decoders on the phase-profile blocks (tools/lz4_profile.py KIND...): wave
# cycles split into issue / stalled / parked, instruction mix, LDS bank conflicts. Two passes (8 SQ
# counters each), each under its own time limit; summary in gpurun_out/lz4_sq_<tag>.txt.
# usage: TAG=x tools/lz4_sq_pmc.sh seqlong normal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-sq}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P2="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  rm -rf gpurun_out/sq_$i
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -f csv -d gpurun_out/sq_$i -o sq -- python3 tools/lz4_profile.py "$@" > gpurun_out/sq_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_$i.log; exit 5; }
done
python3 - "$TAG" > gpurun_out/lz4_sq_$TAG.txt <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for i in (1, 2):
    for f in glob.glob(f"gpurun_out/sq_{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:40]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if i == 1 and r["Counter_Name"] == "SQ_WAVES":
                n[k] += 1
for k, c in acc.items():
    if "lz4" not in k:
        continue
    print(k, "dispatches", n[k])
    for name in sorted(c):
        print(f"   {name:24s} {c[name] / max(n[k], 1):16.0f}")
PY
cat gpurun_out/lz4_sq_$TAG.txt
