#!/bin/bash
# LDS / VALU counters of the LZ4 decoder per block kind (one rocprofv3 pass per counter group and kind).
# usage: KINDS="seqlong uniform3" tools/lz4_pmc.sh ; output under gpurun_out/lz4pmc_<kind>_<i>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for kind in ${KINDS:-seqlong}; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -f csv -d gpurun_out/lz4pmc_${kind}_$i -o pmc -- python3 tools/lz4_profile.py $kind > gpurun_out/lz4pmc_${kind}_$i.log 2>&1 || { echo "pass $kind $i failed"; tail -5 gpurun_out/lz4pmc_${kind}_$i.log; exit 3; }
  done
done
echo done
