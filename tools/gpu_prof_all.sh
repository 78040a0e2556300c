#!/bin/bash
# rocprofv3 evidence for several bench lines in one GPU call: for each CONFIGS entry, tools/gpu_profile.sh
# (kernel trace + stats, then separate FETCH_SIZE and WRITE_SIZE passes); the summary, the PMC json and
# the kernel stats csv are kept per config under gpurun_out/ (TAG_*). Stops at the first failure.
# usage: TAG=r05_v5 CONFIGS="timeseries topn" tools/gpu_prof_all.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-prof}
for cfg in ${CONFIGS:-timeseries topn filtered}; do
  CONFIG=$cfg TAG=$TAG STEPS=${STEPS:-10} timeout -k 10 1100 bash tools/gpu_profile.sh > gpurun_out/${TAG}_prof_$cfg.log 2>&1
  rc=$?
  head -12 gpurun_out/prof_${TAG}_$cfg.txt 2>/dev/null | cut -c1-160
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_prof_$cfg.log; exit $rc; }
  cp gpurun_out/prof_trace/trace_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_$cfg.csv
  cp gpurun_out/pmc_$cfg.json gpurun_out/${TAG}_pmc_$cfg.json
done
