#!/bin/bash
# Per-config evidence on one build: rocprofv3 trace + PMC passes (tools/gpu_profile.sh), the bench_pmc
# json the line reads, then the bench line itself (STEPS_<config> timed steps, CPU baseline on).
# usage: TAG=r06_vNN CONFIGS="topn timeseries" tools/gpu_evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out bench_pmc
TAG=${TAG:-r06}
for cfg in ${CONFIGS:-topn}; do
  case $cfg in topn*|timeseries|filtered) steps=100 ;; *) steps=20 ;; esac
  CONFIG=$cfg TAG=$TAG STEPS=10 timeout -k 10 900 bash tools/gpu_profile.sh > gpurun_out/${TAG}_profile_$cfg.log 2>&1 || { echo "profile $cfg failed"; tail -20 gpurun_out/${TAG}_profile_$cfg.log; exit 4; }
  head -14 gpurun_out/prof_${TAG}_$cfg.txt | cut -c1-150
  cp gpurun_out/prof_trace/trace_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_$cfg.csv
  cp gpurun_out/pmc_$cfg.json bench_pmc/pmc_$cfg.json
  timeout -k 10 600 python -u bench.py --config $cfg --steps $steps --warmup 5 > gpurun_out/${TAG}_bench_$cfg.json 2> gpurun_out/${TAG}_bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/${TAG}_bench_$cfg.err; exit 5; }
  cut -c1-400 gpurun_out/${TAG}_bench_$cfg.json
done
