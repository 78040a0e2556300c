#!/bin/bash
# Hourly configs: host traces, then the evidence (profile + PMC + line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
for cfg in ts_hourly groupby_hourly; do
  DG_HOST_TRACE=1 timeout -k 10 600 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-probes \
    > gpurun_out/${TAG}_trace_$cfg.json 2> gpurun_out/${TAG}_trace_$cfg.err || { tail -5 gpurun_out/${TAG}_trace_$cfg.err; exit 3; }
  grep "dg host" gpurun_out/${TAG}_trace_$cfg.err | tail -3 | cut -c1-400
done
TAG=$TAG CONFIGS="ts_hourly groupby_hourly" bash tools/gpu_evidence.sh
