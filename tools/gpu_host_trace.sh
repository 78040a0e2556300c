#!/bin/bash
# Host-side stamps of the engine's calls (DG_HOST_TRACE=1) over a few bench steps of CONFIG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CONFIG=${CONFIG:-groupby}
DG_HOST_TRACE=1 timeout -k 10 600 python -u bench.py --config $CONFIG --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline \
  > gpurun_out/trace_$CONFIG.json 2> gpurun_out/trace_$CONFIG.err || { tail -5 gpurun_out/trace_$CONFIG.err; exit 3; }
grep "dg host" gpurun_out/trace_$CONFIG.err | tail -6
