#!/bin/bash
# Kernel trace of one bench config (timed steps carry no phase events) and the timeline of its last
# timed step: CONFIG=topn PER_STEP=<launches per step> TAG=r05_vNN bash tools/gpu_timeline.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CONFIG=${CONFIG:-topn}
TAG=${TAG:-tl}
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/${TAG}_trace_$CONFIG -o run -- \
  python3 bench.py --config $CONFIG --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_trace_$CONFIG.log 2>&1 &&
python3 tools/timeline.py gpurun_out/${TAG}_trace_$CONFIG 400 > gpurun_out/${TAG}_timeline_$CONFIG.txt
