#!/bin/bash
# rocprofv3 evidence for a bench line: kernel trace + stats, then separate PMC passes for HBM bytes
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950). The segments are written first, outside
# the profiler. Each GPU step has its own time limit; the summary goes to gpurun_out/prof_<tag>.txt and
# gpurun_out/pmc_<config>.json (commit as bench_pmc/pmc_<config>.json: bench.py's roofline.traffic).
# usage: CONFIG=groupby TAG=r03_v3 STEPS=10 tools/gpu_profile.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CONFIG=${CONFIG:-groupby}
TAG=${TAG:-prof}
ARGS="--config $CONFIG ${BENCH_ARGS:-}"
STEPS=${STEPS:-10}
timeout -k 10 600 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-probes $ARGS > gpurun_out/prof_write_segments.log 2>&1 || { echo "segment write failed"; tail -20 gpurun_out/prof_write_segments.log; exit 4; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_trace -o trace -- \
  python3 bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline --no-probes $ARGS > gpurun_out/prof_trace.log 2>&1 || { echo "trace pass failed"; tail -20 gpurun_out/prof_trace.log; exit 5; }
tail -1 gpurun_out/prof_trace.log | cut -c1-300
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d gpurun_out/prof_fetch -o fetch -- \
  python3 bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline --no-probes $ARGS > gpurun_out/prof_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 gpurun_out/prof_fetch.log; exit 6; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d gpurun_out/prof_write -o write -- \
  python3 bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline --no-probes $ARGS > gpurun_out/prof_write.log 2>&1 || { echo "write pass failed"; tail -20 gpurun_out/prof_write.log; exit 7; }
python3 tools/prof_summary.py gpurun_out "gpurun_out/pmc_$CONFIG.json" "$TAG: bench.py $ARGS --steps $STEPS --warmup 2" > "gpurun_out/prof_${TAG}_$CONFIG.txt"
cat "gpurun_out/prof_${TAG}_$CONFIG.txt" | cut -c1-140 | head -30
