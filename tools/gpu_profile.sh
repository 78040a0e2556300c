#!/bin/bash
# rocprofv3 evidence for the bench line: kernel trace + stats, then a separate PMC pass for HBM bytes
# (FETCH_SIZE / WRITE_SIZE need separate passes on gfx950). Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-}
STEPS=${STEPS:-10}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_trace -o trace -- \
  python3 bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline $ARGS > gpurun_out/prof_trace.log 2>&1 || { echo "trace pass failed"; tail -20 gpurun_out/prof_trace.log; exit 5; }
tail -1 gpurun_out/prof_trace.log
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d gpurun_out/prof_fetch -o fetch -- \
  python3 bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline $ARGS > gpurun_out/prof_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 gpurun_out/prof_fetch.log; exit 6; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d gpurun_out/prof_write -o write -- \
  python3 bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline $ARGS > gpurun_out/prof_write.log 2>&1 || { echo "write pass failed"; tail -20 gpurun_out/prof_write.log; exit 7; }
find gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write -name "*.csv" | head -20
