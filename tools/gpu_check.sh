#!/bin/bash
# One GPU session: parity tests, smoke, short bench. Each GPU step has its own time limit; a fault,
# abort or timeout (any exit status other than 0/1 from pytest) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py --steps "$STEPS" --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.log
