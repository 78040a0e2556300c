#!/bin/bash
# Round-6 GPU session: selected parity tests (TESTS, -k KEXPR), then the headline bench (BENCH_ARGS).
# Every GPU step has its own time limit; a fault, abort or timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v ${KEXPR:+-k "$KEXPR"} --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/${TAG}_pytest.log
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_pytest.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BENCH:-}" ]; then
  for cfg in $BENCH; do
    timeout -k 10 900 python -u bench.py --config "$cfg" ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_$cfg.json \
      2> gpurun_out/${TAG}_bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/${TAG}_bench_$cfg.err; exit 4; }
    cut -c1-1500 gpurun_out/${TAG}_bench_$cfg.json
  done
fi
