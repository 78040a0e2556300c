#!/bin/bash
# Scan fast-path check: time-bucketed timeseries parity tests, then ts_hourly flow-grid A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 900 python -u -m pytest tests/test_cfg5_gpu.py tests/test_calendar_gpu.py tests/test_gpu_parity.py tests/test_filtered_gpu.py tests/test_incremental_gpu.py tests/test_scale_gpu.py tests/test_limit_pushdown_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
CONFIG=ts_hourly VARIANTS="DG_FLOW_WGS=256" STEPS=10 bash tools/gpu_env_ab.sh > gpurun_out/${TAG}_ab_ts_hourly.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_ts_hourly.log; exit 5; }
cat gpurun_out/${TAG}_ab_ts_hourly.log
