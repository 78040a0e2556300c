#!/bin/bash
# Sort change check: probe (sortedness + time), the sort-using parity tests, then the headline evidence.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 120 python tools/sort_probe.py 100000000 10 > gpurun_out/${TAG}_sort_probe.log 2>&1 || { cat gpurun_out/${TAG}_sort_probe.log | tail -5; exit 3; }
grep sort gpurun_out/${TAG}_sort_probe.log
timeout -k 10 900 python -u -m pytest tests/test_scale_gpu.py tests/test_merge_gpu.py tests/test_limit_pushdown_gpu.py tests/test_merge_devices.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
[ -n "${NO_HEADLINE:-}" ] && exit 0
TAG=$TAG bash tools/gpu_headline.sh
