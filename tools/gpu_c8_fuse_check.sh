#!/bin/bash
# Class-8 decoder + fused timeseries check: LZ4 and configs[4] GPU tests, decoder-only kernel times
# per block kind (default routes vs every block on the general decoder), then same-box A/Bs: the
# headline (default vs DG_LZ4_NO_C8=1) and ts_hourly (default vs DG_NO_FUSE=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lz4_gpu.py tests/test_cfg5_gpu.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/c8_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/c8_tests.log | cut -c1-200 | tail -40
[ $rc -eq 0 ] || exit $rc
KINDS=${KINDS:-seqlong time normal mix}
echo "== default routes"; timeout -k 10 300 python -u tools/lz4_profile.py $KINDS > gpurun_out/lz4_phases_c8.log 2>&1 || { tail gpurun_out/lz4_phases_c8.log; exit 5; }
grep -v amdgpu.ids gpurun_out/lz4_phases_c8.log
echo "== general"; DG_LZ4_NO_C8=1 DG_LZ4_NO_DENSE=1 timeout -k 10 300 python -u tools/lz4_profile.py $KINDS > gpurun_out/lz4_phases_gen.log 2>&1 || { tail gpurun_out/lz4_phases_gen.log; exit 5; }
grep -v amdgpu.ids gpurun_out/lz4_phases_gen.log
[ -n "${NO_BENCH:-}" ] && exit 0
STEPS=${STEPS:-10} timeout -k 10 600 tools/gpu_ab.sh env:DG_LZ4_NO_C8 || exit 6
# (the first ts_hourly run writes 8 x 15.6 M-row segments: a progress file while the steps run, each
# under its own time limit)
( while sleep 50; do date > gpurun_out/c8_heartbeat; done ) &
hb=$!
CONFIG=ts_hourly STEPS=${STEPS:-10} timeout -k 10 900 tools/gpu_ab.sh env:DG_NO_FUSE
rc=$?
kill $hb
exit $((rc ? 7 : 0))
