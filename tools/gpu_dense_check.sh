#!/bin/bash
# Dense LZ4 decoder check: GPU LZ4 tests (both routes), decoder-only kernel times per block kind with
# and without the dense decoder (and the pending general-decoder patch variant when built), then the
# headline bench A/B (default vs DG_LZ4_NO_DENSE=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dense_lz4tests.log 2>&1
rc=$?; echo "lz4 gpu tests rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/dense_lz4tests.log | cut -c1-200 | tail -30
[ $rc -eq 0 ] || exit $rc
KINDS=${KINDS:-seqlong normal time uniform3 ulong500 mix}
echo "== dense"; timeout -k 10 300 python -u tools/lz4_profile.py $KINDS > gpurun_out/lz4_phases_dense.log 2>&1 || { tail gpurun_out/lz4_phases_dense.log; exit 5; }
grep -v amdgpu.ids gpurun_out/lz4_phases_dense.log
echo "== general"; DG_LZ4_NO_DENSE=1 timeout -k 10 300 python -u tools/lz4_profile.py $KINDS > gpurun_out/lz4_phases_general.log 2>&1 || { tail gpurun_out/lz4_phases_general.log; exit 5; }
grep -v amdgpu.ids gpurun_out/lz4_phases_general.log
if false; then
  echo "== general, pending resolve patch"; DRUID_AMD_LIB=$PWD/incubator-druid_amd/lib/variants/resolve/libdruidgpu.so timeout -k 10 300 python -u tools/lz4_profile.py $KINDS > gpurun_out/lz4_phases_resolve.log 2>&1 || { tail gpurun_out/lz4_phases_resolve.log; exit 5; }
  grep -v amdgpu.ids gpurun_out/lz4_phases_resolve.log
fi
[ -n "${NO_BENCH:-}" ] && exit 0
STEPS=${STEPS:-10} timeout -k 10 900 tools/gpu_ab.sh env:DG_LZ4_NO_DENSE
