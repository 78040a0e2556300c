#!/bin/bash
# Round-6 session: parity tests of the decode switches, then same-box A/B of the flow-decoder grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_scale_gpu.py tests/test_lz4_gpu.py} -m gpu -x -q \
  -k "${KEXPR:-cfg3_groupby_sort_paths or decoder_stream_switches or lz4}" --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/sort_probe.py 100000000 10 > gpurun_out/${TAG}_sort_probe.log 2>&1 || exit 3
grep sort gpurun_out/${TAG}_sort_probe.log
for cfg in ${CONFIGS:-groupby}; do
  CONFIG=$cfg VARIANTS="${VARIANTS:-DG_FLOW_WGS=160 DG_FLOW_WGS=224 DG_FLOW_WGS=0,DG_GEN_FIRST=0}" STEPS=${STEPS:-20} \
    bash tools/gpu_env_ab.sh > gpurun_out/${TAG}_ab_$cfg.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_$cfg.log; exit 4; }
  cat gpurun_out/${TAG}_ab_$cfg.log
done
