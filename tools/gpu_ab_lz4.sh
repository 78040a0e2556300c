#!/bin/bash
# Same-box A/B of LZ4 decoder variants: tools/lz4_profile.py per variant (decoder-only kernel times
# per block kind) and then the headline bench per variant (tools/gpu_ab.sh). VARIANTS="a b" KINDS="seqlong normal".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in default ${VARIANTS:-}; do
  lib=""; [ "$v" = default ] || lib="$PWD/incubator-druid_amd/lib/variants/$v/libdruidgpu.so"
  echo "== $v"
  DRUID_AMD_LIB=$lib timeout -k 10 300 python -u tools/lz4_profile.py ${KINDS:-seqlong normal time uniform3} > gpurun_out/lz4_phases_$v.log 2>&1 || { tail gpurun_out/lz4_phases_$v.log; exit 5; }
  grep -v amdgpu.ids gpurun_out/lz4_phases_$v.log
done
[ -n "${NO_BENCH:-}" ] && exit 0
STEPS=${STEPS:-10} timeout -k 10 900 tools/gpu_ab.sh ${VARIANTS:-}
