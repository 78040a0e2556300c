set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  lib=""; [ "$v" = default ] || lib="$PWD/incubator-druid_amd/lib/variants/$v/libdruidgpu.so"
  echo "== $v"
  DRUID_AMD_LIB=$lib timeout -k 10 300 python -u tools/lz4_profile.py ${KINDS:-seqlong normal} > gpurun_out/lz4_phases_$v.log 2>&1 || { tail gpurun_out/lz4_phases_$v.log; exit 5; }
  grep -v amdgpu.ids gpurun_out/lz4_phases_$v.log
done
