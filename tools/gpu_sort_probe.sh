#!/bin/bash
# The sort alone (tools/sort_probe.py) for the default library and each variant build, twice, interleaved.
# usage: tools/gpu_sort_probe.sh VARIANT...   (N=100000000 ITERS=10)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for v in default "$@"; do
    lib=""; [ "$v" = default ] || lib="$PWD/incubator-druid_amd/lib/variants/$v/libdruidgpu.so"
    DRUID_AMD_LIB=$lib timeout -k 10 120 python tools/sort_probe.py ${N:-100000000} ${ITERS:-10} || { echo "variant $v failed"; exit 3; }
  done
done
