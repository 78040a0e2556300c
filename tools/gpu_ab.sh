#!/bin/bash
# Same-box A/B of library variants on the headline bench: tools/gpu_ab.sh VARIANT... (built with
# tools/build_variant.sh) or env:VAR; CONFIG=<bench config> (default groupby). Each variant and the
# default library run twice, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
STEPS=${STEPS:-10}
CONFIG=${CONFIG:-groupby}
for round in 1 2; do
  for v in default "$@"; do
    # a variant is a library build (tools/build_variant.sh NAME) or env:VAR (the default library with VAR=1)
    envs=""; lib=""
    case "$v" in default) ;; env:*) envs="${v#env:}=1" ;; *) lib="$PWD/incubator-druid_amd/lib/variants/$v/libdruidgpu.so" ;; esac
    env $envs DRUID_AMD_LIB=$lib timeout -k 10 300 python bench.py --config $CONFIG --steps $STEPS --warmup 2 --no-cpu-baseline \
      > gpurun_out/ab_${v#env:}.json 2> gpurun_out/ab_${v#env:}.err || { echo "variant $v failed"; tail -5 gpurun_out/ab_${v#env:}.err; exit 1; }
    python -c "
import json,sys
b=[json.loads(l) for l in open('gpurun_out/ab_${v#env:}.json') if l.startswith('{')][-1]
print('$v', round(b['ms_per_step'],3), {k: round(x,3) for k,x in b['phases_ms'].items()})"
  done
done
