#!/bin/bash
# Same-box A/B of library variants on the headline bench: tools/gpu_ab.sh VARIANT... (built with
# tools/build_variant.sh). Each variant and the default library run twice, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
STEPS=${STEPS:-10}
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then lib=""; else lib="$PWD/incubator-druid_amd/lib/variants/$v/libdruidgpu.so"; fi
    DRUID_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline \
      > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.err; exit 1; }
    python -c "
import json,sys
b=[json.loads(l) for l in open('gpurun_out/ab_$v.json') if l.startswith('{')][-1]
print('$v', round(b['ms_per_step'],3), {k: round(x,3) for k,x in b['phases_ms'].items()})"
  done
done
