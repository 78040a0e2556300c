#!/bin/bash
# Same-box A/B of the default library against variant builds (incubator-druid_amd/lib/variants/<name>)
# on bench configs: VARIANTS="base" CONFIGS="ts_hourly groupby" STEPS=10 tools/gpu_lib_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for cfg in ${CONFIGS:-ts_hourly}; do
    for v in default ${VARIANTS:-}; do
      lib=""; [ "$v" = default ] || lib="$PWD/incubator-druid_amd/lib/variants/$v/libdruidgpu.so"
      DRUID_AMD_LIB=$lib timeout -k 10 600 python -u bench.py --config $cfg --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-probes \
        > gpurun_out/libab.json 2> gpurun_out/libab.err || { tail -5 gpurun_out/libab.err; exit 3; }
      python3 -c "
import json; b=json.loads(open('gpurun_out/libab.json').read().strip().splitlines()[-1])
print('$round $cfg $v', round(b['ms_per_step'],4), {k: round(x,3) for k,x in b['phases_ms'].items()})" | cut -c1-260
    done
  done
done
