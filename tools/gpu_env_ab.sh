#!/bin/bash
# Same-box A/B of engine environment switches on one bench config: VARIANTS="A=1 B=high" (each an
# env assignment, "none" for the default), CONFIG=groupby. Prints ms/step and the phases per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CONFIG=${CONFIG:-groupby}
for round in 1 2; do
  for v in none ${VARIANTS:-}; do
    e=""; [ "$v" = none ] || e="${v//,/ }"
    env $e timeout -k 10 600 python -u bench.py --config $CONFIG --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
      > gpurun_out/envab_$round.json 2> gpurun_out/envab_$round.err || { tail -5 gpurun_out/envab_$round.err; exit 3; }
    python3 -c "
import json; b=json.loads(open('gpurun_out/envab_$round.json').read().strip().splitlines()[-1])
print('$round $v', round(b['ms_per_step'],3), {k: round(x,2) for k,x in b['phases_ms'].items()})"
  done
done
