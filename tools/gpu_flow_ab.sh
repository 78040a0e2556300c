#!/bin/bash
# Flow decoder check + same-box A/B: the LZ4 parity tests (every route), the decoder-only profile of the
# flow kinds with the flow decoder on and off (DG_NO_FLOW_DECODE=1: k_lz4_decode), then bench lines.
# KINDS="normal zipfdbl ulong500" CONFIGS="groupby ts_hourly" TAG=...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-flow}
if [ -z "${NO_TESTS:-}" ]; then
  bash tools/gpu_tests.sh tests/test_lz4_gpu.py ${TESTS:-} || exit 3
fi
for v in flow noflow; do
  env=""; [ $v = noflow ] && env="DG_NO_FLOW_DECODE=1"
  env $env timeout -k 10 300 python -u tools/lz4_profile.py ${KINDS:-normal zipfdbl ulong500} > gpurun_out/${TAG}_lz4_$v.log 2>&1 \
    || { tail gpurun_out/${TAG}_lz4_$v.log; exit 5; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${TAG}_lz4_$v.log
done
for cfg in ${CONFIGS:-groupby ts_hourly}; do
  for v in flow noflow; do
    env=""; [ $v = noflow ] && env="DG_NO_FLOW_DECODE=1"
    env $env timeout -k 10 600 python -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/${TAG}_bench_${cfg}_$v.json 2> gpurun_out/${TAG}_bench_${cfg}_$v.err || { tail -5 gpurun_out/${TAG}_bench_${cfg}_$v.err; exit 6; }
    python3 -c "
import json; b=json.loads(open('gpurun_out/${TAG}_bench_${cfg}_$v.json').read().strip().splitlines()[-1])
print('$cfg $v', round(b['ms_per_step'],3), {k: round(x,3) for k,x in b['phases_ms'].items()}, {k: v for k, v in (b.get('result_checks') or {}).items() if isinstance(v, bool)})"
  done
done
