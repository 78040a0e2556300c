#!/bin/bash
# topN selection check + quick lines, then the ts_hourly decoder placement A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "topn or TopN or top_n" --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in topn topn_numeric; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 5 --no-cpu-baseline --no-probes > gpurun_out/${TAG}_quick_$cfg.json 2> gpurun_out/${TAG}_quick_$cfg.err || { tail -5 gpurun_out/${TAG}_quick_$cfg.err; exit 4; }
  python3 -c "import json;b=json.loads(open('gpurun_out/${TAG}_quick_$cfg.json').read().strip().splitlines()[-1]);print('$cfg', round(b['ms_per_step'],4))"
done
CONFIG=ts_hourly VARIANTS="DG_FLOW_WGS=192 DG_FLOW_WGS=256 DG_FLOW_WGS=192,DG_GEN_FIRST=1" STEPS=10 bash tools/gpu_env_ab.sh > gpurun_out/${TAG}_ab_ts_hourly.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_ts_hourly.log; exit 5; }
cat gpurun_out/${TAG}_ab_ts_hourly.log
