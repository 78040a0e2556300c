#!/bin/bash
# The whole GPU suite + smoke on this build, then quick bench lines (BENCH configs, no profile).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_pytest_gpu.log
tail -4 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 3; }
tail -1 gpurun_out/${TAG}_smoke.log
for cfg in ${BENCH:-}; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 5 --no-cpu-baseline --no-probes > gpurun_out/${TAG}_quick_$cfg.json 2> gpurun_out/${TAG}_quick_$cfg.err || { tail -5 gpurun_out/${TAG}_quick_$cfg.err; exit 4; }
  python3 -c "import json;b=json.loads(open('gpurun_out/${TAG}_quick_$cfg.json').read().strip().splitlines()[-1]);print('$cfg', round(b['ms_per_step'],4), b['roofline']['kernel'], b.get('result_checks',{}))" | cut -c1-400
done
