#!/bin/bash
# Timeseries fold / scan-skip check: the timeseries parity tests, then quick lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -k "${KEXPR:-timeseries or Timeseries or fused or cfg1 or filter or Filter or kats or calendar or incremental or cfg5 or interrupt or parity}" --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${BENCH:-timeseries filtered}; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --warmup 5 --no-probes --cpu-seconds 3 > gpurun_out/${TAG}_quick_$cfg.json 2> gpurun_out/${TAG}_quick_$cfg.err || { tail -5 gpurun_out/${TAG}_quick_$cfg.err; exit 4; }
  python3 -c "import json;b=json.loads(open('gpurun_out/${TAG}_quick_$cfg.json').read().strip().splitlines()[-1]);print('$cfg', round(b['ms_per_step'],4), b['roofline']['kernel'], b.get('result_checks',{}))" | cut -c1-400
done
