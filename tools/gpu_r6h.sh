#!/bin/bash
# Early-decode check: timeseries parity tests over several segments, interruption tests, then ts_hourly
# host trace and a quick line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 900 python -u -m pytest tests/test_cfg5_gpu.py tests/test_calendar_gpu.py tests/test_interrupt_gpu.py tests/test_merge_devices.py tests/test_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
DG_HOST_TRACE=1 timeout -k 10 600 python -u bench.py --config ts_hourly --steps 3 --warmup 1 --no-cpu-baseline --no-probes \
  > gpurun_out/${TAG}_trace_ts_hourly.json 2> gpurun_out/${TAG}_trace_ts_hourly.err || { tail -5 gpurun_out/${TAG}_trace_ts_hourly.err; exit 3; }
grep "dg host" gpurun_out/${TAG}_trace_ts_hourly.err | tail -3 | cut -c1-300
for cfg in ts_hourly groupby_hourly; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-probes > gpurun_out/${TAG}_quick_$cfg.json 2> gpurun_out/${TAG}_quick_$cfg.err || { tail -5 gpurun_out/${TAG}_quick_$cfg.err; exit 4; }
  python3 -c "import json;b=json.loads(open('gpurun_out/${TAG}_quick_$cfg.json').read().strip().splitlines()[-1]);print('$cfg', round(b['ms_per_step'],4), {k: round(v,3) for k,v in b['phases_ms'].items()})" | cut -c1-400
done
