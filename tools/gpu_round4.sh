#!/bin/bash
# Round-4 measurement set on one GPU box: the GPU test suite, smoke(), the headline bench line (with
# the CPU baseline and per-group checks), the secondary bench lines (each with result_checks), and the
# headline's rocprofv3 kernel trace. Each GPU step has its own time limit; the script stops at the
# first failure. STEPS_TO_RUN selects parts: tests smoke bench secondary prof (default: all).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04}
PARTS=${STEPS_TO_RUN:-tests smoke bench secondary prof}
for part in $PARTS; do
  case $part in
    tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/${TAG}_pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG}_pytest_gpu.log; tail -3 gpurun_out/${TAG}_pytest_gpu.log
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 600 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 900 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
      rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
      python3 -c "
import json; b=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print(b['ms_per_step'], b['value'], {k: round(v,3) for k,v in b['phases_ms'].items()})
print('roofline', {k: b['roofline'][k] for k in ('kernel','achieved','frac','avg_launch_ms')})
print('checks', b.get('result_checks')); print('cpu', {k: b['cpu_baseline'][k] for k in ('value','cores')})" ;;
    secondary)
      for cfg in ${CONFIGS:-timeseries topn filtered ts_hourly groupby_hourly topn_numeric topn_alphanumeric}; do
        timeout -k 10 900 python -u bench.py --config "$cfg" --steps ${SEC_STEPS:-10} --warmup 2 \
          > gpurun_out/${TAG}_bench_$cfg.json 2> gpurun_out/${TAG}_bench_$cfg.err || { echo "$cfg failed"; tail -5 gpurun_out/${TAG}_bench_$cfg.err; exit 4; }
        python3 -c "
import json; b=json.loads(open('gpurun_out/${TAG}_bench_$cfg.json').read().strip().splitlines()[-1])
print('$cfg', round(b['ms_per_step'],3), '%.3g' % b['value'], b['roofline']['kernel'], '%.4f' % (b['roofline']['frac'] or 0), 'checks:', {k: v for k, v in (b.get('result_checks') or {}).items() if isinstance(v, bool)}, 'cpu', '%.3g' % b['cpu_baseline']['value'], b['cpu_baseline']['cores'])"
      done ;;
    prof)
      CONFIG=groupby TAG=${TAG}_groupby STEPS=10 timeout -k 10 1200 bash tools/gpu_profile.sh > gpurun_out/${TAG}_prof.log 2>&1
      rc=$?; tail -25 gpurun_out/${TAG}_prof.log; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
