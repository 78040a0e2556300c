set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_lz4_gpu.py -m gpu -v --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_win.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_win.log; grep -E "PASSED|FAILED|Error|first diff" gpurun_out/pytest_win.log | cut -c1-300 | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/lz4_profile.py seqlong time normal > gpurun_out/lz4_phases_win.log 2>&1 || { tail gpurun_out/lz4_phases_win.log; exit 5; }
cat gpurun_out/lz4_phases_win.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_win.json 2> gpurun_out/bench_win.err || { tail -20 gpurun_out/bench_win.err; exit 4; }
python3 -c "
import json; b=json.loads(open('gpurun_out/bench_win.json').read().strip().splitlines()[-1]); print(b['ms_per_step'], b['phases_ms'], b['result_checks'].get('per_group_equal'))"
