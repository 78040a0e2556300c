#!/bin/bash
# LZ4 decoder A/B on one box: parity of the decoder tests, per-kind kernel times (tools/lz4_profile.py),
# then the headline bench with the light decoder on and off (DG_LZ4_NO_LIGHT=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_lz4_gpu.py} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lz4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lz4_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/lz4_profile.py > gpurun_out/lz4_phases.log 2>&1 || { tail -5 gpurun_out/lz4_phases.log; exit 3; }
grep -E "kernel=" gpurun_out/lz4_phases.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_light.json 2> gpurun_out/bench_light.err || { tail -5 gpurun_out/bench_light.err; exit 4; }
cut -c1-200 gpurun_out/bench_light.json; python -c "import json;d=json.load(open('gpurun_out/bench_light.json'));print(d['phases_ms'], d['roofline'])"
DG_LZ4_NO_LIGHT=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_nolight.json 2> gpurun_out/bench_nolight.err || { tail -5 gpurun_out/bench_nolight.err; exit 5; }
python -c "import json;d=json.load(open('gpurun_out/bench_nolight.json'));print('nolight', d['ms_per_step'], d['phases_ms'])"
