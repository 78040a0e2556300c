#!/bin/bash
# Round 5: the chase-resolution decoder variant (parity on every LZ4 test stream, per-kind decoder
# times, headline A/B), then the small configs with the overlapped short decoders (parity, bench
# lines, host split). Each step bounded; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/incubator-druid_amd/lib/variants/chase/libdruidgpu.so
DRUID_AMD_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_v6_pytest_lz4_chase.log 2>&1 || { tail -30 gpurun_out/r05_v6_pytest_lz4_chase.log; exit 3; }
tail -2 gpurun_out/r05_v6_pytest_lz4_chase.log
VARIANTS=chase KINDS="normal ulong500 zipfdbl" NO_BENCH=1 timeout -k 10 600 bash tools/gpu_ab_lz4.sh > gpurun_out/r05_v6_lz4_chase.log 2>&1 || { tail -30 gpurun_out/r05_v6_lz4_chase.log; exit 4; }
grep -E "==|kernel=|resolve=" gpurun_out/r05_v6_lz4_chase.log
STEPS=10 timeout -k 10 900 bash tools/gpu_ab.sh chase > gpurun_out/r05_v6_ab_chase_groupby.log 2>&1 || { tail -20 gpurun_out/r05_v6_ab_chase_groupby.log; exit 5; }
cat gpurun_out/r05_v6_ab_chase_groupby.log
bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_scale_gpu.py::test_cfg1_selector_timeseries_on_lz4_hc_segments tests/test_scale_gpu.py::test_cfg2_topn_matches_oracle > /dev/null || { tail -20 gpurun_out/pytest_sel.log; exit 6; }
tail -1 gpurun_out/pytest_sel.log
TAG=r05_v6 STEPS_TO_RUN="secondary" CONFIGS="timeseries topn" bash tools/gpu_round4.sh || exit 7
timeout -k 10 300 python -u tools/small_profile.py timeseries topn > gpurun_out/r05_v6_small_profile.log 2>&1 || { tail -20 gpurun_out/r05_v6_small_profile.log; exit 8; }
head -40 gpurun_out/r05_v6_small_profile.log
