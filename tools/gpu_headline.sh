#!/bin/bash
# Headline evidence on one build: sort probe, rocprofv3 trace + PMC passes (tools/gpu_profile.sh), then
# the bench line reading that profile's bench_pmc json. TAG names the files.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r06}
CONFIG=${CONFIG:-groupby}
timeout -k 10 120 python tools/sort_probe.py 100000000 10 > gpurun_out/${TAG}_sort_probe.log 2>&1 || exit 3
grep sort gpurun_out/${TAG}_sort_probe.log
CONFIG=$CONFIG TAG=$TAG STEPS=${PSTEPS:-10} bash tools/gpu_profile.sh > gpurun_out/${TAG}_profile_$CONFIG.log 2>&1 || { tail -20 gpurun_out/${TAG}_profile_$CONFIG.log; exit 4; }
head -12 gpurun_out/prof_${TAG}_$CONFIG.txt | cut -c1-160
mkdir -p bench_pmc && cp gpurun_out/pmc_$CONFIG.json bench_pmc/pmc_$CONFIG.json
timeout -k 10 600 python -u bench.py --config $CONFIG --steps ${STEPS:-20} --warmup 3 > gpurun_out/${TAG}_bench_$CONFIG.json 2> gpurun_out/${TAG}_bench_$CONFIG.err || { tail -20 gpurun_out/${TAG}_bench_$CONFIG.err; exit 5; }
cut -c1-2500 gpurun_out/${TAG}_bench_$CONFIG.json
