#!/bin/bash
# LZF variant of the headline: bench line + rocprofv3 kernel stats (k_lzf_decode).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --compression lzf --cpu-seconds 6 > gpurun_out/bench_lzf.json 2> gpurun_out/bench_lzf.err || { tail -20 gpurun_out/bench_lzf.err; exit 4; }
cat gpurun_out/bench_lzf.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_lzf -o trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --compression lzf > gpurun_out/prof_lzf.log 2>&1 || { tail -20 gpurun_out/prof_lzf.log; exit 6; }
echo done
