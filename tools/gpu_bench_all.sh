#!/bin/bash
# Secondary bench lines (every config of bench.py except the headline), one GPU step each with its own
# time limit; the 1B-row hourly datasets are written on the box first (parallel writers), LZ4-HC like the
# reference's CompressionStrategy.LZ4 (lz4High, CompressionStrategy.java:310).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CONFIGS:-topn_numeric topn_alphanumeric timeseries groupby filtered ts_hourly groupby_hourly}; do
  mode=${LZ4_MODE:-hc}  # the reference writes LZ4 blocks with lz4-java's high compressor
  timeout -k 10 900 python -u bench.py --config "$cfg" --steps 5 --warmup 1 --cpu-seconds 8 --lz4-mode "$mode" \
    > "gpurun_out/bench_$cfg.json" 2> "gpurun_out/bench_$cfg.err" || { echo "$cfg failed"; tail -5 "gpurun_out/bench_$cfg.err"; exit 4; }
  cut -c1-240 "gpurun_out/bench_$cfg.json"
done
