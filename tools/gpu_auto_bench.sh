set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --long-encoding auto > gpurun_out/bench_auto_topn.json 2> gpurun_out/bench_auto_topn.err || { tail -20 gpurun_out/bench_auto_topn.err; exit 4; }
cat gpurun_out/bench_auto_topn.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --config timeseries --long-encoding auto > gpurun_out/bench_auto_ts.json 2> gpurun_out/bench_auto_ts.err || { tail -20 gpurun_out/bench_auto_ts.err; exit 5; }
cat gpurun_out/bench_auto_ts.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_auto -o trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --long-encoding auto > gpurun_out/prof_auto.log 2>&1 || { tail -20 gpurun_out/prof_auto.log; exit 6; }
echo done
