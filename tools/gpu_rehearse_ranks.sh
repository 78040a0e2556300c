#!/bin/bash
# Rehearsal of the bench's multi-rank path on a one-GPU box: 2 ranks started by bench.py itself, every rank's engine on GPU 0,
# the collectives over gloo on the host (RCCL refuses two ranks on one device). Exercises the
# per-rank runs, the groupBy key-range exchange (export, partition, all_to_all, merge on the GPU),
# the timeseries all-reduce and the topN gather, the barriers and the max-over-ranks timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in groupby timeseries topn; do
  DG_DIST_BACKEND=gloo DG_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --config $cfg --rows ${ROWS:-400000} --segments 2 \
    --steps 3 --warmup 1 --data-dir /tmp/druid_amd_rehearse > gpurun_out/rehearse_$cfg.json 2> gpurun_out/rehearse_$cfg.err
  rc=$?
  echo "$cfg rc=$rc"; tail -c 400 gpurun_out/rehearse_$cfg.json; echo
  [ $rc -eq 0 ] || { grep -v "^\[" gpurun_out/rehearse_$cfg.err | tail -15; exit $rc; }
done
