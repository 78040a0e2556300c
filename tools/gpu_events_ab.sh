#!/bin/bash
# Same-box A/B: small configs with and without the phase-timing events (DG_NO_PHASE_EVENTS=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in on off; do e=""; [ $v = off ] && e="DG_NO_PHASE_EVENTS=1"; for c in timeseries topn; do env $e timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ev_${v}_$c.json 2>gpurun_out/ev_${v}_$c.err || exit 3; python3 -c "import json; b=json.loads(open(\"gpurun_out/ev_${v}_$c.json\").read().strip().splitlines()[-1]); print(\"$v $c\", round(b[\"ms_per_step\"],4))"; done; done
