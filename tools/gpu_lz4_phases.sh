set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lz4_profile.py seqlong normal > gpurun_out/lz4_phases_win.log 2>&1 || { tail gpurun_out/lz4_phases_win.log; exit 5; }
cat gpurun_out/lz4_phases_win.log
