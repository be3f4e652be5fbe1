#!/bin/bash
# a-trous A/B, then the full GPU session
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_atrous.py > gpurun_out/ba.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -12 gpurun_out/ba.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_session.sh
