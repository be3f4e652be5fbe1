#!/bin/bash
# rocprofv3 at the round's last commit (reprojection block fetch, fused modulate): K = 4 both views with the traffic
# passes, K = 1 kernel traces. Summaries: tools/summarize_profile.py -> profiles/r03/final_*.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
FIF=4 PASSES="trace fetch write sq" bash tools/gpu_profile.sh r03f_k4 && \
FIF=4 VIEW=surface PASSES="trace fetch write" bash tools/gpu_profile.sh r03f_k4s && \
FIF=1 PASSES=trace bash tools/gpu_profile.sh r03f_k1 && FIF=1 VIEW=surface PASSES=trace bash tools/gpu_profile.sh r03f_k1s
