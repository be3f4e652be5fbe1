#!/bin/bash
# rocprofv3 at the headline configuration on HEAD's library (SLP off, 4-wide any-hit walk): K = 4, both views,
# kernel trace + PMC passes; then K = 1 kernel traces (each kernel alone). Summaries: tools/summarize_profile.py.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
FIF=4 bash tools/gpu_profile.sh r03h_k4 && FIF=4 VIEW=surface bash tools/gpu_profile.sh r03h_k4s && \
FIF=1 PASSES=trace bash tools/gpu_profile.sh r03h_k1 && FIF=1 VIEW=surface PASSES=trace bash tools/gpu_profile.sh r03h_k1s
