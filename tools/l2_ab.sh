#!/bin/bash
# L2 hit rates of the traversal kernels for two library builds (the 4-wide node stride A/B): rocprofv3 TCC_HIT /
# TCC_MISS passes of the 4K bench at K = 4 on both views, plus the scene's working-set sizes (PTSVGF_SCENE_INFO).
R=$GRAFT_REPO_ROOT
PTSVGF_SCENE_INFO=1 timeout -k 10 300 python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-1080p --no-extras \
  2>&1 >/dev/null | grep "ptsvgf scene" | head -1
for L in lib lib_exp/s8; do
  for V in default surface; do
    N=$(echo $L | tr / _)_$V
    PTSVGF_LIB_DIR="$R/path-tracing-svgf_amd/$L" FIF=4 VIEW=$V PASSES="l2" timeout -k 10 600 bash "$R/tools/gpu_profile.sh" "l2_$N" \
      > /dev/null || exit 1
  done
done
echo l2-done
