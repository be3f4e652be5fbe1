# occupancy of the traversal kernels (waves per SIMD) and fine-leaf size, same box
cd "$GRAFT_REPO_ROOT"
L="$GRAFT_REPO_ROOT/path-tracing-svgf_amd"
REPS=2 bash tools/env_ab_views.sh PTSVGF_LIB_DIR $L/lib $L/lib_exp/w5 $L/lib_exp/w6 || exit $?
REPS=2 bash tools/env_ab_views.sh PTSVGF_FINE_LEAVES 0 4
