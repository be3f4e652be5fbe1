cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/path-tracing-svgf_amd
REPS=2 bash tools/env_ab_views.sh PTSVGF_LIB_DIR $L/lib $L/lib_exp/r6 $L/lib_exp/sh6 $L/lib_exp/r8
