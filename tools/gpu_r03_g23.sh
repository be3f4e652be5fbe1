# under the 4-wide walk: fine-leaf size, and nearest-first order for the shadow rays' children
cd "$GRAFT_REPO_ROOT"
REPS=2 bash tools/env_ab_views.sh PTSVGF_FINE_LEAVES 4 2 1 8 || exit $?
L=$GRAFT_REPO_ROOT/path-tracing-svgf_amd
REPS=2 bash tools/env_ab_views.sh PTSVGF_LIB_DIR $L/lib $L/lib_exp/ssort
