# triangle tests per ray (PT_NODE_VISIT=0 build) by fine-leaf size
cd "$GRAFT_REPO_ROOT"
export PTSVGF_LIB_DIR="$GRAFT_REPO_ROOT/path-tracing-svgf_amd/lib_exp/tris"
REPS=1 bash tools/env_ab_views.sh PTSVGF_FINE_LEAVES 0 1 4
