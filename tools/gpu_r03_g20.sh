cd "$GRAFT_REPO_ROOT"
REPS=2 bash tools/uniform_ab_views.sh wide_bvh 0 1
