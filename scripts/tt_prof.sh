cd "$GRAFT_REPO_ROOT" || exit 9
export ABL_TOPO=TT
bash scripts/profile_edge_counters.sh || exit $?
bash scripts/edge_lds_counters.sh || exit $?
