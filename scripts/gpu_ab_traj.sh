cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_ab.sh ab_traj base traj192 traj160 traj128 base traj160 traj128 2>&1
