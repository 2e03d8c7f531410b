# one call for two A/Bs (the pool is busy): tools/gpu_r4x.sh (shared-state event without the
# system fence) then tools/gpu_r4y.sh (V1 ranks by value, then the GPU suite on the new build)
set -e
bash "$GRAFT_REPO_ROOT/tools/gpu_r4x.sh"
bash "$GRAFT_REPO_ROOT/tools/gpu_r4y.sh"
