set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
bash tools/pmc.sh || exit $?
