cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
RANKS="8" N=27 TAG=r5hypre EXTRA="--inner hypre" timeout -k 10 600 bash tools/rehearse_dist.sh || exit 1
RANKS="1" N=27 TAG=r5hypreR8_ EXTRA="--inner hypre --opt pls.hypre_ranks=8" timeout -k 10 600 bash tools/rehearse_dist.sh || exit 1
RANKS="1" N=27 TAG=r5hypre1_ EXTRA="--inner hypre" timeout -k 10 600 bash tools/rehearse_dist.sh
