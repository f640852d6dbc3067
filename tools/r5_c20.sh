cd "${GRAFT_REPO_ROOT:-/root/repo}"
TLIM=500 bash tools/r5_rob.sh footing exact || exit $?
NS="10 20" TLIM=300 bash tools/r5_rob.sh footing inexact
