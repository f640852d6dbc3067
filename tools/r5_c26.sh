cd "${GRAFT_REPO_ROOT:-/root/repo}"
ANCHOR=k_mdot SKIP=60 COUNT=16 BEFORE=12 bash tools/r5_trace.sh hyp_on2 --inner hypre --opt pls.fp_pipeline=1 | head -20
