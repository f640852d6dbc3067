cd "${GRAFT_REPO_ROOT:-/root/repo}"
ANCHOR=k_spmv_short SKIP=60 bash tools/r5_trace.sh hyp_on --inner hypre --opt pls.fp_pipeline=1 | head -30
ANCHOR=k_spmv_short SKIP=60 bash tools/r5_trace.sh hyp_off --inner hypre --opt pls.fp_pipeline=0 | head -30
