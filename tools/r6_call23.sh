#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash tools/r6_sweep_ab.sh d160 swelling 160 || exit $?
bash tools/r6_sweep_ab.sh d160nl swelling 160 pls.ring_probe=32768 || exit $?
bash tools/r6_sweep_ab.sh d160ns swelling 160 pls.ring_probe=34816 || exit $?
