#!/bin/bash
# round 6 final robustness refresh (TL 280 s per outer solve; reason -100 = cut)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
SET=inexact TL=280 bash tools/r6_rob.sh "$@"
