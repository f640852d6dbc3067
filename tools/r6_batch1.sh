#!/bin/bash
# round 6: window depth A/B, headline fp-pipeline A/B, then the harness's fast cases
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash tools/r6_sweep_variants.sh swelling 80 diagonal 6 "" "pls.window_depth=3" || exit $?
bash tools/r6_ab.sh "" "pls.fp_pipeline_cus=12" "pls.fp_pipeline=0" || exit $?
SET=exact TL=240 bash tools/r6_rob.sh swelling 10 diagonal swelling 40 diagonal swelling 160 diagonal \
    swelling 10 "diagonal 3-way" swelling 160 "diagonal 3-way" footing 10 undrained footing 80 undrained \
    footing 10 "undrained 3-way" footing 80 "undrained 3-way" || exit $?
SET=inexact TL=240 bash tools/r6_rob.sh swelling 10 diagonal swelling 20 diagonal swelling 40 diagonal \
    swelling 80 diagonal swelling 10 "diagonal 3-way" swelling 20 "diagonal 3-way" swelling 40 "diagonal 3-way" \
    footing 10 undrained footing 20 undrained footing 40 undrained footing 10 "undrained 3-way" \
    footing 40 "undrained 3-way" || exit $?
