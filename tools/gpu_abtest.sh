#!/bin/bash
# GPU tests (quiet) then A/B of the working tree against build_ab/REV.
# usage: bash tools/gpu_abtest.sh REV "CONFIGS" VARIANTS
set -o pipefail
bash tools/gpu_tests.sh || exit 1
bash tools/gpu_abrev.sh "$@"
