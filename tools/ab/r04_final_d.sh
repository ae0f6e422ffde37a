#!/bin/bash
# Round-end measurement after the grid changes (part 1: tests, smoke, bench lines).
#   tools/ab/r04_final_d.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r04fe}
bash tools/gpu_run.sh "$T" test smoke c2 c1 c4k vcf load c5 c3 c4 dropin gloo2 || exit 1
echo DONE-D
