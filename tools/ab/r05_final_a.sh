#!/bin/bash
# Round-5 measurement (part A): GPU suite, smoke and every bench line on one box.
#   tools/ab/r05_final_a.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r05fa}
bash tools/gpu_run.sh "$T" test smoke c2 c1 c4k vcf load c5 c3 c4 dropin gloo2 || exit 1
echo DONE-A
