#!/bin/bash
# Round 5: GPU suite on the current tree, then K0 with / without the public line
# table (tools/vcf_lines_ab.py) and the C2 per-launch-event A/B (tools/ab/c2_events_ab.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_run.sh r05d test smoke || exit 1
timeout -k 10 300 python tools/vcf_lines_ab.py 10 > gpurun_out/r05d/vcf_lines_ab.json 2>&1 || { tail -5 gpurun_out/r05d/vcf_lines_ab.json; exit 1; }
cat gpurun_out/r05d/vcf_lines_ab.json
bash tools/ab/c2_events_ab.sh r05d_c2ev || exit 1
echo DONE
