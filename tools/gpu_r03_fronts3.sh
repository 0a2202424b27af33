#!/bin/bash
# fronts A/B on one box, cfg4, final reduce (gpurun)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/ab_env.sh r03fr5/ab4 cfg4 "ADAM_BQSR_FRONTS=0" "ADAM_BQSR_X=default" "ADAM_BQSR_FRONTS=6" "ADAM_BQSR_FRONTS=0" "ADAM_BQSR_X=default" "ADAM_BQSR_FRONTS=6"
