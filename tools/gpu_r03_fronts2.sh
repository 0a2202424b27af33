#!/bin/bash
# fronts count A/B on cfg4 (gpurun)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/ab_env.sh r03fr2/ab4 cfg4 "ADAM_BQSR_FRONTS=8" "ADAM_BQSR_FRONTS=16" "ADAM_BQSR_FRONTS=32" "ADAM_BQSR_FRONTS=12" "ADAM_BQSR_FRONTS=21"
