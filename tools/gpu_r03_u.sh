#!/bin/bash
# apply kApplyU A/B (gpurun): kernel stats of candidate libraries
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/ab_lib.sh r03u "cfg2" - "$R/tools/probe/lib_u3.so" "$R/tools/probe/lib_u5.so" "$R/tools/probe/lib_u6.so"
echo done
