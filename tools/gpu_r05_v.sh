#!/bin/bash
# r05v: cfg2 timing probes -- prep (listed reads, bitmap atomics, word-store form)
# and observe (base-code loads, qual loads)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_ab.sh r05v cfg2 "" "LIB=adam_amd/ab/libadam_bqsr_prep_no_list.so" \
  "LIB=adam_amd/ab/libadam_bqsr_prep_no_atomics.so" "LIB=adam_amd/ab/libadam_bqsr_prep_store.so" \
  "LIB=adam_amd/ab/libadam_bqsr_obs_no_base_loads.so" "LIB=adam_amd/ab/libadam_bqsr_obs_one_qual_load.so"
