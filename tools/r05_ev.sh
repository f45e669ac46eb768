#!/bin/bash
# Round 5: k_fragment counters of the product build vs the all-table variant, then the round evidence.
set -o pipefail
export TMPDIR=/tmp
bash tools/variant_pmc.sh gpurun_out/r05/vpmc base alltab 2>&1 | tee gpurun_out/r05/alltab_pmc.txt || exit 1
bash tools/round_evidence.sh gpurun_out/ev_r05 || exit 1
