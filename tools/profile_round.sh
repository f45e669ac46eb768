#!/bin/bash
# Round profile of the default bench workload (run on the GPU box):
#   1. rocprofv3 --kernel-trace --stats        -> <out>/trace/run_kernel_stats.csv
#   2. rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ counters) -> <out>/pmc*/...
#   3. tools/pmc_summary.py -> per-kernel averages over the timed dispatches, and pmc_traffic.json
# Usage: bash tools/profile_round.sh gpurun_out/prof_rNN
#   env: STEPS, BENCH_EXTRA (extra bench.py args), WORKLOAD (pmc_traffic.json key), TRACE_ONLY=1
set -o pipefail
OUT=${1:-gpurun_out/prof}
STEPS=${STEPS:-20}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOTDIR=$(pwd)
BARGS="--steps $STEPS --warmup 2 --no-cpu-baseline $BENCH_EXTRA"
WORKLOAD=${WORKLOAD:-full/P_over/3840x2160/N1}
TRACE_ONLY=${TRACE_ONLY:-0}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/$OUT/trace" -o run --output-format csv -- python3 bench.py $BARGS > "$OUT/trace.log" 2>&1 || exit 1
[ "$TRACE_ONLY" = 1 ] && exit 0
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$ROOTDIR/$OUT/pmc$i" -o run -- python3 bench.py $BARGS > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" --last "$STEPS" --workload "$WORKLOAD"
# the per-dispatch CSVs are large (the box returns at most 64 MiB of gpurun_out/): keep the stats and
# the summaries made from them
find "$OUT" \( -name '*kernel_trace.csv' -o -name '*counter_collection.csv' -o -name '*agent_info.csv' \) -delete
