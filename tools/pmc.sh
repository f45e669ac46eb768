#!/bin/bash
# Hardware-counter passes over the bench workload (one rocprofv3 --pmc pass per counter group;
# FETCH_SIZE and WRITE_SIZE each need their own pass on gfx950).  Usage (on the GPU box):
#   bash tools/pmc.sh <outdir> [bench args...]
# PMC_CMD overrides the profiled command (default: python3 bench.py <args>), e.g.
#   PMC_CMD="python3 tools/overhead_probe.py --scene icosa-stress --nparts 8 --steps 10 --data /tmp/s.bin"
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
ARGS=${@:---steps 10 --warmup 2 --no-cpu-baseline}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOTDIR=$(pwd)
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_VMEM_WR" \
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU SQ_INSTS_VSKIPPED SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_LEVEL_WAVES" \
  "FETCH_SIZE" \
  "WRITE_SIZE" \
  "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$ROOTDIR/$OUT/p$i" -o run -- ${PMC_CMD:-python3 bench.py $ARGS} > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT"
