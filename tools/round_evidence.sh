#!/bin/bash
# Round evidence on the GPU box: default-workload profile (trace + PMC passes), stress-scene
# profile (trace + FETCH/WRITE passes), bench matrix, and the default bench line with cpu_baseline.
# Usage: bash tools/round_evidence.sh gpurun_out/ev_rNN
set -o pipefail
OUT=${1:-gpurun_out/ev}
mkdir -p "$OUT"
STEPS=20 bash tools/profile_round.sh "$OUT/default" > "$OUT/default.log" 2>&1 || { tail -20 "$OUT/default.log"; exit 1; }
echo "default profile done"
STEPS=10 BENCH_EXTRA="--scene icosa-stress --pose P_id" WORKLOAD="icosa-stress/P_id/3840x2160/N1" \
  bash tools/profile_round.sh "$OUT/stress" > "$OUT/stress.log" 2>&1 || { tail -20 "$OUT/stress.log"; exit 1; }
echo "stress profile done"
bash tools/bench_matrix.sh "$OUT/matrix.jsonl" > "$OUT/matrix.log" 2>&1 || { tail -20 "$OUT/matrix.log"; exit 1; }
echo "matrix done"
timeout -k 10 400 python3 bench.py > "$OUT/bench_default.log" 2>&1 || { tail -20 "$OUT/bench_default.log"; exit 1; }
grep '^{' "$OUT/bench_default.log" | tail -1 > "$OUT/bench.json"
echo "bench done"
