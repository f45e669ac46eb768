#!/bin/bash
# One bench.py line per BASELINE config that fits one GPU (run on the GPU box):
#   cfg2  flat scene, 1920x1080, P_over            (flat-colour path)
#   cfg3  full scene, 3840x2160, P_over and P_id   (ripmap path; the default bench workload)
#   cfg4  full scene, 7680x4320, P_over            (the 8-GPU config, here on one GPU)
#   cfg5  icosa-stress (1 M icosahedra), 3840x2160 (the 8-GPU stress config, here on one GPU)
# plus P_clip at 4K.  Output: JSON lines in $1 (default gpurun_out/matrix.jsonl).
set -o pipefail
OUT=${1:-gpurun_out/matrix.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
run() {
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > /tmp/bm.log 2>&1 || { tail -5 /tmp/bm.log; exit 1; }
  grep '^{' /tmp/bm.log | tail -1 >> "$OUT"
  echo "$*: done"
}
run --scene flat --pose P_over --width 1920 --height 1080
run --scene full --pose P_over
run --scene full --pose P_id
run --scene full --pose P_clip
run --scene full --pose P_over --width 7680 --height 4320
run --scene icosa-stress --pose P_id --steps 50 --warmup 5 --data /tmp/s3r_stress.bin
