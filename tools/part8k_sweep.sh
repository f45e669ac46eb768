#!/bin/bash
# 7680x4320 part 0 of N (N = 4, 8) on one GPU: the fragment stage's segment width and workgroup order
# knobs (S3R_MIN_BLOCKS, S3R_SEG3, S3R_LPT_MIN) -- tools/overhead_probe.py, JSON lines in $1.
mkdir -p gpurun_out
set -o pipefail
OUT=${1:-gpurun_out/part8k_sweep.jsonl}
: > "$OUT"
for n in 8 4; do
  for spec in "default|" "mb4000|S3R_MIN_BLOCKS=4000" "mb3000_seg3|S3R_MIN_BLOCKS=3000 S3R_SEG3=1" "mb8000|S3R_MIN_BLOCKS=8000" "lpt0|S3R_LPT_MIN=0" "mb4000_lpt0|S3R_MIN_BLOCKS=4000 S3R_LPT_MIN=0" "mb4000_lptoff|S3R_MIN_BLOCKS=4000 S3R_LPT_MIN=1000000"; do
    IFS='|' read -r tag envs <<< "$spec"
    env $envs timeout -k 10 120 python3 tools/overhead_probe.py --width 7680 --height 4320 --nparts $n --steps 1500 2>>gpurun_out/tools_stderr.log \
      | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d.update(tag='$tag', fps=1e6/d['wall_us']); print(json.dumps(d)); print('$tag N=$n', round(d['fps']), round(d['frag_us'],1), file=sys.stderr)" >> "$OUT" || exit 1
  done
done
