#!/bin/bash
# Fragment-stage knobs (S3R_MIN_BLOCKS: segment width; S3R_LPT_MIN: longest-first threshold) over
# frame sizes and row-band parts (part 0 of N), frames pipelined; JSON lines in $1.
mkdir -p gpurun_out
set -o pipefail
OUT=${1:-gpurun_out/knob_sweep.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for cfg in "3840 2160 1 full" "3840 2160 2 full" "1920 1080 1 flat" "7680 4320 8 full" "7680 4320 4 full"; do
  set -- $cfg
  for mb in 2000 3000 4000; do
    for lpt in 4000 0; do
      S3R_MIN_BLOCKS=$mb S3R_LPT_MIN=$lpt timeout -k 10 120 python3 tools/overhead_probe.py --width $1 --height $2 --nparts $3 --scene $4 --steps 1000 2>>gpurun_out/tools_stderr.log \
        | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d.update(width=$1, scene='$4', min_blocks=$mb, lpt_min=$lpt, fps=1e6/d['wall_us']); print(json.dumps(d))" >> "$OUT" || exit 1
    done
  done
done
