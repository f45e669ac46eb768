#!/bin/bash
# What one rank of an N-GPU row-band split does per frame, measured on ONE MI355X by rendering part 0
# of N (tools/overhead_probe.py --nparts N): the bench workload (full scene, P_over) at 3840x2160
# and at 7680x4320 (BASELINE config 4), N = 1, 2, 4, 8.  Output: JSON lines in $1.
mkdir -p gpurun_out
set -o pipefail
OUT=${1:-gpurun_out/parts.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for wh in "3840 2160" "7680 4320"; do
  set -- $wh
  for n in 1 2 4 8; do
    timeout -k 10 120 python3 tools/overhead_probe.py --width $1 --height $2 --nparts $n --steps 2000 2>>gpurun_out/tools_stderr.log \
      | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d.update(width=$1, height=$2, fps=1e6/d['wall_us']); print(json.dumps(d))" >> "$OUT" || exit 1
    echo "$1x$2 N=$n done"
  done
done
