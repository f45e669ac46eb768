#!/bin/bash
# Part 0 of an 8-way split at 4K (the one-rank share of the N = 8 bench) under the fragment-stage
# knobs: segment width (S3R_MIN_BLOCKS picks the widest segment still launching that many
# workgroups) and the longest-first order threshold (S3R_LPT_MIN).  JSON lines in $1.
mkdir -p gpurun_out
set -o pipefail
OUT=${1:-gpurun_out/part_knobs.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for mb in 2000 1000 4000; do
  for lpt in 4000 0; do
    S3R_MIN_BLOCKS=$mb S3R_LPT_MIN=$lpt timeout -k 10 120 python3 tools/overhead_probe.py --nparts ${NPARTS:-8} --steps 2000 2>>gpurun_out/tools_stderr.log \
      | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d.update(min_blocks=$mb, lpt_min=$lpt, fps=1e6/d['wall_us']); print(json.dumps(d))" >> "$OUT" || exit 1
  done
done
