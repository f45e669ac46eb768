#!/bin/bash
# Frames in flight (s3r_set_overlap): part 0 of N of the 4K bench workload with 1, 2 and 3 frames in
# flight (K streams / output buffers in turn).  JSON lines in $1.  (GPU box)
set -o pipefail
OUT=${1:-gpurun_out/inflight.jsonl}
: > "$OUT"
for n in ${PARTS:-1 8}; do
  for k in ${INFLIGHT:-1 2 3 1 2}; do
    timeout -k 10 120 python3 tools/overhead_probe.py --nparts $n --inflight $k --steps 2000 ${PROBE_EXTRA} 2>/dev/null | grep '^{' \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['fps']=1e6/d['wall_us']; print(json.dumps(d)); print('N=$n inflight=$k', round(d['fps']), 'fps, frag', round(d['frag_us'],1), file=sys.stderr)" >> "$OUT" || exit 1
  done
done
