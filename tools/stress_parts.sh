#!/bin/bash
# The icosahedron stress scene (BASELINE config 5, 1 M icosahedra, tile path) at 3840x2160 on one
# MI355X: part 0 of an N-way row-band split, N = 1, 2, 4, 8 (tools/overhead_probe.py), JSON lines in $1.
# Bands: the library's choice for the tile path, two per part (s3r_frame_band: ceil(2160 / 2N) rows);
# BAND=k forces k rows.
mkdir -p gpurun_out
set -o pipefail
OUT=${1:-gpurun_out/stress_parts.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for n in 1 2 4 8; do
  timeout -k 10 300 python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts $n --band ${BAND:-$(( (2160 + 2 * n - 1) / (2 * n) ))} --steps ${STEPS:-40} 2>>gpurun_out/tools_stderr.log \
    | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d.update(fps=1e6/d['wall_us']); print(json.dumps(d))" >> "$OUT" || exit 1
  echo "stress N=$n done"
done
