#!/bin/bash
# Stress scene, part 0 of N (N = 1 and 8) at 4K, for several variant builds on one box
# (build/librender_<tag>.so from tools/variants.py build).  Usage: bash tools/stress_ab.sh tag...
mkdir -p gpurun_out
set -o pipefail
for tag in "$@"; do
  for n in 1 8; do
    S3R_LIB=build/librender_$tag.so timeout -k 10 300 python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts $n --steps 30 2>>gpurun_out/tools_stderr.log \
      | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'N=$n', round(1e6/d['wall_us']), 'fps  frag', round(d['frag_us'],1), 'frame', round(d['frame_us'],1))" || exit 1
  done
done
