#!/bin/bash
# Round 4: tile-path cluster cull -- the tile tests, then the stress scene (config 5) at 4K, part 0 of
# N = 1 and 8, with the cull (default) and without (S3R_CLUSTERS=0).  GPU box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_tiles.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_tiles.log 2>&1
rc=$?; tail -4 gpurun_out/r04_tiles.log; [ $rc -eq 0 ] || exit $rc
for cl in 1 0; do
  for n in 1 8; do
    S3R_CLUSTERS=$cl timeout -k 10 300 python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts $n --steps ${STEPS:-30} 2>/dev/null \
      | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('clusters=$cl N=$n', round(1e6/d['wall_us']), 'fps', json.dumps(d))" | tee -a gpurun_out/r04_cluster_ab.txt || exit 1
  done
done
