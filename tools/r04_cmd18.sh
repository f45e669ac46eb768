# delivered tile frames as sub-frames (S3R_TILE_SPLIT): tile tests, then delivered stress frames k = 1..4
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tiles.py -m gpu -x -q --timeout 300 --timeout-method thread -k "split or deliver or line_offsets" > gpurun_out/r04_tiles9.log 2>&1
rc=$?; tail -3 gpurun_out/r04_tiles9.log; [ $rc -eq 0 ] || exit $rc
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
for spec in "1|" "2|S3R_TILE_SPLIT=2" "3|S3R_TILE_SPLIT=3" "4|S3R_TILE_SPLIT=4" "1|" "2|S3R_TILE_SPLIT=2"; do
  IFS='|' read -r tag envs <<< "$spec"
  env $envs timeout -k 10 200 python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 100 --warmup 10 --delivery direct --data $D > gpurun_out/r04_e2e_split.log 2>&1 || { tail -3 gpurun_out/r04_e2e_split.log; exit 1; }
  grep '^{' gpurun_out/r04_e2e_split.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('split $tag', d['fps'], d['median_ms'], d['p10_ms'])"
done
