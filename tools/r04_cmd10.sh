# tile grid on the caller's line grid: tile + multi-device suites, stress bench, delivered frames at
# buffer offsets (malloc = 16 B past a line, 0, 16) -- each also with the shift off (S3R_TILE_LINE=0)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tiles.py tests/test_multi_device.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_tiles7.log 2>&1
rc=$?; tail -3 gpurun_out/r04_tiles7.log; [ $rc -eq 0 ] || exit $rc
D=/tmp/s3r_stress.bin
timeout -k 10 300 python3 bench.py --scene icosa-stress --pose P_id --steps 50 --warmup 5 --no-cpu-baseline --data $D > gpurun_out/r04_bs_line.log 2>&1 || { tail -3 gpurun_out/r04_bs_line.log; exit 1; }
grep '^{' gpurun_out/r04_bs_line.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stress bench', d['value'], d['median_ms'], 'device_fps', d['device_fps'])"
for spec in "malloc|" "0|" "16|" "malloc|S3R_TILE_LINE=0" "malloc|" "malloc|S3R_TILE_LINE=0"; do
  IFS='|' read -r off envs <<< "$spec"
  o=""; [ "$off" != malloc ] && o="--line-offset $off"
  env $envs timeout -k 10 200 python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 100 --warmup 10 --delivery direct --data $D $o > gpurun_out/r04_e2e_off.log 2>&1 || { tail -3 gpurun_out/r04_e2e_off.log; exit 1; }
  grep '^{' gpurun_out/r04_e2e_off.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('offset $off $envs', d['fps'], d['median_ms'], d['p10_ms'])"
done
# whole-frame setup (bins): grid per shard, vertex stage, and ablations (timing only: no returning
# atomics / no binning) -- pipelined fps and serialised kernel averages at N = 1
PROF=1 PROF_NS="1" NS="1" bash tools/stress_lib_ab.sh "g1024||" "g256||S3R_TILE_GRID=256" "g0||S3R_TILE_GRID=0" "vs||S3R_VERTEX_STAGE=1" || exit 1
