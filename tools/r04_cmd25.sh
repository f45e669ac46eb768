# stress: raster stage size (S3R_TSTAGE 64 / 128 default / 256 builds) and whole-frame setup grid (256 vs 1024
# workgroups per shard): whole frame and part 0 of 8 (band 135) pipelined, then delivered whole frames
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
NS="1" bash tools/stress_lib_ab.sh "def||" "ts64|build/librender_ts64.so|" "ts256|build/librender_ts256.so|" "g256||S3R_TILE_GRID=256" "def2||" || exit 1
BAND=135 NS="8" bash tools/stress_lib_ab.sh "def||" "ts64|build/librender_ts64.so|" "ts256|build/librender_ts256.so|" "def2||" || exit 1
for spec in "def||" "ts256|build/librender_ts256.so|" "g256||S3R_TILE_GRID=256" "def||" "ts256|build/librender_ts256.so|" "g256||S3R_TILE_GRID=256"; do
  IFS='|' read -r tag lib envs <<< "$spec"
  env $envs ${lib:+S3R_LIB=$lib} timeout -k 10 200 python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 100 --warmup 10 --delivery direct --data $D > gpurun_out/r04_e2e_t.log 2>&1 || { tail -3 gpurun_out/r04_e2e_t.log; exit 1; }
  grep '^{' gpurun_out/r04_e2e_t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('delivered $tag', d['fps'], d['median_ms'])"
done
