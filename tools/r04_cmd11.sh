# whole-frame stress setup (bins): grid per shard x vertex stage, and the no-binning ablation (timing
# only); pipelined fps + serialised kernel averages at N = 1; then delivered frames for two settings
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
PROF=1 PROF_NS="1" NS="1" bash tools/stress_lib_ab.sh "g1024||" "g0||S3R_TILE_GRID=0" "g256||S3R_TILE_GRID=256" "vs||S3R_VERTEX_STAGE=1" "vs_g0||S3R_VERTEX_STAGE=1 S3R_TILE_GRID=0" "vs_g256||S3R_VERTEX_STAGE=1 S3R_TILE_GRID=256" "abl16|build/librender_tabl16.so|" "tv8|build/librender_tv8.so|" "tv2|build/librender_tv2.so|" || exit 1
for spec in "def|" "vs_g0|S3R_VERTEX_STAGE=1 S3R_TILE_GRID=0" "def|" "vs_g0|S3R_VERTEX_STAGE=1 S3R_TILE_GRID=0" "vs|S3R_VERTEX_STAGE=1" "g0|S3R_TILE_GRID=0"; do
  IFS='|' read -r tag envs <<< "$spec"
  env $envs timeout -k 10 200 python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 100 --warmup 10 --delivery direct --data $D > gpurun_out/r04_e2e_s.log 2>&1 || { tail -3 gpurun_out/r04_e2e_s.log; exit 1; }
  grep '^{' gpurun_out/r04_e2e_s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('delivered $tag', d['fps'], d['median_ms'], d['p10_ms'])"
done
