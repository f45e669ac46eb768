# tile_visit steps in flight (1 / 2 / 4) x vertex stage, stress N = 1 and part 0 of 8, then delivered
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
PROF=1 PROF_NS="1 8" NS="1 8" bash tools/stress_lib_ab.sh "tv4||" "tv2|build/librender_tv2.so|" "tv1|build/librender_tv1.so|" "tv2vs|build/librender_tv2.so|S3R_VERTEX_STAGE=1" "tv4b||" || exit 1
for spec in "tv4||" "tv2|build/librender_tv2.so|" "tv1|build/librender_tv1.so|" "tv4||" "tv2|build/librender_tv2.so|" "tv1|build/librender_tv1.so|"; do
  IFS='|' read -r tag lib envs <<< "$spec"
  env $envs ${lib:+S3R_LIB=$lib} timeout -k 10 200 python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 100 --warmup 10 --delivery direct --data $D > gpurun_out/r04_e2e_s.log 2>&1 || { tail -3 gpurun_out/r04_e2e_s.log; exit 1; }
  grep '^{' gpurun_out/r04_e2e_s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('delivered $tag', d['fps'], d['median_ms'], d['p10_ms'])"
done
