# delivered fused rasters stage 256 triangles: the whole GPU suite, then delivered stress A/B against a
# 128-stage build (build/librender_tsl128.so) and the stress bench line
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r04_gputest_t.log 2>&1
rc=$?; grep -n "s3r:\|passed\|failed\|Fatal" gpurun_out/r04_gputest_t.log | head -10; [ $rc -eq 0 ] || exit $rc
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
for spec in "new||" "old|build/librender_tsl128.so|" "new||" "old|build/librender_tsl128.so|"; do
  IFS='|' read -r tag lib envs <<< "$spec"
  env $envs ${lib:+S3R_LIB=$lib} timeout -k 10 200 python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 100 --warmup 10 --delivery direct --data $D > gpurun_out/r04_e2e_t.log 2>&1 || { tail -3 gpurun_out/r04_e2e_t.log; exit 1; }
  grep '^{' gpurun_out/r04_e2e_t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('delivered $tag', d['fps'], d['median_ms'])"
done
timeout -k 10 300 python3 bench.py --scene icosa-stress --pose P_id --steps 50 --warmup 5 --no-cpu-baseline --data $D > gpurun_out/r04_bs_final.log 2>&1 || { tail -3 gpurun_out/r04_bs_final.log; exit 1; }
grep '^{' gpurun_out/r04_bs_final.log | tee gpurun_out/r04_stress_bench_final.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stress bench', d['value'], d['median_ms'], 'device_fps', d['device_fps'], 'frame', d['roofline']['frame']['frac_device'], d['roofline']['frame']['frac_delivered'])"
