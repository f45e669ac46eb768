set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tiles.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bins or fused or 100k" > gpurun_out/r04_tiles6.log 2>&1
rc=$?; tail -3 gpurun_out/r04_tiles6.log; [ $rc -eq 0 ] || exit $rc
PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh "list||" "bins||S3R_TILE_BINS=1" || exit 1
for spec in "list|" "bins|S3R_TILE_BINS=1"; do
  IFS='|' read -r tag envs <<< "$spec"
  env $envs timeout -k 10 300 python3 bench.py --scene icosa-stress --pose P_id --steps 50 --warmup 5 --no-cpu-baseline --data /tmp/s3r_stress.bin > gpurun_out/r04_bs_$tag.log 2>&1 || { tail -3 gpurun_out/r04_bs_$tag.log; exit 1; }
  grep '^{' gpurun_out/r04_bs_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stress bench $tag', d['value'], d['median_ms'], 'device_fps', d['device_fps'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stress_dtrace -o run -- python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 40 --warmup 5 --delivery direct --data /tmp/s3r_stress.bin > gpurun_out/stress_dtrace.log 2>&1 || { tail -3 gpurun_out/stress_dtrace.log; exit 1; }
tail -c 600 gpurun_out/stress_dtrace.log
