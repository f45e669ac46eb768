set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
g++ -O2 -mavx2 -pthread tools/micro/host_stream.cpp -o tools/micro/host_stream || exit 1
timeout -k 10 120 ./tools/micro/host_stream --mb 133 --reps 7 --threads 1,2,4,8,16,24,32,48,64 > gpurun_out/r04_host_stream.json || exit 1
cat gpurun_out/r04_host_stream.json
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -mavx2 tools/micro/stage_read.hip -o tools/micro/stage_read -lpthread || exit 1
timeout -k 10 120 ./tools/micro/stage_read > gpurun_out/r04_stage_read.txt || exit 1
cat gpurun_out/r04_stage_read.txt
timeout -k 10 600 python -u -m pytest tests/test_multi.py tests/test_multi_device.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_multi.log 2>&1
rc=$?; tail -5 gpurun_out/r04_multi.log; [ $rc -eq 0 ] || exit $rc
for spec in "pack0_t4|S3R_PACK=0 S3R_FILL_THREADS=4" "pack1_t4|S3R_PACK=1 S3R_FILL_THREADS=4" "pack1_t8|S3R_PACK=1 S3R_FILL_THREADS=8" "pack0_t4b|S3R_PACK=0 S3R_FILL_THREADS=4" "pack1_t8b|S3R_PACK=1 S3R_FILL_THREADS=8" "pack1_t12|S3R_PACK=1 S3R_FILL_THREADS=12"; do
  IFS='|' read -r tag envs <<< "$spec"
  env $envs timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-device > gpurun_out/r04_b_$tag.log 2>&1 || { tail -3 gpurun_out/r04_b_$tag.log; exit 1; }
  grep '^{' gpurun_out/r04_b_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); fp=d['delivery']['fill_profile']; print('$tag', d['value'], d['median_ms'], 'p90', d['p90_ms'], 'link', d['delivery']['link_bytes_per_frame'], 'dev_end', fp.get('dev_end_us'), 'fill_end', fp.get('fill_end_us'), 'widen_us', [t['covered_us'] for t in fp.get('threads', [])])"
done
