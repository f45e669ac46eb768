set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tiles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_tiles2.log 2>&1
rc=$?; tail -3 gpurun_out/r04_tiles2.log; [ $rc -eq 0 ] || exit $rc
PROF=1 PROF_NS="8" bash tools/stress_lib_ab.sh "new||" || exit 1
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/r04_bench_a.log 2>&1 || { tail -5 gpurun_out/r04_bench_a.log; exit 1; }
grep '^{' gpurun_out/r04_bench_a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['roofline']['frame'], d['delivery']['per_device'], d['steps_requested'])"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --devices 0,0 > gpurun_out/r04_bench_b.log 2>&1 || { tail -5 gpurun_out/r04_bench_b.log; exit 1; }
grep '^{' gpurun_out/r04_bench_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench 2 parts', d['value'], d['delivery']['per_device'], d['delivery']['fill_profile'])"
