set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/par.log 2>&1 || { echo PARITY_FAIL; tail -20 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
for pose in P_over P_id P_clip; do
  timeout -k 10 120 python bench.py --pose $pose --steps 100 --warmup 10 --no-cpu-baseline --no-e2e 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pose', d['value'], 'fps frag_ms', d['fragment_kernel_ms'], 'frac', d['roofline']['frac'])" || exit 1
done
