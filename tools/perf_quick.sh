# Quick check on the GPU box: the GPU test suite, then bench lines for three poses (frame rate,
# fragment kernel from HIP events) and the rocprof kernel averages of the default bench workload.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1 || { echo PARITY_FAIL; tail -30 gpurun_out/par.log; exit 1; }
tail -1 gpurun_out/par.log
for pose in P_over P_id P_clip; do
  timeout -k 10 120 python bench.py --pose $pose --steps 200 --warmup 20 --no-cpu-baseline $BENCH_EXTRA 2>>gpurun_out/tools_stderr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pose', d['value'], 'fps frag_ms', d['fragment_kernel_ms'], 'frac', d['roofline']['frac'])" || exit 1
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pq -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline $BENCH_EXTRA > gpurun_out/pq.log 2>&1 || exit 1
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/pq/**/run_kernel_stats.csv', recursive=True)[0])):
    print('  rocprof', r['Name'].split('(')[0][:40], round(float(r['AverageNs'])/1e3, 2), 'us x', r['Calls'])
"
