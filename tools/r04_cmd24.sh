# the whole GPU suite three times, uncaptured, then smoke() and the default bench (round-end rehearsal)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1 2 3; do
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r04_gputest_r$k.log 2>&1
  rc=$?; grep -n "s3r:\|passed\|failed\|Fatal" gpurun_out/r04_gputest_r$k.log | head -10; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_end.log 2>&1 || { tail -5 gpurun_out/r04_bench_end.log; exit 1; }
grep '^{' gpurun_out/r04_bench_end.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['median_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
