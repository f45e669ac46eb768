set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest_s3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03_gputest_s3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench_s3.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r03_bench_s3.log | cut -c1-400
exit $rc
