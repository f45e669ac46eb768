set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest1.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python -u bench.py > gpurun_out/r03_bench1.json 2> gpurun_out/r03_bench1.err && \
timeout -k 10 300 python -u bench.py --devices 0,0,0,0,0,0,0,0 --no-cpu-baseline > gpurun_out/r03_bench1_dev8.json 2> gpurun_out/r03_bench1_dev8.err
echo "bench rc=$?"
tail -3 gpurun_out/r03_gputest1.log
