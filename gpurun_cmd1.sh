set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest2.log 2>&1
echo "pytest rc=$?"
for f in 8 4 16 0; do
  S3R_FILL_THREADS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device > gpurun_out/r03_bench2_fill$f.json 2> gpurun_out/r03_bench2_fill$f.err || { echo "bench fill$f failed"; break; }
done
S3R_FILL_THREADS=8 timeout -k 10 300 python -u bench.py --devices 0,0,0,0,0,0,0,0 --no-cpu-baseline --no-device > gpurun_out/r03_bench2_dev8.json 2> gpurun_out/r03_bench2_dev8.err
echo "bench rc=$?"
tail -3 gpurun_out/r03_gputest2.log
