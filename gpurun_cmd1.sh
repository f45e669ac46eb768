set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest6.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r03_gputest6.log
for k in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03_bench6_$k.json 2> gpurun_out/r03_bench6_$k.err || { echo bench fail; exit 1; }; done
for f in 2 4 16; do S3R_FILL_THREADS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device > gpurun_out/r03_bench6_f$f.json 2>/dev/null || exit 1; done
echo done
