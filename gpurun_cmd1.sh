set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest11.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/r03_gputest11.log
timeout -k 10 120 python3 tools/e2e_probe.py --delivery fill 2>/dev/null | cut -c1-200
