set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest9.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/r03_gputest9.log
for d in 0 0,0 0,0,0,0 0,0,0,0,0,0,0,0; do timeout -k 10 120 python3 tools/e2e_probe.py --delivery fill --devices $d 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$d', d['fps'], d['median_ms'], d['p90_ms'], 'gpu8ths', d['fill_gpu_eighths'], 'link', d['link_bytes'], 'thr', d['fill_threads'])" || exit 1; done
for d in 0,0 0,0,0,0; do timeout -k 10 120 python3 tools/e2e_probe.py --delivery direct --devices $d 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('direct $d', d['fps'], d['median_ms'])" || exit 1; done
