# final build: the whole GPU suite (uncaptured) and smoke()
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r04_gputest_final.log 2>&1
rc=$?; grep -n "s3r:\|passed\|failed\|Fatal" gpurun_out/r04_gputest_final.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
