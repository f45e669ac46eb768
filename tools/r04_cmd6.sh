set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tiles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_tiles5.log 2>&1
rc=$?; tail -3 gpurun_out/r04_tiles5.log; [ $rc -eq 0 ] || exit $rc
PROF=1 PROF_NS="8" bash tools/stress_lib_ab.sh "new||" "fused||S3R_TILE_FUSED=1"
