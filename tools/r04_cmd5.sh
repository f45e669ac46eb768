set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tiles.py tests/test_multi_device.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_tiles4.log 2>&1
rc=$?; tail -3 gpurun_out/r04_tiles4.log; exit $rc
