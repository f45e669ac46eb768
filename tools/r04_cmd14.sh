# fused raster for every frame: tile + multi-device + multi suites, then part 0 of 8 A/B (grid per shard)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tiles.py tests/test_multi_device.py tests/test_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_tiles8.log 2>&1
rc=$?; tail -3 gpurun_out/r04_tiles8.log; [ $rc -eq 0 ] || exit $rc
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
NS="8" bash tools/stress_lib_ab.sh "def||" "g128||S3R_TILE_GRID=128" "g192||S3R_TILE_GRID=192" "def2||" "g128b||S3R_TILE_GRID=128" || exit 1
NS="1" bash tools/stress_lib_ab.sh "def||" "g128||S3R_TILE_GRID=128" || exit 1
