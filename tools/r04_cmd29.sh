# XCD-aware tile order in the fused raster (S3R_TILE_XCD=1): tile + multi-device suites with it on, then
# stress whole frame and part 0 of 8 pipelined, and delivered frames, on vs off
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S3R_TILE_XCD=1 timeout -k 10 600 python -u -m pytest tests/test_tiles.py tests/test_multi_device.py -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r04_xcd_tests.log 2>&1
rc=$?; grep -n "s3r:\|passed\|failed\|Fatal" gpurun_out/r04_xcd_tests.log | head -5; [ $rc -eq 0 ] || exit $rc
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
NS="1" bash tools/stress_lib_ab.sh "off||" "xcd||S3R_TILE_XCD=1" "off2||" "xcd2||S3R_TILE_XCD=1" || exit 1
BAND=135 NS="8" bash tools/stress_lib_ab.sh "off||" "xcd||S3R_TILE_XCD=1" "off2||" "xcd2||S3R_TILE_XCD=1" || exit 1
for spec in "off|" "xcd|S3R_TILE_XCD=1" "off|" "xcd|S3R_TILE_XCD=1"; do
  IFS='|' read -r tag envs <<< "$spec"
  env $envs timeout -k 10 200 python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 100 --warmup 10 --delivery direct --data $D > gpurun_out/r04_e2e_x.log 2>&1 || { tail -3 gpurun_out/r04_e2e_x.log; exit 1; }
  grep '^{' gpurun_out/r04_e2e_x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('delivered $tag', d['fps'], d['median_ms'])"
done
