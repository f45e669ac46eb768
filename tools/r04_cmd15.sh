# stress part 0 of N for interleaved band heights (rows per band): 16 (default), 27, 54, 90, 135, 270
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
for b in 16 27 54 90 135 270 16; do
  BAND=$b NS="8" bash tools/stress_lib_ab.sh "band$b||" || exit 1
done
for b in 16 54 135; do
  BAND=$b NS="2 4" bash tools/stress_lib_ab.sh "band$b||" || exit 1
done
