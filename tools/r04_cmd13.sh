# part 0 of 8 (stress, bins, 2 binning steps): fused raster + resolve, setup grid per shard, 32-row bands
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
NS="8" bash tools/stress_lib_ab.sh "def||" "fused||S3R_TILE_FUSED=1" "g128||S3R_TILE_GRID=128" "g512||S3R_TILE_GRID=512" "def2||" "fused2||S3R_TILE_FUSED=1" || exit 1
BAND=32 NS="8" bash tools/stress_lib_ab.sh "band32||" || exit 1
PROF=1 PROF_NS="8" NS="8" bash tools/stress_lib_ab.sh "fusedp||S3R_TILE_FUSED=1" || exit 1
