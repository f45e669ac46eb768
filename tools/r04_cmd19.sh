# the whole GPU suite after the pending-array / split-knob / band changes
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/r04_full.sh
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
PROF=1 PROF_NS="8" NS="8" BAND=135 bash tools/stress_lib_ab.sh "b135||" || exit 1
