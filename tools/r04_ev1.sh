# round-4 evidence part 1: the whole GPU suite, stress parts (N = 1, 2, 4, 8), serialised stress kernel stats
set -o pipefail
mkdir -p gpurun_out/ev_r04; export TMPDIR=/tmp
bash tools/r04_full.sh || exit 1
cp gpurun_out/r04_gputest.log gpurun_out/ev_r04/gputest.log
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
bash tools/stress_parts.sh gpurun_out/ev_r04/stress_parts.jsonl || exit 1
PROF=1 PROF_NS="1 8" NS="1" bash tools/stress_lib_ab.sh "ev||" > gpurun_out/ev_r04/stress_prof.txt 2>&1 || { tail -5 gpurun_out/ev_r04/stress_prof.txt; exit 1; }
cat gpurun_out/ev_r04/stress_prof.txt
