# round-4 evidence part 2: stress parts again (fused parts), default-workload profile (kernel trace + PMC
# passes), the bench matrix (configs 2-5) and the default bench line
set -o pipefail
OUT=gpurun_out/ev_r04
mkdir -p $OUT; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
bash tools/stress_parts.sh $OUT/stress_parts2.jsonl || exit 1
PROF=1 PROF_NS="1 8" NS="1" bash tools/stress_lib_ab.sh "ev2||" > $OUT/stress_prof2.txt 2>&1 || { tail -5 $OUT/stress_prof2.txt; exit 1; }
cat $OUT/stress_prof2.txt
STEPS=20 bash tools/profile_round.sh $OUT/default > $OUT/default.log 2>&1 || { tail -20 $OUT/default.log; exit 1; }
echo "default profile done"
bash tools/bench_matrix.sh $OUT/matrix.jsonl > $OUT/matrix.log 2>&1 || { tail -20 $OUT/matrix.log; exit 1; }
echo "matrix done"
timeout -k 10 400 python3 bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
grep '^{' $OUT/bench_default.log | tail -1 > $OUT/bench.json
echo "bench done"
