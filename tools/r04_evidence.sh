#!/bin/bash
# Round-4 evidence on the GPU box, into gpurun_out/ev_r04:
#   stress parts (part 0 of N = 1, 2, 4, 8, pipelined) + serialised kernel stats of part 0 of 8 and of
#   the whole frame (setup + binning per part), the default-workload profile (kernel trace + PMC
#   passes: k_fragment's counters), the bench matrix (configs 2-5) and the default bench line.
set -o pipefail
OUT=gpurun_out/ev_r04
mkdir -p "$OUT"; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
bash tools/stress_parts.sh "$OUT/stress_parts.jsonl" || exit 1
PROF=1 PROF_NS="1 8" NS="1" bash tools/stress_lib_ab.sh "ev||" > "$OUT/stress_prof.txt" 2>&1 || { tail -5 "$OUT/stress_prof.txt"; exit 1; }
cp -r gpurun_out/stress_ab/ev_n1 gpurun_out/stress_ab/ev_n8 "$OUT/" || exit 1
echo "stress done"
STEPS=20 bash tools/profile_round.sh "$OUT/default" > "$OUT/default.log" 2>&1 || { tail -20 "$OUT/default.log"; exit 1; }
echo "default profile done"
bash tools/bench_matrix.sh "$OUT/matrix.jsonl" > "$OUT/matrix.log" 2>&1 || { tail -20 "$OUT/matrix.log"; exit 1; }
echo "matrix done"
timeout -k 10 400 python3 bench.py > "$OUT/bench_default.log" 2>&1 || { tail -20 "$OUT/bench_default.log"; exit 1; }
grep '^{' "$OUT/bench_default.log" | tail -1 > "$OUT/bench.json"
echo "bench done"
