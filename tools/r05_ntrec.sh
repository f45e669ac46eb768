#!/bin/bash
# Stress scene: the setup's record / bin stores plain vs non-temporal (variant builds), N = 1 and 8
# pipelined, then serialised rocprof kernel times at N = 1.
set -o pipefail
OUT=gpurun_out/r05; mkdir -p "$OUT"; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
echo "stress data ready"
NS="1 8" BAND=135 PROF=1 PROF_NS="1" bash tools/stress_lib_ab.sh "base||" "ntrec|build/librender_ntrec.so|" "ntall|build/librender_ntall.so|" "base2||" 2>&1 | tee "$OUT/ntrec_ab.txt"
