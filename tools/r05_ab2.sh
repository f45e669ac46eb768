#!/bin/bash
# k_fragment variants against the product build: S3R_ALLTAB (sequential-add tables for every chunk,
# unroll 4: no spills) and S3R_SEG_STATES (per-segment start states from k_geometry).  Parity of the
# row-path suites with each, frame rates (bench, part 0 of 8), rocprof kernel averages, SQ counters.
set -o pipefail
OUT=gpurun_out/r05; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in alltab segst; do
  S3R_LIB=build/librender_$v.so timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 280 --timeout-method thread \
      tests/test_gpu_parity.py tests/test_multi_device.py tests/test_multi.py tests/test_stream_order.py > "$OUT/${v}_parity.log" 2>&1 || { tail -30 "$OUT/${v}_parity.log"; exit 1; }
  echo "$v parity:"; tail -1 "$OUT/${v}_parity.log"
done
PARTS8=1 bash tools/lib_ab.sh "base||" "alltab|build/librender_alltab.so|" "segst|build/librender_segst.so|" "base2||" "alltab2|build/librender_alltab.so|" "segst2|build/librender_segst.so|" 2>&1 | tee "$OUT/ab2.txt" || exit 1
S3R_VARIANTS='{"base": {}, "alltab": {"S3R_ALLTAB": 1}, "segst": {"S3R_SEG_STATES": 1}}' S3R_VARIANT_BENCH="--scene full --pose P_over" timeout -k 10 600 python3 tools/variants.py run 2>&1 | tee -a "$OUT/ab2.txt" || exit 1
find gpurun_out/variants \( -name '*kernel_trace.csv' -o -name '*agent_info.csv' \) -delete
bash tools/variant_pmc.sh gpurun_out/r05/vpmc2 base alltab segst 2>&1 | tee "$OUT/ab2_pmc.txt" || exit 1
