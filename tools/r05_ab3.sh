#!/bin/bash
# The table-walk fragment kernel (product build, occupancy 6 for the waterfall instance) against
# occupancy 7 (72 VGPRs; LDS cut by 9 tables / 3 state batches = at7a, or 12 tables / 2 state
# batches = at7b), and the waterfall instance for frame parts too (S3R_WATERFALL_BINS=0).  Parity of
# the row-path suites with each build, frame rates, rocprof kernel averages.
set -o pipefail
OUT=gpurun_out/r05; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in prod at7a at7b; do
  lib=build/librender_$v.so; [ $v = prod ] && lib=swift3drenderer_amd/librender.so
  S3R_LIB=$lib timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 280 --timeout-method thread \
      tests/test_gpu_parity.py tests/test_multi_device.py tests/test_multi.py > "$OUT/${v}_parity.log" 2>&1 || { tail -30 "$OUT/${v}_parity.log"; exit 1; }
  echo "$v parity:"; tail -1 "$OUT/${v}_parity.log"
done
PARTS8=1 bash tools/lib_ab.sh "prod||" "at7a|build/librender_at7a.so|" "at7b|build/librender_at7b.so|" \
   "prod_wf||S3R_WATERFALL_BINS=0" "at7a_wf|build/librender_at7a.so|S3R_WATERFALL_BINS=0" \
   "prod2||" "at7a2|build/librender_at7a.so|" "at7b2|build/librender_at7b.so|" 2>&1 | tee "$OUT/ab3.txt" || exit 1
cp swift3drenderer_amd/librender.so build/librender_prod.so
S3R_VARIANTS='{"prod": {}, "at7a": {}, "at7b": {}}' S3R_VARIANT_BENCH="--scene full --pose P_over" timeout -k 10 600 python3 tools/variants.py run 2>&1 | tee -a "$OUT/ab3.txt" || exit 1
find gpurun_out/variants \( -name '*kernel_trace.csv' -o -name '*agent_info.csv' \) -delete
