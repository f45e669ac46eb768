#!/bin/bash
# Table-walk tuning: conservative pruning before the fill (S3R_TW=8; 9 = also no scheduling barrier)
# against the product build: parity of the row-path suites, rocprof kernel averages, frame rates.
set -o pipefail
OUT=gpurun_out/r05; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in tw8 tw9; do
  S3R_LIB=build/librender_$v.so timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 280 --timeout-method thread \
      tests/test_gpu_parity.py tests/test_multi_device.py tests/test_multi.py > "$OUT/${v}_parity.log" 2>&1 || { tail -30 "$OUT/${v}_parity.log"; exit 1; }
  echo "$v parity:"; tail -1 "$OUT/${v}_parity.log"
done
cp swift3drenderer_amd/librender.so build/librender_prod.so
S3R_VARIANTS='{"prod": {}, "tw8": {}, "tw9": {}, "prod2": {}, "tw8b": {}}' S3R_VARIANT_BENCH="--scene full --pose P_over" timeout -k 10 900 python3 tools/variants.py run 2>&1 | tee "$OUT/tw_ab2.txt" || exit 1
PARTS8=1 bash tools/lib_ab.sh "prod||" "tw8|build/librender_tw8.so|" "prod2||" "tw8b|build/librender_tw8.so|" 2>&1 | tee -a "$OUT/tw_ab2.txt" || exit 1
find gpurun_out/variants \( -name '*kernel_trace.csv' -o -name '*agent_info.csv' \) -delete
