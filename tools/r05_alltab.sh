#!/bin/bash
# k_fragment with every overlapping (triangle, component) walked by sequential adds into LDS tables
# (S3R_ALLTAB build) against the product build: parity of the row-path suites with the variant, then
# frame rates / fragment times (bench, part 0 of 8) and rocprof kernel averages on the default workload.
set -o pipefail
OUT=gpurun_out/r05; mkdir -p "$OUT"; export TMPDIR=/tmp
S3R_LIB=build/librender_alltab.so timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 280 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_multi_device.py tests/test_multi.py tests/test_host_loop.py tests/test_stream_order.py 2>&1 | tee "$OUT/alltab_parity.log" | tail -3 || exit 1
PARTS8=1 bash tools/lib_ab.sh "base||" "alltab|build/librender_alltab.so|" "base2||" "alltab2|build/librender_alltab.so|" 2>&1 | tee "$OUT/alltab_ab.txt" || exit 1
S3R_VARIANTS='{"base": {}, "alltab": {"S3R_ALLTAB": 1}}' S3R_VARIANT_BENCH="--scene full --pose P_over" timeout -k 10 600 python3 tools/variants.py run 2>&1 | tee -a "$OUT/alltab_ab.txt" || exit 1
find gpurun_out/variants \( -name '*kernel_trace.csv' -o -name '*agent_info.csv' \) -delete
