#!/bin/bash
# Repeat of the deciding k_geometry VGPR-cap cases (variants from tools/variants.py build, names in
# $GEO_VARIANTS, default "go5 go6 go7"): 4K P_over and P_id, longest-first at its default threshold.
set -o pipefail
for r in 1 2; do for a in "" "--pose P_id"; do for v in ${GEO_VARIANTS:-go5 go6 go7}; do
S3R_LIB=build/librender_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/ab.log 2>&1 || exit 1
echo "[$a] $v $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fragment_kernel_ms'])")"
done; done; done
