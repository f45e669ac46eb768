#!/bin/bash
# Frame rate with 2 / 3 / 4 geometry streams (variants gs2 gs3 gs4 from tools/variants.py build),
# longest-first order at its default threshold and forced on; 4K P_over, 4K P_id, 8K P_over.
set -o pipefail
for a in "" "--pose P_id" "--width 7680 --height 4320 --steps 100"; do for v in gs2 gs3 gs4; do for m in 8000 0; do
S3R_LIB=build/librender_$v.so S3R_LPT_MIN=$m timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/ab.log 2>&1 || exit 1
echo "[$a] $v lpt_min=$m $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fragment_kernel_ms'])")"
done; done; done
