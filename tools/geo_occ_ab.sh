#!/bin/bash
# Frame rate with k_geometry's VGPR budget capped (S3R_GEO_OCC variants go1 go6 go8 from
# tools/variants.py build): 4K P_over / P_id with the longest-first order at its threshold and
# forced on, and 8K P_over.
set -o pipefail
for a in "" "--pose P_id" "--width 7680 --height 4320 --steps 100"; do for v in go1 go6 go8; do for m in 8000 0; do
[ -n "$a" ] && [ "${a#--width}" != "$a" ] && [ $m = 0 ] && continue
S3R_LIB=build/librender_$v.so S3R_LPT_MIN=$m timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/ab.log 2>&1 || exit 1
echo "[$a] $v lpt_min=$m $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fragment_kernel_ms'])")"
done; done; done
