set -o pipefail
for a in "" "--pose P_id"; do for v in g128 g64 g32; do for m in 999999999 0; do
S3R_LIB=build/librender_$v.so S3R_LPT_MIN=$m timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/ab.log 2>&1 || exit 1
echo "[$a] $v lpt_min=$m $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fragment_kernel_ms'], d['device_frame_ms'])")"
done; done; done
