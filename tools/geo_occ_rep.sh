set -o pipefail
for r in 1 2; do for a in "" "--pose P_id"; do for vm in "go1 8000" "go6 8000" "go6 0"; do set -- $vm
S3R_LIB=build/librender_$1.so S3R_LPT_MIN=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e $a > gpurun_out/ab.log 2>&1 || exit 1
echo "[$a] $1 lpt_min=$2 $(tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fragment_kernel_ms'])")"
done; done; done
