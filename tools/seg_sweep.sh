for mb in 2048 4000 8000; do
 for cfg in "--scene flat --width 1920 --height 1080" "--scene full --width 1920 --height 1080" ; do
  S3R_MIN_BLOCKS=$mb timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 200 $cfg > /tmp/o.log 2>&1 || exit 1
  echo "mb=$mb $cfg $(grep '^{' /tmp/o.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["fragment_kernel_ms"])')"
 done
done
for mb in 2048 8000 12000 20000; do
  S3R_MIN_BLOCKS=$mb timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 200 > /tmp/o.log 2>&1 || exit 1
  echo "mb=$mb 4K $(grep '^{' /tmp/o.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["fragment_kernel_ms"])')"
done
