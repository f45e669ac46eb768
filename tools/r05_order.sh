# longest-first bin order: work-unit costs (default) vs measured wall time (S3R_ORDER_WALL build):
# fps / device fps / HIP-event fragment time at 4K P_over, 8K, P_id; part 0 of 8; per-workgroup timeline
set -o pipefail
mkdir -p gpurun_out/order
W='build/librender_owall.so'
PARTS8=1 bash tools/lib_ab.sh 'work||' "wall|$W|" 'work2||' "wall2|$W|" 2>&1 | tee gpurun_out/order/ab4k.txt &&
BENCH_EXTRA='--width 7680 --height 4320' bash tools/lib_ab.sh 'work 8K||' "wall 8K|$W|" 2>&1 | tee gpurun_out/order/ab8k.txt &&
BENCH_EXTRA='--pose P_id' bash tools/lib_ab.sh 'work P_id||' "wall P_id|$W|" 2>&1 | tee gpurun_out/order/abpid.txt &&
S3R_WGT_DUMP=gpurun_out/order/n1.npy timeout -k 10 240 python -u tools/wg_timeline.py > gpurun_out/order/n1.txt 2>&1
