# k_fragment segment width at 4K (6 / 3 / 2 / 1 chunks per workgroup): fps, device fps, HIP-event fragment time
set -o pipefail
mkdir -p gpurun_out/seg
PARTS8=1 bash tools/lib_ab.sh 'base||' 'seg3||S3R_SEG3=1 S3R_MIN_BLOCKS=6000' 'seg2||S3R_MIN_BLOCKS=8000' 'seg1||S3R_MIN_BLOCKS=20000' 'base2||' 2>&1 | tee gpurun_out/seg/ab.txt
