# work-unit vs wall-time bin order: host-side sections per frame (S3R_HOSTPROF) of the pipelined 4K frames
set -o pipefail
mkdir -p gpurun_out/order3
for spec in 'work|' 'wall|build/librender_owall.so' 'work2|' 'wall2|build/librender_owall.so'; do
  IFS='|' read -r tag lib <<< "$spec"
  env ${lib:+S3R_LIB=$lib} S3R_HOSTPROF=1 timeout -k 10 120 python3 tools/overhead_probe.py --steps 2000 > gpurun_out/order3/$tag.log 2>&1 || exit 1
  echo "== $tag"; grep -E '^\{|hostprof' gpurun_out/order3/$tag.log | cut -c1-300
done
