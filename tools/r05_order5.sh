# bin order diagnosis: work units (work), wall time (wall), sky bins first (wsky), and both orders with
# k_geometry's walks removed (timing only: wgeo / owgeo) -- pipelined 4K frames
set -o pipefail
mkdir -p gpurun_out/order5
for rep in 1 2; do
for spec in 'work|' 'wall|build/librender_owall.so' 'wsky|build/librender_wsky.so' 'wgeo|build/librender_wgeo.so' 'owgeo|build/librender_owgeo.so'; do
  IFS='|' read -r tag lib <<< "$spec"
  env ${lib:+S3R_LIB=$lib} timeout -k 10 120 python3 tools/overhead_probe.py --steps 2000 2>/dev/null | grep '^{' | sed "s/^/$tag /" | cut -c1-130 | tee -a gpurun_out/order5/probe.txt || exit 1
done
done
