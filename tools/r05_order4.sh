# bin order (work units / wall time) x geometry stream priority (highest / default): pipelined 4K frames
set -o pipefail
mkdir -p gpurun_out/order4
for rep in 1 2; do
for spec in 'work|' 'wall|build/librender_owall.so' 'work_p0|' 'wall_p0|build/librender_owall.so'; do
  IFS='|' read -r tag lib <<< "$spec"
  pe=''; case $tag in *_p0) pe='S3R_GEO_PRIO=0';; esac
  env $pe ${lib:+S3R_LIB=$lib} timeout -k 10 120 python3 tools/overhead_probe.py --steps 2000 2>/dev/null | grep '^{' | sed "s/^/$tag /" | cut -c1-200 | tee -a gpurun_out/order4/probe.txt || exit 1
done
done
