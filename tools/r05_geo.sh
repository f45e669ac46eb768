# k_geometry's exact walks in device-resident 4K frames: walker iteration counters (stats build), and the
# pipelined period with the segment starts walked by the fragment workgroups instead (S3R_ROW_STARTS_DEV)
set -o pipefail
mkdir -p gpurun_out/geo
timeout -k 10 180 python3 tools/frame_stats.py --device > gpurun_out/geo/stats_dev.txt 2>&1 || { cat gpurun_out/geo/stats_dev.txt; exit 1; }
timeout -k 10 180 python3 tools/frame_stats.py > gpurun_out/geo/stats_host.txt 2>&1 || exit 1
cat gpurun_out/geo/stats_dev.txt gpurun_out/geo/stats_host.txt
for rep in 1 2; do
for spec in 'work|' 'work_rs|S3R_ROW_STARTS_DEV=1' 'wall|S3R_LIB=build/librender_owall.so' 'wall_rs|S3R_LIB=build/librender_owall.so S3R_ROW_STARTS_DEV=1'; do
  IFS='|' read -r tag envs <<< "$spec"
  env $envs timeout -k 10 120 python3 tools/overhead_probe.py --steps 2000 2>/dev/null | grep '^{' | sed "s/^/$tag /" | cut -c1-130 | tee -a gpurun_out/geo/probe.txt || exit 1
done
done
