# stress-scene profile (kernel trace + PMC passes: HBM traffic of the setup and the fused raster)
set -o pipefail
mkdir -p gpurun_out/ev_r04; export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
STEPS=10 BENCH_EXTRA="--scene icosa-stress --pose P_id --data $D" WORKLOAD="icosa-stress/P_id/3840x2160/N1" \
  bash tools/profile_round.sh gpurun_out/ev_r04/stress > gpurun_out/ev_r04/stress.log 2>&1 || { tail -20 gpurun_out/ev_r04/stress.log; exit 1; }
cat gpurun_out/ev_r04/stress/pmc_traffic.json
