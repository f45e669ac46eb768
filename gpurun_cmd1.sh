set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tiles.py tests/test_multi_device.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest7.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r03_gputest7.log
timeout -k 10 600 bash tools/stress_ab.sh skip noskip > gpurun_out/r03_stress_ab.txt 2>&1; echo "ab rc=$?"; cat gpurun_out/r03_stress_ab.txt
for tag in skip noskip; do
  for c in FETCH_SIZE WRITE_SIZE; do
    S3R_LIB=build/librender_$tag.so timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r03_spmc_${tag}_$c -o run -- python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts 1 --steps 5 > gpurun_out/r03_spmc_${tag}_$c.log 2>&1 || { echo "pmc $tag $c failed"; exit 1; }
  done
done
echo pmc done
