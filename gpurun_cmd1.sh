set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multi_device.py tests/test_gpu_parity.py tests/test_host_loop.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest5.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/r03_gputest5.log
for k in 1 2 3; do timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03_bench5_$k.json 2> gpurun_out/r03_bench5_$k.err || { echo bench fail; exit 1; }; done
S3R_DATA_PATH=swift3drenderer_amd/data.bin timeout -k 10 120 ./host/main_loop --lib swift3drenderer_amd/librender.so --size 3840 2160 --frames 2000 > gpurun_out/r03_mainloop_4k.txt 2>&1; echo "loop rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof5 -o prof --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r03_prof5.log 2>&1
echo "prof rc=$?"
