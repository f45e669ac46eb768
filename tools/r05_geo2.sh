# k_geometry per-workgroup timeline (timing build): serialised and pipelined 4K P_over device frames
set -o pipefail
mkdir -p gpurun_out/geo2
S3R_SERIAL=1 timeout -k 10 180 python3 tools/geo_timeline.py > gpurun_out/geo2/serial.txt 2>&1 || { cat gpurun_out/geo2/serial.txt; exit 1; }
timeout -k 10 180 python3 tools/geo_timeline.py > gpurun_out/geo2/pipelined.txt 2>&1 || exit 1
cat gpurun_out/geo2/serial.txt gpurun_out/geo2/pipelined.txt
