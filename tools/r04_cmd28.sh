# final bench lines: default workload (the driver's command) and the stress scene
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_final.log 2>&1 || { tail -5 gpurun_out/r04_bench_final.log; exit 1; }
grep '^{' gpurun_out/r04_bench_final.log > gpurun_out/r04_bench_final.json
python3 -c "import json; d=json.load(open('gpurun_out/r04_bench_final.json')); print('bench', d['value'], d['median_ms'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
timeout -k 10 300 python3 bench.py --scene icosa-stress --pose P_id --steps 50 --warmup 5 --no-cpu-baseline --data $D > gpurun_out/r04_bs_final.log 2>&1 || { tail -3 gpurun_out/r04_bs_final.log; exit 1; }
grep '^{' gpurun_out/r04_bs_final.log > gpurun_out/r04_stress_bench_final.json
python3 -c "import json; d=json.load(open('gpurun_out/r04_stress_bench_final.json')); print('stress', d['value'], d['median_ms'], d['device_fps'], d['roofline']['frac'], d['roofline']['traffic'], d['setup_ms'], d['setup_traffic'])"
