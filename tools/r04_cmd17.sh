# round-end rehearsal: smoke(), the driver's default bench, and its torchrun form with 2 ranks (parts
# on the one GPU: --devices 0,0), full scene and stress scene (library band)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.log 2>&1 || { tail -5 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench_drv.log 2>&1 || { tail -5 gpurun_out/r04_bench_drv.log; exit 1; }
grep '^{' gpurun_out/r04_bench_drv.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench N=1', d['value'], d['median_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], d['steps'], d['steps_requested'])"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --devices 0,0 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04_bench_tr2.log 2>&1 || { tail -5 gpurun_out/r04_bench_tr2.log; exit 1; }
grep '^{' gpurun_out/r04_bench_tr2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('torchrun 2 ranks (parts on one GPU)', d['value'], d['median_ms'], d['config']['band_rows'], d['delivery']['per_device'])"
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --devices 0,0 --scene icosa-stress --pose P_id --steps 20 --warmup 5 --no-cpu-baseline --data $D > gpurun_out/r04_bench_tr2s.log 2>&1 || { tail -5 gpurun_out/r04_bench_tr2s.log; exit 1; }
grep '^{' gpurun_out/r04_bench_tr2s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('torchrun 2 ranks stress', d['value'], d['median_ms'], d['config']['band_rows'], d['delivery']['per_device'])"
