# band by path, stage timing, binned-entry totals: the whole GPU suite, the stress bench line, the
# stress scene as 8 parts on one GPU behind updateAndRender (the library's band), part 0 of N at the library's band (two per part)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/r04_full.sh || exit 1
D=/tmp/s3r_stress.bin
[ -f $D ] || python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
timeout -k 10 300 python3 bench.py --scene icosa-stress --pose P_id --steps 50 --warmup 5 --no-cpu-baseline --data $D > gpurun_out/r04_bs_16.log 2>&1 || { tail -3 gpurun_out/r04_bs_16.log; exit 1; }
grep '^{' gpurun_out/r04_bs_16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stress bench', d['value'], d['median_ms'], 'device_fps', d['device_fps'], 'setup_ms', d['setup_ms'], 'roof', d['roofline']['frac'], d['roofline']['algorithmic_bytes_per_launch'], d['roofline']['kernel'])"
timeout -k 10 300 python3 bench.py --scene icosa-stress --pose P_id --devices 0,0,0,0,0,0,0,0 --steps 30 --warmup 5 --no-cpu-baseline --no-device --data $D > gpurun_out/r04_bs_8p.log 2>&1 || { tail -3 gpurun_out/r04_bs_8p.log; exit 1; }
grep '^{' gpurun_out/r04_bs_8p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stress 8 parts on one GPU', d['value'], d['median_ms'], 'band', d['config']['band_rows'], {k: v['fps'] for k, v in d['delivery']['modes'].items()})"
for n in 2 4 8; do BAND=$(( (2160 + 2 * n - 1) / (2 * n) )) NS="$n" bash tools/stress_lib_ab.sh "band_auto||" || exit 1; done
