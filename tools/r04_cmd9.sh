# bins by default: the whole GPU suite, then the stress bench line (delivered + device-resident),
# then delivered stress frames into buffers at 16 B (malloc) / 0 B past a 64-B line
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/r04_full.sh || exit 1
D=/tmp/s3r_stress.bin
timeout -k 10 300 python3 bench.py --scene icosa-stress --pose P_id --steps 50 --warmup 5 --no-cpu-baseline --data $D > gpurun_out/r04_bs_default.log 2>&1 || { tail -3 gpurun_out/r04_bs_default.log; exit 1; }
grep '^{' gpurun_out/r04_bs_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stress bench', d['value'], d['median_ms'], 'device_fps', d['device_fps'])"
for off in malloc 0 16 malloc 0; do
  o=""; [ "$off" != malloc ] && o="--line-offset $off"
  timeout -k 10 200 python3 tools/e2e_probe.py --scene icosa-stress --pose P_id --frames 100 --warmup 10 --delivery direct --data $D $o > gpurun_out/r04_e2e_off.log 2>&1 || { tail -3 gpurun_out/r04_e2e_off.log; exit 1; }
  grep '^{' gpurun_out/r04_e2e_off.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('offset $off', d['fps'], d['median_ms'], d['p10_ms'])"
done
