# bins-mode parity + list-vs-bins A/B (stress, N = 1 / 8, delivered) + delivered-frame trace +
# contiguous-halves parts on one GPU (delivered stress frame)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/r04_cmd7.sh || exit 1
D=/tmp/s3r_stress.bin
for spec in "halves|0,0|1080|" "halves_fused|0,0|1080|S3R_TILE_FUSED=1" "quarters_fused|0,0,0,0|540|S3R_TILE_FUSED=1" "bands16_fused|0,0|16|S3R_TILE_FUSED=1"; do
  IFS='|' read -r tag devs band envs <<< "$spec"
  env $envs timeout -k 10 300 python3 bench.py --scene icosa-stress --pose P_id --devices $devs --band $band --steps 50 --warmup 5 --no-cpu-baseline --no-device --data $D > gpurun_out/r04_bp_$tag.log 2>&1 || { tail -3 gpurun_out/r04_bp_$tag.log; exit 1; }
  grep '^{' gpurun_out/r04_bp_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('parts $tag', d['value'], d['median_ms'], {k: v['fps'] for k, v in d['delivery']['modes'].items()})"
done
