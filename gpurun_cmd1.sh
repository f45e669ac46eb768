set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tiles.py -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r03_gputest10.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/r03_gputest10.log
for vs in 0 1; do for n in 1 8; do
  S3R_VERTEX_STAGE=$vs timeout -k 10 300 python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts $n --steps 30 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('VS=$vs N=$n', round(1e6/d['wall_us']), 'fps frag', round(d['frag_us'],1))" || exit 1
done; done
for vs in 0 1; do
  S3R_VERTEX_STAGE=$vs S3R_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_vs$vs -o run --output-format csv -- python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts 8 --steps 20 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/r03_vs$vs/**/run_kernel_stats.csv', recursive=True)[0])): print('VS=$vs serial part0/8', r['Name'].split('(')[0][:40], round(float(r['AverageNs'])/1e3,1), 'us')"
done
