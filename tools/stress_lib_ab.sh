#!/bin/bash
# Stress scene (config 5, 1 M icosahedra) at 4K on one GPU: part 0 of N = 1 and 8 for several
# library builds / settings, then a rocprof kernel summary of part 0 of 8 per spec.
# Usage: bash tools/stress_lib_ab.sh 'tag|lib|ENV=..' ...  (lib '' = the product library; GPU box)
mkdir -p gpurun_out
set -o pipefail
mkdir -p gpurun_out/stress_ab
export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r tag lib envs <<< "$spec"
  for n in ${NS:-1 8}; do
    env $envs ${lib:+S3R_LIB=$lib} timeout -k 10 300 python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts $n --band ${BAND:-16} --steps ${STEPS:-30} 2>>gpurun_out/tools_stderr.log \
      | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag N=$n', round(1e6/d['wall_us']), 'fps  frag', round(d['frag_us'],1), 'frame', round(d['frame_us'],1))" || exit 1
  done
done
if [ -n "$PROF" ]; then
  for spec in "$@"; do
    IFS='|' read -r tag lib envs <<< "$spec"
    for n in ${PROF_NS:-8}; do
      d=gpurun_out/stress_ab/${tag}_n$n
      env $envs ${lib:+S3R_LIB=$lib} S3R_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/overhead_probe.py --scene icosa-stress --pose P_id --data /tmp/s3r_stress.bin --nparts $n --steps 20 >> gpurun_out/tools_output.log 2>&1 || exit 1
      f=$(find $d -name '*kernel_stats.csv' | head -1)
      echo "== $tag N=$n (serialised)"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:12]: print('  %-60s %8s calls  avg %9.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
    done
  done
fi
