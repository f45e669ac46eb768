# work-unit vs wall-time bin order: pipelined HIP-event times (overhead_probe) and kernel traces of the
# pipelined whole-frame 4K P_over sequence
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/order2
for spec in 'work|' 'wall|build/librender_owall.so' 'work2|' 'wall2|build/librender_owall.so'; do
  IFS='|' read -r tag lib <<< "$spec"
  env ${lib:+S3R_LIB=$lib} timeout -k 10 120 python3 tools/overhead_probe.py --steps 1000 2>/dev/null | grep '^{' | sed "s/^/$tag /" | tee -a gpurun_out/order2/probe.txt || exit 1
done
for spec in 'work|' 'wall|build/librender_owall.so'; do
  IFS='|' read -r tag lib <<< "$spec"
  S3R_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/order2/tr_$tag -o tr -- python3 tools/overhead_probe.py --steps 300 > gpurun_out/order2/tr_$tag.log 2>&1 || exit 1
  f=$(find gpurun_out/order2/tr_$tag -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_timeline.py "$f" --first 200 --count 12 > gpurun_out/order2/timeline_$tag.txt || exit 1
  rm -f "$f"
done
