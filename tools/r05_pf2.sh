# two-deep setup pipeline (tile path) + work-unit bin order: tile parity tests, stress A/B against the
# previous build (build/librender_owall.so: one-deep setup, wall-time order), then the order probes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pf2
timeout -k 10 600 python -u -m pytest tests/test_tiles.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pf2/tiles.log 2>&1 || { tail -30 gpurun_out/pf2/tiles.log; exit 1; }
tail -2 gpurun_out/pf2/tiles.log
NS="1 8" PROF=1 PROF_NS="1 8" bash tools/stress_lib_ab.sh 'pf2||' 'old|build/librender_owall.so|' 'pf2b||' 'oldb|build/librender_owall.so|' 2>&1 | tee gpurun_out/pf2/stress_ab.txt || exit 1
bash tools/r05_order2.sh
