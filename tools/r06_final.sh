#!/bin/bash
# Round 6 final evidence (GPU box), every figure from the one library this tree ships:
#   the GPU suite (once, output uncaptured), every part of the N-way splits (configs 3, 4, 5), the
#   per-stage breakdown of the 4K and 8K eighths, the round evidence (default-workload and stress
#   profiles with PMC passes, the bench matrix, the default bench line with cpu_baseline), and
#   profiles/pmc_traffic.json's entries stamped with the library's SHA-256 (tools/pmc_traffic.py).
# Each step writes its own log under gpurun_out/r06f/; a failing step ends the call.
OUT=gpurun_out/r06f
mkdir -p "$OUT"
export TMPDIR=/tmp
D=/tmp/s3r_stress.bin
step() {   # step <name> <seconds> <command...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 3 "$OUT/$name.log"
  return $rc
}
step gputest 1000 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread || exit 1
[ -f $D ] || step stress_data 300 python3 -c "from swift3drenderer_amd import stress; stress.write_named('icosa-stress', '$D')" || exit 1
step parts 900 python3 -u tools/parts_all.py --configs 3,4,5 --out "$OUT/parts_all.jsonl" || exit 1
OUT_R06=$OUT bash tools/r06.sh eighth > "$OUT/eighth.log" 2>&1 || { tail -20 "$OUT/eighth.log"; exit 1; }
step evidence 1000 bash tools/round_evidence.sh "$OUT/ev" || exit 1
step traffic_default 60 python3 tools/pmc_traffic.py "$OUT/ev/default" --workload full/P_over/3840x2160/N1 \
    --kernel 'k_fragment<6u, true, false>' --out "$OUT/pmc_traffic.json" \
    --source 'profiles/r06_final_pmc_summary.json (tools/r06_final.sh -> tools/round_evidence.sh)' || exit 1
step traffic_stress 60 python3 tools/pmc_traffic.py "$OUT/ev/stress" --workload icosa-stress/P_id/3840x2160/N1 \
    --kernel 'k_tile_raster<128u>' --setup-kernel 'k_tile_setup<false, false>' --out "$OUT/pmc_traffic.json" \
    --source 'profiles/r06_final_stress_pmc_summary.json (tools/r06_final.sh -> tools/round_evidence.sh; device-resident pass)' || exit 1
du -sh gpurun_out
