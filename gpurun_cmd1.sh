set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in 1 2 3; do
timeout -k 10 120 python3 tools/e2e_probe.py --delivery fill 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('probe', d['median_ms'], d['p10_ms'], d['p90_ms'])" || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bench', d['median_ms'], d['p10_ms'], d['p90_ms'], d['delivery']['modes']['fill']['median_ms'])" || exit 1
done
