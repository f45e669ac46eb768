# the whole GPU suite after the pending-array / split-knob / band changes
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/r04_full.sh
