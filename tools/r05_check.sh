#!/bin/bash
# Round 5: the GPU suite once with every library launch checked (S3R_CHECK=1), then the RCCL experiment:
# the in-process RCCL gather (round 4's form) followed by the multi-device and tile suites, checked.
set -o pipefail
OUT=gpurun_out/r05
mkdir -p "$OUT"; export TMPDIR=/tmp
S3R_CHECK=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/gputest_check.log" 2>&1 || { tail -40 "$OUT/gputest_check.log"; exit 1; }
tail -3 "$OUT/gputest_check.log"
S3R_CHECK=1 S3R_TEST_RCCL_INPROCESS=1 timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 \
    --timeout-method thread tests/test_multi.py::test_nccl_gather_in_process tests/test_multi_device.py tests/test_tiles.py \
    > "$OUT/rccl_experiment.log" 2>&1 || { tail -40 "$OUT/rccl_experiment.log"; exit 1; }
tail -3 "$OUT/rccl_experiment.log"
