#!/bin/bash
# Round-5 batch 5 (one gpurun call): the device-shuffle drop-in tests (streamed last shuffle,
# early counts), then the drop-in's host timeline at C3 size.
set -e
export TMPDIR=/tmp
T=${1:-r05s15}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_devshuffle.py > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 python3 -u tools/time_dropin_parts.py 8 > gpurun_out/${T}_dropin.log 2>&1
echo batch done
