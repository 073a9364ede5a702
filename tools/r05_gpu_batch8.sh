#!/bin/bash
# Round-5 batch 8: the fused wide SGD step — its bit-identity tests, the learning GPU tests,
# and the C5 step rate with and without it (tools/time_c5.py-style probe).
set -e
export TMPDIR=/tmp
T=${1:-r05s23}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_segment.py > gpurun_out/${T}_segment_tests.log 2>&1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learning.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py > gpurun_out/${T}_learning_tests.log 2>&1
timeout -k 10 300 python3 -u tools/probe_wide_fused.py > gpurun_out/${T}_wide_fused.log 2>&1
echo batch done
