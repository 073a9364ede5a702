#!/bin/bash
# GPU pass used for the fused narrow SGD step (tw_sgd_step): the learning tests,
# the C4 timing and a kernel trace of it.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_learning.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fuse_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/time_sgd.py > gpurun_out/fuse_sgd.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fuse_prof -o run -- python3 tools/time_sgd.py > gpurun_out/fuse_prof.log 2>&1
