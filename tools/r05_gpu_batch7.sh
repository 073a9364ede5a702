#!/bin/bash
# Round-5 batch 7: multi-rank / RCCL / rank-image tests after the handshake and sample-sort
# changes, and the ranking's kernel trace.
set -e
export TMPDIR=/tmp
T=${1:-r05s20}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_rankimage.py tests/test_gpu_chain.py > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_rankprof -o run -- python3 tools/time_ranking.py > gpurun_out/${T}_time_ranking.log 2>&1
echo batch done
