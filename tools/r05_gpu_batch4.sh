#!/bin/bash
# Round-5 batch 4 (one gpurun call): rank-image, chain and multi-rank GPU tests after the
# ranking changes, the ranking's kernel trace, and the step-chain probe at K = 4 and 20.
set -e
export TMPDIR=/tmp
T=${1:-r05s14}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rankimage.py tests/test_gpu_chain.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_rankprof -o run -- python3 tools/time_ranking.py > gpurun_out/${T}_time_ranking.log 2>&1
timeout -k 10 500 python3 -u tools/chain_probe.py 4 20 > gpurun_out/${T}_chain_probe.log 2>&1
echo batch done
