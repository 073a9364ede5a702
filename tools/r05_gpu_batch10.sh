#!/bin/bash
# Round-5 batch 10: the chain / multi-rank / RCCL tests with the carried images, and the step-chain
# probe (first call vs carried images) at K = 4 and 20.
set -e
export TMPDIR=/tmp
T=${1:-r05s65}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 600 python3 -u tools/chain_probe.py 4 20 > gpurun_out/${T}_chain_probe.log 2>&1
echo batch done
