#!/bin/bash
# Round-5 batch 3 (one gpurun call): the chain and multi-rank GPU tests (the lead step of the
# step chains), then the step-chain probe at K = 4 and K = 20 with and without the lead step.
set -e
export TMPDIR=/tmp
T=${1:-r05s13}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 500 python3 -u tools/chain_probe.py 4 20 > gpurun_out/${T}_chain_probe.log 2>&1
echo batch done
