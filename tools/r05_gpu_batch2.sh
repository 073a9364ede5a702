#!/bin/bash
# Round-5 measurement batch 2 (one gpurun call): the multi-rank and RCCL tests, learning over one and two co-resident ranks at
# the C5 shape with per-kernel device times (torch.profiler), the drop-in's host timeline, the
# product device-RNG count timing, and the step-chain probe at K = 4 and K = 20.
set -e
export TMPDIR=/tmp
T=${1:-r05s12}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_rccl.py > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 python3 -u tools/probe_learn_ranks.py 1 c5 trace > gpurun_out/${T}_learn1.log 2>&1
timeout -k 10 300 python3 -u tools/probe_learn_ranks.py 2 c5 trace > gpurun_out/${T}_learn2.log 2>&1
timeout -k 10 300 python3 -u tools/time_dropin_parts.py 6 > gpurun_out/${T}_dropin.log 2>&1
timeout -k 10 120 python3 -u tools/ab_rng_img.py 20 > gpurun_out/${T}_rngimg.log 2>&1
timeout -k 10 400 python3 -u tools/chain_probe.py 4 20 > gpurun_out/${T}_chain_probe.log 2>&1
echo batch done
