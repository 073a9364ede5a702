#!/bin/bash
# Round-5 batch 6 (one gpurun call): the whole GPU test suite, smoke(), the default bench line,
# and its kernel trace (the traced headline figure, tools/traced_chain.py).
set -e
export TMPDIR=/tmp
T=${1:-r05s19}
mkdir -p gpurun_out
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-sgd --no-cpu-baseline > gpurun_out/${T}_bench_prof.json 2> gpurun_out/${T}_bench_prof.err
python3 tools/traced_chain.py $(ls gpurun_out/${T}_prof/*/run_kernel_trace.csv gpurun_out/${T}_prof/run_kernel_trace.csv 2>/dev/null | head -1) 20 gpurun_out/${T}_count_chain_traced.json
echo batch done
