#!/bin/bash
# The round's evidence on the GPU box, in one call: the -m gpu suite, smoke(), the default bench
# line, a rocprofv3 kernel trace + stats of the bench's headline (no SGD lines) with the traced
# k_count_chain figure, and the paper's estimation experiment.  Every GPU step has its own time
# limit; the first failure ends the script (set -e).  Outputs: gpurun_out/<R>_*.
#     bash tools/evidence.sh r06s10
set -e
export TMPDIR=/tmp
R=${1:?round tag}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/${R}_gpu_tests.log 2>&1
tail -2 $O/${R}_gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1
tail -1 $O/${R}_smoke.log
timeout -k 10 400 python -u bench.py > $O/${R}_bench.json 2> $O/${R}_bench.err
tail -c 600 $O/${R}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_trace -o run \
  -- python3 bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-sgd > $O/${R}_trace.log 2>&1
T=$(find $O/${R}_trace -name run_kernel_trace.csv | sort | head -n 1)
S=$(find $O/${R}_trace -name run_kernel_stats.csv | sort | head -n 1)
cp "$S" $O/${R}_bench_nosgd_kernel_stats.csv
python3 tools/traced_chain.py "$T" 20 $O/${R}_count_chain_traced.json
cat $O/${R}_count_chain_traced.json
timeout -k 10 300 python -u tools/estimation_experiment.py --cpu-tries 200 \
  > $O/${R}_estimation_experiment.log 2>&1
cat $O/${R}_estimation_experiment.log
echo evidence-done
