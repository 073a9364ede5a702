#!/bin/bash
# rocprofv3 passes for the step-chain kernels of the bench's timed UnN_many call (run on the
# GPU box): a kernel trace with stats, then one --pmc pass per counter group (never combined),
# summarised per kernel: k_count_chain (all K steps of a chunk in one launch) and k_chain_emit.
set -e
export TMPDIR=/tmp
R=${1:-r04}
K=${2:-20}
B="python3 bench.py --steps $K --warmup 1 --settle-ms 0 --no-cpu-baseline --no-sgd"
O=gpurun_out/pmc_$R
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O.trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p1 -o run -- $B > $O.p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p2 -o run -- $B > $O.p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS --output-format csv -d $O/p3 -o run -- $B > $O.p3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU --output-format csv -d $O/p4 -o run -- $B > $O.p4.log 2>&1
python3 tools/pmc_summary.py $O/chain_count_pmc.json k_count_chain $O/p1 $O/p2 $O/p3 $O/p4 > /dev/null
python3 tools/pmc_summary.py $O/chain_emit_pmc.json k_chain_emit $O/p1 $O/p2 $O/p3 $O/p4 > /dev/null
echo done
