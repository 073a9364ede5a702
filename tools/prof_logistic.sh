#!/bin/bash
# PMC passes for the one-pass logistic coefficient kernel (GPU box), one counter group a run.
set -e
export TMPDIR=/tmp
O=gpurun_out/pmc_logistic
mkdir -p $O
B="python3 tools/time_complete.py 1 logistic"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU --output-format csv -d $O/p2 -o run -- $B > $O/p2.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d $O/p3 -o run -- $B > $O/p3.log 2>&1
python3 tools/pmc_summary.py $O/logistic_pmc.json k_logistic_coef $O/p1 $O/p2 $O/p3
