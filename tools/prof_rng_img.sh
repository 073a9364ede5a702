#!/bin/bash
# rocprofv3 --pmc passes for the device-RNG image count k_count_rng_img (bench `incomplete`,
# DESIGN.md §4.2 issue model) driven by tools/tune_rng_img.py at the default unroll (GPU box):
# one counter group per run, never combined with tracing domains, summarised per kernel.
set -e
export TMPDIR=/tmp
R=${1:-r03}
P="python3 tools/tune_rng_img.py 2"
O=gpurun_out/pmcrng_$R
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/p3 -o run -- $P > $O.p3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p4 -o run -- $P > $O.p4.log 2>&1
python3 tools/pmc_summary.py $O/rng_img_pmc.json "k_count_rng_img<double, 0, 2>" $O/p3 $O/p4 > /dev/null
echo done
