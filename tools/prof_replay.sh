#!/bin/bash
# rocprofv3 passes for the replay-mode incomplete count (tools/time_replay.py, the bench's
# incomplete_replay line: the image kernel, plus the int64 ranked call and the plain kernel
# timed beside it) on the GPU box: a kernel trace with stats, then one --pmc pass per
# counter group (never combined with tracing domains), summarised per kernel.
set -e
export TMPDIR=/tmp
R=${1:-r02}
P="python3 tools/time_replay.py"
O=gpurun_out/pmcrep_$R
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $P > $O.trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p1 -o run -- $P > $O.p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p2 -o run -- $P > $O.p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/p3 -o run -- $P > $O.p3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p4 -o run -- $P > $O.p4.log 2>&1
python3 tools/pmc_summary.py $O/img_pmc.json "k_count_idx_img<double, 0, int," $O/p1 $O/p2 $O/p3 $O/p4 > /dev/null
python3 tools/pmc_summary.py $O/count_pmc.json "k_count_idx_ranked<double, 0, int" $O/p1 $O/p2 $O/p3 $O/p4 > /dev/null || true
python3 tools/pmc_summary.py $O/codes_pmc.json "k_rank_codes_bucket<double, 0, false>" $O/p1 $O/p2 $O/p3 $O/p4 > /dev/null || true
echo done
