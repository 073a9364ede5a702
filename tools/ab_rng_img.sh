#!/bin/bash
# VERDICT r04 item 4 on the GPU box: every attribution build of k_count_rng_img (make ab-rngimg)
# and the product — timing (tools/ab_rng_img.py) and two rocprofv3 --pmc passes each (issue and
# LDS counters; one counter group per run, never with tracing), summarised per build by
# tools/pmc_summary.py into gpurun_out/abrng_$R/<build>.json.
set -e
export TMPDIR=/tmp
R=${1:-r05}
O=gpurun_out/abrng_$R
mkdir -p $O
for V in product 1 2 3 4; do
  if [ $V = product ]; then LIB=$PWD/trade-offs-in-distributed-tuplewise-estimation-and-learning_amd/libtuplewise.so
  else LIB=$PWD/tools/variants/libtuplewise_rngimg$V.so; fi
  TW_LIB_PATH=$LIB timeout -k 10 120 python3 tools/ab_rng_img.py 20 | tee -a $O/timing.log
  TW_LIB_PATH=$LIB timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/$V/p1 -o run -- python3 tools/ab_rng_img.py 5 > $O/$V.p1.log 2>&1
  TW_LIB_PATH=$LIB timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/$V/p2 -o run -- python3 tools/ab_rng_img.py 5 > $O/$V.p2.log 2>&1
  python3 tools/pmc_summary.py $O/$V.json "k_count_rng_img" $O/$V/p1 $O/$V/p2 > /dev/null
done
echo done
