#!/bin/bash
# Round-5 measurement batch on the GPU box (one gpurun call): the device-RNG count attribution
# builds, the default bench line, its kernel trace (the traced headline figure), and a 3-rank
# gloo rehearsal of bench.py with the learning lines (uneven C4 shard split).
set -e
export TMPDIR=/tmp
T=${1:-r05s8}
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab_rng_img.sh $T
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-sgd --no-cpu-baseline > gpurun_out/${T}_bench_prof.json 2> gpurun_out/${T}_bench_prof.err
python3 tools/traced_chain.py $(ls gpurun_out/${T}_prof/*/run_kernel_trace.csv gpurun_out/${T}_prof/run_kernel_trace.csv 2>/dev/null | head -1) 20 gpurun_out/${T}_count_chain_traced.json
TW_BENCH_BACKEND=gloo timeout -k 10 900 python3 bench.py --gpus 3 --steps 20 --warmup 5 --no-c5 --n 960000 --shards 48 > gpurun_out/${T}_rehearse3.json 2> gpurun_out/${T}_rehearse3.err
echo batch done
