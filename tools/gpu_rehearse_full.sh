# 2-rank rehearsal of bench.py on one GPU with the learning lines (gloo, real HIP kernels):
# the estimation lines, C4 over the ranks and the C4 trade-off curve (C5 left out: its
# partitioned reshuffles move GBs of rows, which gloo stages through the host).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp TW_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --no-c5 > gpurun_out/${1:-r1}_rehearse2_full.json 2> gpurun_out/${1:-r1}_rehearse2_full.err
