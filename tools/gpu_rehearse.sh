# 2-rank rehearsal of the multi-GPU bench path on one GPU (gloo, real HIP kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp TW_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-sgd > gpurun_out/${1:-r1}_rehearse2.json 2> gpurun_out/${1:-r1}_rehearse2.err
