set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload tag --steps 3 --warmup 1 > gpurun_out/bench_tag.log 2>&1 && tail -1 gpurun_out/bench_tag.log &&
VGE_BENCH_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload tag --steps 2 --warmup 1 > gpurun_out/bench_tag2.log 2>&1 && tail -1 gpurun_out/bench_tag2.log
