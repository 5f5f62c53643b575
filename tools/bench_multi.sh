# multi-rank rehearsal of the bench contract on this box's GPU(s): usage bash tools/bench_multi.sh <N> <workload>
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus $1 --steps 3 --warmup 1 --workload ${2:-c3} --no-cpu --no-parity
