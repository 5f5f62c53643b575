set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03u
O=gpurun_out/r03u
timeout -k 10 500 python -u bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu > $O/g4.log 2>&1 &&
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > $O/g2_tdr.log 2>&1
rc=$?
tail -1 $O/g4.log | cut -c1-300; grep '"metric"' $O/g2_tdr.log | cut -c1-300
exit $rc
