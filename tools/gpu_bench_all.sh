#!/bin/bash
# GPU box: the three bench workloads + ArcFace b256 probe + per-layer ArcFace profile.
# Any abort/fault/timeout stops the script.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
run bench_c3 400 python -u bench.py --steps 5 --warmup 2
run bench_c4 400 python -u bench.py --workload c4 --batch 16 --steps 3 --warmup 1
run bench_c5 300 python -u bench.py --workload c5 --steps 5 --warmup 2
#run arc 200 python -u tools/probe_arcface.py 256
#run layers_arc 200 python -u tools/probe_layers.py arc 256
