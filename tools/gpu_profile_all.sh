#!/bin/bash
# GPU box: bench (C3, default flags), ArcFace b256 MFMA profile, bench round profile.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
bash tools/profile_arcface.sh $TAG || exit $?
bash tools/profile_round.sh $TAG || exit $?
echo done
