#!/bin/bash
# GPU box: full -m gpu suite + smoke, then the C3 bench with the embed stream on and off.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_full.sh || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_c3.log; [ $rc -eq 0 ] || exit $rc
PERSON_CAPTURE_AMD_EMBED_STREAM=0 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c3_1stream.log 2>&1
rc=$?; echo "bench 1-stream rc=$rc"; tail -1 gpurun_out/bench_c3_1stream.log | cut -c1-300; exit $rc
