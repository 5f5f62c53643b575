#!/bin/bash
# GPU box: extract_batch pipeline tests + C3 bench line
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_face_embedder.py tests/test_gpu_bench_config.py tests/test_gpu_fallbacks.py tests/test_gpu_prescan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1
rc=$?; echo "pipe tests rc=$rc"; tail -3 gpurun_out/pipe_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_c3.log | cut -c1-420; exit $rc
