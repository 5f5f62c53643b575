#!/bin/bash
# GPU box: conv/SCRFD/face-embedder parity after a kernel change, then the C3 bench and a
# kernel-trace summary of it. Any failure stops the script.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pool_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pool_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_pool.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_pool.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_pool" -o bench -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$ROOT/gpurun_out/prof_pool.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
