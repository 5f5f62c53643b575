set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03dd
O=gpurun_out/r03dd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_small_plans.py tests/test_gpu_face_embedder.py tests/test_gpu_arcface.py > $O/t.log 2>&1 &&
PC_SMALL_SPLITK=1 timeout -k 10 200 python -u bench.py --no-cpu --frames per-frame --steps 2 --warmup 1 > $O/pf_split.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --frames per-frame --steps 2 --warmup 1 > $O/pf_nosplit.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c5 > $O/c5.log 2>&1
rc=$?
tail -3 $O/t.log
for f in pf_split pf_nosplit c5; do tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['roofline'].get('per_net'))"; done
exit $rc
