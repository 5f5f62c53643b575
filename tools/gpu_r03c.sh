set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PERSON_CAPTURE_AMD_DET_PRECISION=f32 timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_c3_det32.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-parity > gpurun_out/bench_c3_nochain2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-parity --precision f32 > gpurun_out/bench_c3_f32.log 2>&1
rc=$?
for f in det32 nochain2 f32; do tail -1 gpurun_out/bench_c3_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['roofline']['per_net'], d.get('parity',{}).get('accept_mismatch_0.32'), d.get('parity',{}).get('attribution'))"; done
exit $rc
