set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03q
O=gpurun_out/r03q
timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/a_default.log 2>&1 &&
PERSON_CAPTURE_AMD_EMBED_STREAM=0 timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/b_one_chain.log 2>&1 &&
PERSON_CAPTURE_AMD_EMBED_STREAM=0 PC_CHAIN=0 timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/c_one_nochain.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/d_default2.log 2>&1
rc=$?
for f in a_default b_one_chain c_one_nochain d_default2; do tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['per_net'])"; done
exit $rc
