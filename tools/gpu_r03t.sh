set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03t
O=gpurun_out/r03t
timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/a.log 2>&1 &&
PERSON_CAPTURE_AMD_CHAIN=on PERSON_CAPTURE_AMD_EMBED_PRIORITY=-1 timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/b.log 2>&1 &&
PERSON_CAPTURE_AMD_EMBED_PRIORITY=-1 timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/c.log 2>&1 &&
PERSON_CAPTURE_AMD_CHAIN=on timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/d.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/e.log 2>&1
rc=$?
for f in a b c d e; do tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['per_net'])"; done
exit $rc
