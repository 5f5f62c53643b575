set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03aa
O=gpurun_out/r03aa
timeout -k 10 200 python -u tools/probe_layers.py scrfd 32 > $O/scrfd32.txt 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/a.log 2>&1 &&
PC_NO_SMALL_PLANS=1 timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/b.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/c.log 2>&1 &&
PC_NO_SMALL_PLANS=1 timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/d.log 2>&1
rc=$?
head -12 $O/scrfd32.txt
for f in a b c d; do tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['per_net'])"; done
exit $rc
