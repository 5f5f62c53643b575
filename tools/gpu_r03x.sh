set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03x
O=gpurun_out/r03x
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_arcface.py tests/test_gpu_chain.py > $O/t.log 2>&1 &&
PC_CHAIN=0 timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_nochain.txt 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/c3a.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --no-parity > $O/c3b.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c2 > $O/c2.log 2>&1
rc=$?
tail -2 $O/t.log; head -6 $O/arc_nochain.txt
for f in c3a c3b; do tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['per_net'], d['roofline']['kernel_avg_launch_us'])"; done
tail -1 $O/c2.log | cut -c1-300
exit $rc
