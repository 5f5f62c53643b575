set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03bb
O=gpurun_out/r03bb
timeout -k 10 600 python -u bench.py --no-cpu > $O/c3.log 2>&1
rc=$?
tail -1 $O/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']); p=d['parity']; print({k:p[k] for k in ('faces_f32','accept_mismatch_0.32','box_mismatch')}); print(p['smooth_frames']); print(p['detector_f32_mode'])"
exit $rc
