# interleaved C3 / C2 A/B on one box: this session's kernels (new) vs the session-start build (old, e925577)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2ab; mkdir -p $O
L=person_capture_amd/lib
cp $L/libpcgpu.so $L/libpcgpu_new.so
rc=0
for r in 1 2; do
  for v in new old; do
    cp $L/libpcgpu_$v.so $L/libpcgpu.so
    timeout -k 10 300 python -u bench.py --no-cpu --no-parity > $O/c3_${v}_$r.log 2>&1 || { rc=1; break 2; }
    timeout -k 10 200 python -u bench.py --workload c2 > $O/c2_${v}_$r.log 2>&1 || { rc=1; break 2; }
    echo "$v $r c3 $(tail -1 $O/c3_${v}_$r.log | cut -c90-130) c2 $(tail -1 $O/c2_${v}_$r.log | cut -c120-150)"
  done
done
cp $L/libpcgpu_new.so $L/libpcgpu.so
exit $rc
