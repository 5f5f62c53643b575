# interleaved A/B of two builds of libpcgpu.so on one box (new t2d epilogue addressing vs old)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2m; mkdir -p $O
L=person_capture_amd/lib
cp $L/libpcgpu.so $L/libpcgpu_new.so
rc=0
for r in 1 2; do
  for v in new old; do
    cp $L/libpcgpu_$v.so $L/libpcgpu.so
    PROBE_SHAPES=sc_160_64,sc_80_96,s1_3x3_64,s0_3x3_64_112 timeout -k 10 200 python -u tools/probe_conv.py auto 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/probe.log || { rc=1; break 2; }
    timeout -k 10 200 python -u tools/probe_layers.py scrfd 32 2>&1 | grep "batch 32" | sed "s/^/$v /" >> $O/probe.log || { rc=1; break 2; }
  done
done
cp $L/libpcgpu_new.so $L/libpcgpu.so
cat $O/probe.log
exit $rc
