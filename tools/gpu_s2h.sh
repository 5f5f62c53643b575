# SCRFD odd-multiple-of-32 channel layers: generic kernel (auto) vs conv_fast tiles after the MUBUF change
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2h; mkdir -p $O
PROBE_SHAPES=sc_20_224,sc_40_96,sc_80_96 PC_CONV_T2D=0 timeout -k 10 300 python -u tools/probe_conv.py auto f8 f8:64 f5 f5:64 f11 f11:64 f7 f4 f1 f3 > $O/probe.log 2>&1
rc=$?
grep -v amdgpu.ids $O/probe.log
exit $rc
