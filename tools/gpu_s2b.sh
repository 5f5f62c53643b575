# chain register stream 7 ahead (PC_CHAIN_MODE=2) vs LDS ring vs 3 ahead; conv_fast 256x224 phase split
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2b; mkdir -p $O
AB_WL=2 AB_MODE=1,2,0 timeout -k 10 200 python -u tools/probe_chain_ab.py 256 3 > $O/chain_ab.log 2>&1 &&
for d in 0 1 2 3 4; do PC_CONV_DBG=$d PROBE_SHAPES=s3_3x3_256 timeout -k 10 100 python -u tools/probe_conv.py f13 | sed "s/^/dbg $d /" || exit 1; done > $O/fast_dbg.log 2>&1
rc=$?
cat $O/chain_ab.log $O/fast_dbg.log | grep -v amdgpu.ids
exit $rc
