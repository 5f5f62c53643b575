set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03y
O=gpurun_out/r03y
PC_CHAIN=0 timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_r128.txt 2>&1 &&
PC_CHAIN=0 PC_CONV_ROWB=64 timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_r64.txt 2>&1 &&
PC_CHAIN=0 timeout -k 10 200 python -u tools/probe_layers.py arc 292 > $O/arc292_r128.txt 2>&1 &&
PC_CHAIN=0 PC_CONV_ROWB=64 timeout -k 10 200 python -u tools/probe_layers.py arc 292 > $O/arc292_r64.txt 2>&1
rc=$?
for f in arc_r128 arc_r64 arc292_r128 arc292_r64; do echo "== $f"; sed -n 2,5p $O/$f.txt; done
exit $rc
