set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03w
O=gpurun_out/r03w
PROBE_F32=1 timeout -k 10 300 python -u tools/probe_layers.py scrfd 32 > $O/scrfd32_f32.txt 2>&1
rc=$?
head -30 $O/scrfd32_f32.txt
exit $rc
