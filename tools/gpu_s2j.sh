# PMC passes over the 160x160x64 t2d conv (SCRFD's largest layer) and the 256x224 conv_fast tile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2j
PROBE_SHAPES=sc_160_64 timeout -k 10 400 bash tools/pmc_cmd.sh s2j_t2d conv_t2d tools/probe_conv.py auto > gpurun_out/s2j/t2d.txt 2>&1 &&
PROBE_SHAPES=s3_3x3_256 timeout -k 10 400 bash tools/pmc_cmd.sh s2j_fast conv_fast tools/probe_conv.py f13 > gpurun_out/s2j/fast.txt 2>&1
rc=$?
cat gpurun_out/s2j/t2d.txt gpurun_out/s2j/fast.txt | grep -v "^pass"
exit $rc
