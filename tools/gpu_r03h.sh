set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03h
O=gpurun_out/r03h
timeout -k 10 200 python -u tools/probe_layers.py scrfd 64 > $O/scrfd64.txt 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc256.txt 2>&1
rc=$?
cat $O/scrfd64.txt; cat $O/arc256.txt
exit $rc
