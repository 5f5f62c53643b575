set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03cc
O=gpurun_out/r03cc
PERSON_CAPTURE_AMD_EMBED_STREAM=0 timeout -k 10 200 python -u tools/probe_c3_arc.py 3 > $O/one_chain.txt 2>&1 &&
PERSON_CAPTURE_AMD_EMBED_STREAM=0 PC_CHAIN=0 timeout -k 10 200 python -u tools/probe_c3_arc.py 3 > $O/one_nochain.txt 2>&1 &&
timeout -k 10 200 python -u tools/probe_c3_arc.py 3 > $O/two_default.txt 2>&1
rc=$?
for f in one_chain one_nochain two_default; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
exit $rc
