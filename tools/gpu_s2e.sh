# C3 schedule A/B: two streams (default, chains off) vs one stream with resident chains vs one stream without
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2e; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/c3_two.log 2>&1 &&
PERSON_CAPTURE_AMD_EMBED_STREAM=0 timeout -k 10 300 python -u bench.py > $O/c3_one_chain.log 2>&1 &&
PERSON_CAPTURE_AMD_EMBED_STREAM=0 PC_CHAIN_MIN=1000000 timeout -k 10 300 python -u bench.py > $O/c3_one_nochain.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/c3_two_again.log 2>&1
rc=$?
for f in c3_two c3_one_chain c3_one_nochain c3_two_again; do echo $f; tail -1 $O/$f.log | cut -c1-160; done
exit $rc
