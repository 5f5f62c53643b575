set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh r03 > gpurun_out/prof_r03.log 2>&1
rc=$?
tail -5 gpurun_out/prof_r03.log
ls gpurun_out/prof_r03
exit $rc
