# C3 pipeline knobs with the r03s2 kernels (default chunk 32 / ahead 2 / quantum 146)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2i; mkdir -p $O
run() { n=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --no-cpu --no-parity > $O/$n.log 2>&1 && echo "$n $(tail -1 $O/$n.log | cut -c1-120)"; }
run default PERSON_CAPTURE_AMD_SEED=0 &&
run q292 PERSON_CAPTURE_AMD_EMBED_QUANTUM=292 &&
run chunk16 PERSON_CAPTURE_AMD_PIPE_CHUNK=16 &&
run ahead3 PERSON_CAPTURE_AMD_PIPE_AHEAD=3 &&
run default2 PERSON_CAPTURE_AMD_SEED=0
