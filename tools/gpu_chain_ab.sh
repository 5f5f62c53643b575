set -o pipefail
cd $GRAFT_REPO_ROOT
export PC_CHAIN_MODE=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_chain.py
unset PC_CHAIN_MODE
timeout -k 10 250 python -u tools/probe_chain_ab.py 256 3
