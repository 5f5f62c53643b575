# per-layer times of one net under each forced conv_fast tile (PC_CONV_FAST=k+1) next to the default plan
# usage: bash tools/tile_sweep.sh <arc|arcx3|scrfd|scrfdx3> <batch> <tiles...>   (PROBE_MAXB / PROBE_D pass through)
cd ${GRAFT_REPO_ROOT:-.}
NET=$1; B=$2; shift 2
echo "== default"
timeout -k 10 120 python -u tools/probe_layers.py $NET $B || exit $?
for k in "$@"; do
  echo "== PC_CONV_FAST=$((k + 1)) (tile $k)"
  PC_CONV_FAST=$((k + 1)) timeout -k 10 120 python -u tools/probe_layers.py $NET $B || exit $?
done
