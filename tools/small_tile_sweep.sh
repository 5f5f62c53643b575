# per-layer times of the f16x3 ArcFace at a per-frame batch under each forced conv_fast tile
# usage: bash tools/small_tile_sweep.sh <batch> <tiles...>   (PC_CONV_FAST=k+1 forces tile k)
cd ${GRAFT_REPO_ROOT:-.}
B=$1; shift
echo "== default"
PROBE_MAXB=512 timeout -k 10 120 python -u tools/probe_layers.py arcx3 $B || exit $?
for k in "$@"; do
  echo "== PC_CONV_FAST=$((k + 1)) (tile $k)"
  PC_CONV_FAST=$((k + 1)) PROBE_MAXB=512 timeout -k 10 120 python -u tools/probe_layers.py arcx3 $B || exit $?
done
