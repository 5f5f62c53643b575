#!/bin/bash
# One parametrised GPU-box runner (replaces the per-session gpu_*.sh scripts).
# usage (GPU box):  bash tools/gpu_run.sh <tag> "<step>" ["<step>" ...]
# Every step runs under its own time limit; the first failing step ends the run
# (no retries, nothing else touches the GPU after an abort / fault / timeout).
# Logs go to gpurun_out/<tag>/<n>_<kind>.log. Steps:
#   suite [pytest -k expr]        the -m gpu suite (one process)
#   smoke                         __graft_entry__.smoke()
#   bench <workload> [args...]    bench.py --workload <workload> (c2 / c3 / c4 / c5)
#   profile <tag>                 tools/profile_round.sh (kernel trace + PMC traffic + MFMA busy)
#   pmc <match> <script> [args]   tools/pmc_cmd.sh counter passes over one python script
#   probe <script> [args...]      python tools/<script> args
#   ab <libA> <libB> <reps> <script> [args]
#                                 interleaved A/B of two library builds (PC_LIB_PATH), one box
#   abenv <VAR> <valA> <valB> <reps> <script> [args]
#                                 interleaved A/B of one environment variable, one box
# Leading KEY=VALUE words of a step are exported for that step only, e.g.
#   "PC_BENCH_NOPROF=1 bench c3 --frames per-frame"
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
i=0
for step in "$@"; do
  i=$((i + 1))
  read -r -a a <<< "$step"
  envs=()
  while [[ ${#a[@]} -gt 0 && ${a[0]} == *=* ]]; do envs+=("${a[0]}"); a=("${a[@]:1}"); done
  kind=${a[0]}
  log=$O/${i}_${kind}.log
  (
  [ ${#envs[@]} -gt 0 ] && export "${envs[@]}"
  case $kind in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
        ${a[1]:+-k "${a[*]:1}"} > "$log" 2>&1 ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py --workload "${a[1]}" "${a[@]:2}" > "$log" 2>&1 ;;
    profile)
      timeout -k 10 1500 bash tools/profile_round.sh "${a[1]}" > "$log" 2>&1 ;;
    pmc)
      timeout -k 10 900 bash tools/pmc_cmd.sh "$TAG/pmc_${a[1]}" "${a[1]}" "tools/${a[2]}" "${a[@]:3}" > "$log" 2>&1 ;;
    probe)
      timeout -k 10 400 python -u "tools/${a[1]}" "${a[@]:2}" > "$log" 2>&1 ;;
    sh)
      timeout -k 10 600 bash "tools/${a[1]}" "${a[@]:2}" > "$log" 2>&1 ;;
    ab)
      rc=0
      for r in $(seq 1 "${a[3]}"); do
        for lib in "${a[1]}" "${a[2]}"; do
          echo "== $lib rep $r" >> "$log"
          PC_LIB_PATH=$lib timeout -k 10 300 python -u "tools/${a[4]}" "${a[@]:5}" >> "$log" 2>&1 || { rc=$?; break 2; }
        done
      done
      (exit $rc) ;;
    abenv)
      rc=0
      for r in $(seq 1 "${a[4]}"); do
        for v in "${a[2]}" "${a[3]}"; do
          echo "== ${a[1]}=$v rep $r" >> "$log"
          env "${a[1]}=$v" timeout -k 10 300 python -u "tools/${a[5]}" "${a[@]:6}" >> "$log" 2>&1 || { rc=$?; break 2; }
        done
      done
      (exit $rc) ;;
    *)
      echo "unknown step: $step" > "$log"; false ;;
  esac
  )
  rc=$?
  echo "step $i ($step): rc=$rc"
  tail -3 "$log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
