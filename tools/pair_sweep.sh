#!/bin/bash
# Per-class rates of the precomputed (OANet + Procrustes) workload as a function of the pair batch:
# how much of the point-conv stream the Infinity Cache absorbs when a batch's activations fit in it.
# usage: tools/pair_sweep.sh <outdir> [pairs...]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/$1"; shift
mkdir -p "$OUT"
PAIRS=("$@")
[ ${#PAIRS[@]} -eq 0 ] && PAIRS=(8 16 32 64 128 435)
for p in "${PAIRS[@]}"; do
  steps=$(( 4000 / p )); [ $steps -lt 5 ] && steps=5
  timeout -k 10 240 python3 "$R/bench.py" --workload precomputed --pairs $p --steps $steps --warmup 3 \
    --no-cpu-baseline > "$OUT/pairs_$p.json" 2> "$OUT/pairs_$p.err" || exit $?
  echo "pairs $p done"
done
