#!/bin/bash
# HBM traffic of the bench's kernels: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE cannot
# share a pass on gfx950) over one timed bench step, each with the per-launch class sequence (one
# stream: counter collection serialises the dispatches anyway, and the class join needs one launch order).
# usage: tools/pmc_bench.sh <outdir> [bench args, e.g. --math split16]   (then: python tools/pmc_traffic.py <outdir>)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/$1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  MVR_PROF_MARK=1 timeout -k 10 600 rocprofv3 --pmc $c -d "$OUT/$c" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --no-pipeline --prof-seq "$OUT/seq_$c.json" "${@:2}" \
    > "$OUT/bench_$c.log" 2>&1 || exit $?
done
