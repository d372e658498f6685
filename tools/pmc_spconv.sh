#!/bin/bash
# Beyond-L2 read traffic (rocprofv3 --pmc FETCH_SIZE) of the sparse conv per kernel-map row order:
# tools/spconv_micro.py's launches of one FCGF layer, in its order (orders x xcd, 2 warmup + iters each).
# usage: tools/pmc_spconv.sh <outdir> <layer tag, e.g. s1:1:64:64> [iters]   (then: python tools/pmc_spconv.py <outdir>)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/$1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/FETCH_SIZE" -o pmc --output-format csv -- \
  python3 "$R/tools/spconv_micro.py" --only "$2" --iters "${3:-3}" > "$OUT/micro.log" 2>&1
