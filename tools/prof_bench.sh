#!/bin/bash
# rocprofv3 kernel-trace + stats of the default bench workload -> <outdir>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/$1"; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o trace --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline "$@"
