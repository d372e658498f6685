#!/bin/bash
# Run GPU steps in order; each "STEP <timeout> <logname> <cmd...>" line of the
# job file runs under its own time limit.  Stops at the first step that did not
# exit 0/1 (fault, abort, segfault, timeout) — nothing more touches the GPU then.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
JOB="$1"
while IFS= read -r line; do
  [[ -z "$line" || "$line" == \#* ]] && continue
  read -r to name cmd <<< "$line"
  echo "[step] $name (limit ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[step] $name rc=$rc in $(( $(date +%s) - start ))s"
  tail -5 "gpurun_out/$name.log"
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then
    echo "[step] stopping: $name exited $rc"
    exit $rc
  fi
done < "$JOB"
