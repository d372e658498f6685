#!/bin/bash
# sample GPU power / clocks while a command runs: tools/smi_sample.sh <outfile> <cmd...>
OUT=$1; shift
( while true; do date +%s.%N; timeout 5 rocm-smi -d 0 --showpower --showclocks 2>/dev/null | grep -E "Power|sclk|fclk|mclk"; sleep 0.2; done ) > "$OUT" 2>&1 &
P=$!
"$@"
rc=$?
kill $P 2>/dev/null
wait $P 2>/dev/null
exit $rc
