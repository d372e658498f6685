#!/bin/bash
# rocprofv3 kernel stats of tools/vox_micro.py for the default library and each tools/vsp/vp_*.so variant
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for lib in "$R/3d_multiview_reg_amd/libmvreg_hip.so" "$R"/tools/vsp/vp_*.so; do
  n=$(basename "$lib" .so)
  MVR_LIB="$lib" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vox_$n" -o t --output-format csv -- \
    python3 "$R/tools/vox_micro.py" 20 || exit $?
  python3 "$R/tools/kseq.py" "$R/gpurun_out/vox_$n/t_kernel_stats.csv" 40 vox_part vox_keys compact scan
done
