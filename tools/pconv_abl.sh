#!/bin/bash
# Point-conv ablation timings (tools/build_variant.sh pconv.hip pc_abl<bits> -DPCONV_ABL=<bits>):
# 1 no MFMA, 2 no split, 4 no epilogue, 8 no activation loads (results wrong; timing only)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for c in conv_pro_stats conv_res; do
  echo "== $c"
  python3 "$R/tools/gemm_micro.py" --math 1 --only $c 2>&1 | grep pconv
  for so in "$R"/tools/vsp/pc_abl*.so; do
    echo -n "$(basename $so .so): "
    MVR_LIB=$so python3 "$R/tools/gemm_micro.py" --math 1 --only $c 2>&1 | grep pconv
  done
done
