#!/bin/bash
# SQ counter passes over one sparse-conv layer of tools/spconv_micro.py (one order, xcd 0).
# usage: tools/pmc_spconv_sq.sh <outdir> <layer tag> [order]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/$1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 "$R/tools/spconv_micro.py" --only "$2" --order "${3:-mask+morton}" --xcd 0 --iters 3 > "$OUT/p$i.log" 2>&1 || exit $?
done
