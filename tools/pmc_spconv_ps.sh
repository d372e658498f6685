#!/bin/bash
# Counter passes over one sparse-conv layer of tools/spconv_planes_micro.py: the fp32-gather kernel (PS = 0) and the
# pre-split-planes kernel (PS = 1) in one process, told apart by their template names.
# usage: tools/pmc_spconv_ps.sh <outdir> <layer tag, e.g. s1:1:64:64>   (then: python tools/pmc_spconv_ps.py <outdir>)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/$1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "GRBM_GUI_ACTIVE SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 "$R/tools/spconv_planes_micro.py" --only "$2" --iters 3 > "$OUT/p$i.log" 2>&1 || exit $?
done
