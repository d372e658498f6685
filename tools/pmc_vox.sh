#!/bin/bash
# SQ counter passes over tools/vox_micro.py (the voxelisation kernels) -> <outdir>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/$1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 "$R/tools/vox_micro.py" 3 > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 "$R/tools/pmc_summary.py" "$OUT"
