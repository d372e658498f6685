#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group) over the fused attention micro benchmark.
# usage: tools/pmc_attn.sh <pool|unpool> <outdir>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CASE=$1; OUT="$R/$2"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT" \
           "SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 "$R/tools/attn_micro.py" --only "$CASE" --iters 3 --math 0 > "$OUT/p$i.log" 2>&1 || exit $?
done
