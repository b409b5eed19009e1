#!/bin/bash
# PMC passes over tools/e2e_profile.py (run_epoch at the reference defaults on its own
# sentences, eager path): per-kernel instruction mix and stall counters of the
# small general-path products.  Usage (GPU box): bash tools/e2e_pmc.sh OUTDIR
set -e
OUT=${1:-gpurun_out/e2e_pmc}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o p -- python3 tools/e2e_profile.py --no-cprofile > "$OUT/pass$i.log" 2>&1
done
