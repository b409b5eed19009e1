#!/bin/bash
# PMC passes over one k_gemm / k_gemm_ring shape (tools/gemm_ring_probe.py):
# bash tools/ring_pmc.sh OUTDIR M N K al bl prec kernel
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_WAVES" \
  "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o p -- python3 tools/gemm_ring_probe.py "$@" 3 > "$OUT/pass$i.log" 2>&1
done
