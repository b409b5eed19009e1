#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, no tracing
# domains mixed in).  Usage (GPU box): bash tools/pmc_profile.sh OUTDIR [bench args]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---steps 2 --warmup 1 --no-cpu-baseline --no-side}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o p -- python3 bench.py $ARGS > "$OUT/pass$i.log" 2>&1
done
PMC_BENCH_ARGS="$ARGS" python3 tools/pmc_summary.py "$OUT" "$OUT/pmc_traffic.json"
