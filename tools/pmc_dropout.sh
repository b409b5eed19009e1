#!/bin/bash
# L2 / HBM counters of the config-3 step's kernels with and without edge
# dropout (tools/ab_step.py variants), one counter group per pass.
# Usage (GPU box): bash tools/pmc_dropout.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc_dropout}
export TMPDIR=/tmp
mkdir -p "$OUT"
for v in skip ek90; do
  i=0
  for grp in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    mkdir -p "$OUT/$v"
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/$v/pass$i" -o p -- python3 tools/ab_step.py --variants $v --rounds 1 --steps 10 > "$OUT/$v/pass$i.log" 2>&1
  done
  python3 tools/pmc_summary.py "$OUT/$v" > "$OUT/$v.txt"
done
