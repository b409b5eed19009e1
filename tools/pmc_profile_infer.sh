#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over inference-only forwards (tools/gru_infer_probe.py),
# one counter per pass.  Usage (GPU box): bash tools/pmc_profile_infer.sh OUTDIR [precision]
set -e
OUT=${1:-gpurun_out/pmc_infer}
PREC=${2:-bf16}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o p -- python3 tools/gru_infer_probe.py $PREC 3 > "$OUT/pass$i.log" 2>&1
done
PMC_BENCH_ARGS="tools/gru_infer_probe.py --precision $PREC (inference forwards)" python3 tools/pmc_summary.py "$OUT" "$OUT/pmc_traffic.json"
