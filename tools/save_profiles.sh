#!/bin/bash
# Copy one GPU round's evidence from gpurun_out/ (scratch) into profiles/
# (tracked).  Usage: bash tools/save_profiles.sh TAG
set -e
TAG=$1
grep '^{' gpurun_out/${TAG}_bench.log | tail -1 > profiles/${TAG}_bench.json
cp gpurun_out/${TAG}_trace/bench_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
cp gpurun_out/${TAG}_pmc/summary.json profiles/${TAG}_pmc_summary.json
cp gpurun_out/${TAG}_pmc.log profiles/${TAG}_pmc_table.txt
cp gpurun_out/${TAG}_pmc/pmc_traffic.json profiles/pmc_traffic.json
if [ -d gpurun_out/${TAG}_pmcbf16 ]; then
  cp gpurun_out/${TAG}_pmcbf16/summary.json profiles/${TAG}_bf16_pmc_summary.json
  cp gpurun_out/${TAG}_pmcbf16.log profiles/${TAG}_bf16_pmc_table.txt
  cp gpurun_out/${TAG}_pmcbf16/pmc_traffic.json profiles/pmc_traffic_bf16.json
fi
if [ -d gpurun_out/${TAG}_pmcinfer ]; then
  cp gpurun_out/${TAG}_pmcinfer/summary.json profiles/${TAG}_bf16_infer_pmc_summary.json
  cp gpurun_out/${TAG}_pmcinfer/pmc_traffic.json profiles/pmc_traffic_bf16_infer.json
fi
[ -f gpurun_out/${TAG}_gputests.log ] && cp gpurun_out/${TAG}_gputests.log profiles/${TAG}_gputests.log
true
