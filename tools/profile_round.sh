#!/bin/bash
# One round's GPU evidence (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats over the bench command
#   2. PMC passes (tools/pmc_profile.sh) -> per-launch HBM traffic, fp32-parity
#      and bf16 modes (profiles/pmc_traffic.json, profiles/pmc_traffic_bf16.json)
#   3. the default bench line (with the CPU baseline), roofline.traffic filled
# Usage: bash tools/profile_round.sh TAG   (outputs under gpurun_out/TAG_*)
set -e
TAG=${1:-r02}
export TMPDIR=/tmp
# the bench's own timed leg and nothing else (dropout off, no side lines): the
# k_fwd_fused / k_gru_bwd averages of this trace and the roofline of the JSON
# line in ${TAG}_trace.log come from the same launches
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o bench -- \
  python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-side --no-dropout-leg > gpurun_out/${TAG}_trace.log 2>&1
PMC_RUN=$TAG bash tools/pmc_profile.sh gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc.log 2>&1
cp gpurun_out/${TAG}_pmc/pmc_traffic.json profiles/pmc_traffic.json
PMC_RUN=$TAG bash tools/pmc_profile.sh gpurun_out/${TAG}_pmcbf16 --steps 2 --warmup 1 --no-cpu-baseline --no-side \
  --precision bf16 --pmc-unfused-leg > gpurun_out/${TAG}_pmcbf16.log 2>&1
cp gpurun_out/${TAG}_pmcbf16/pmc_traffic.json profiles/pmc_traffic_bf16.json
# inference-only forwards (no saves): the GRU's bytes against SURVEY §8d's 12 v h
bash tools/pmc_profile_infer.sh gpurun_out/${TAG}_pmcinfer bf16 > gpurun_out/${TAG}_pmcinfer.log 2>&1
cp gpurun_out/${TAG}_pmcinfer/pmc_traffic.json profiles/pmc_traffic_bf16_infer.json
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
