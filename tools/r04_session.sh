# Round-4 GPU session 3: small-product scaling probe and PMC passes over run_epoch
# (raw counter CSVs stay in /tmp on the box; only the per-kernel summary returns).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 bash tools/small_gemm_probe.sh > gpurun_out/r04i_small_gemm.log 2>&1
timeout -k 10 600 bash tools/e2e_pmc.sh /tmp/r04i_e2e_pmc > gpurun_out/r04i_e2e_pmc.log 2>&1
python3 tools/pmc_summary.py /tmp/r04i_e2e_pmc > gpurun_out/r04i_e2e_pmc_summary.txt 2>&1
cp /tmp/r04i_e2e_pmc/summary.json gpurun_out/r04i_e2e_pmc_summary.json
