# Round-4 GPU session 6: small-product kernel durations from the kernel trace
# (tools/small_gemm_trace.sh), and the per-kernel split of the reference
# configuration's 20-sentence training step under edge dropout (k_edge_bits and
# the masked dW product).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/small_gemm_trace.sh /tmp/sgt > gpurun_out/r04l_small_gemm_trace.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r04l_ab -o ab -- \
  python3 tools/ab_step.py --reference --batch 20 --variants keep9 --rounds 1 --steps 30 > gpurun_out/r04l_ab_keep9.log 2>&1
cp "$(find /tmp/r04l_ab -name '*kernel_stats.csv' | head -1)" gpurun_out/r04l_ab_keep9_b20_kernel_stats.csv
