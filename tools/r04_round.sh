# Round-4 GPU session: small-GEMM probe, library A/B, the whole GPU suite, bench.
set -e
mkdir -p gpurun_out
timeout -k 10 240 bash tools/small_gemm_probe.sh > gpurun_out/r04e_small_gemm.log 2>&1
timeout -k 10 600 bash tools/r04_ab_pack.sh > gpurun_out/r04f_ab_pack.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 400 --timeout-method thread > gpurun_out/r04g_gputests.log 2>&1
timeout -k 10 700 python bench.py > gpurun_out/r04g_bench.log 2>&1
