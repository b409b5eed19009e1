# Round-4 GPU session 8: k_gemm_ks with 1 / 2 / 4 column blocks per wave
# group: the whole GPU suite, kernel-trace durations of one product per split,
# and the reference configuration A/B against the pre-fusion library.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r04n_tests.log 2>&1
for k in 3 4 5; do
  timeout -k 10 300 bash tools/small_gemm_trace.sh /tmp/sgt$k $k > gpurun_out/r04n_small_gemm_trace_k$k.txt 2>&1
done
for b in 20 256; do
  GGNN_LIB=tools/lib_pack.so timeout -k 10 200 python tools/ab_step.py --reference --batch $b --variants skip,keep9 --rounds 1 --steps 50 >> gpurun_out/r04n_ab.log 2>&1
  timeout -k 10 200 python tools/ab_step.py --reference --batch $b --variants skip,keep9 --rounds 1 --steps 50 >> gpurun_out/r04n_ab.log 2>&1
done
