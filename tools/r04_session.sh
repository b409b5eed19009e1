# Round-4 GPU session 16: the GRU weight gradients with the timesteps as terms
# of one chunk (fewer fp32 atomics per output): the GPU suite, then the
# reference configuration (b = 20, 256) against the previous library.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r04z_tests.log 2>&1
for b in 20 256; do
  for lib in tools/lib_prev.so ggnn_amd/libggnn.so; do
    GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py --reference --batch $b --variants skip,keep9 --rounds 1 --steps 50 >> gpurun_out/r04z_ab.log 2>&1
  done
done
