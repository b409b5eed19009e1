# Round-4 GPU session 14: the ring / K-split epilogues load a column's E
# factors or old D values (GG_ADD) up front instead of one round trip per
# element: the GPU suite, then the reference configuration (b = 20, 256) and
# config 3 against the previous library (tools/lib_prev.so).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r04u_tests.log 2>&1
for b in 20 256; do
  for lib in tools/lib_prev.so ggnn_amd/libggnn.so; do
    GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py --reference --batch $b --variants skip,keep9 --rounds 1 --steps 50 >> gpurun_out/r04u_ab.log 2>&1
  done
done
for lib in tools/lib_prev.so ggnn_amd/libggnn.so; do
  GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py --variants skip --rounds 1 --steps 100 >> gpurun_out/r04u_ab.log 2>&1
done
