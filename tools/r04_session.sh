# Round-4 GPU session 13: k_wgrad256 with whole NBUF groups and a separate
# tail (no exit test inside the unrolled group): the GPU suite, then the
# config-3 step and the real-density reference configuration against the
# previous library (tools/lib_cur.so), alternated.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r04s_tests.log 2>&1
for rep in 1 2; do
  for lib in tools/lib_cur.so ggnn_amd/libggnn.so; do
    GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py --variants skip --rounds 1 --steps 100 >> gpurun_out/r04s_ab.log 2>&1
    GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py --trees --variants skip --rounds 1 --steps 100 >> gpurun_out/r04s_ab.log 2>&1
  done
done
