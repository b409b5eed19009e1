# round-5 GPU session script (the command of one gpurun call)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r05b}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
for i in 1 2; do
  for lib in tools/lib_r03.so tools/lib_r04.so ggnn_amd/libggnn.so tools/lib_gbd4.so; do
    GGNN_LIB=$lib timeout -k 10 120 python tools/ab_step.py --variants skip --rounds 2 --steps 100 >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  done
done
grep '"round": 1' gpurun_out/${TAG}_ab.log
