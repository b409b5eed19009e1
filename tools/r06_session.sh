# round-6 GPU session: full -m gpu suite, then the config-3 step A/B of the
# in-tree library against other builds (alternated runs), then the MFMA shape
# probe; every step bounded, chained so that a failure ends the call
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r06e}
shift
LIBS=${@:-tools/lib_r05.so}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python tools/ab_step.py --variants skip,keep90 --rounds 1 --steps 100 >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  for L in $LIBS; do
    GGNN_LIB=$L timeout -k 10 200 python tools/ab_step.py --variants skip,keep90 --rounds 1 --steps 100 >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  done
done
timeout -k 10 200 tools/mfma_shape_probe 3 2 > gpurun_out/${TAG}_mfma_shape.json 2>&1 || exit 1
