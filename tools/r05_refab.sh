# b=256 and b=20 reference-model A/B (the general path's pair mode) over
# libraries, plus rocprofv3 kernel stats per library at b=256.
#   LIBS="a.so b.so" PROF="a.so b.so" TAG=... bash tools/r05_refab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for args in "--reference --variants skip,keep90 --rounds 1 --steps 30" "--reference --batch 20 --variants skip,keep90 --rounds 1 --steps 100"; do
  for lib in $LIBS; do
    GGNN_LIB=$lib timeout -k 10 240 python3 tools/ab_step.py $args >> gpurun_out/${TAG}_refab.log 2>&1 || { echo REFAB_FAILED; tail -5 gpurun_out/${TAG}_refab.log; exit 1; }
  done
done
for lib in $PROF; do
  n=$(basename $lib .so)
  GGNN_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_$n -o p -- python3 tools/ab_step.py --reference --variants skip --rounds 1 --steps 20 > gpurun_out/${TAG}_prof_$n.log 2>&1 || { echo PROF_FAILED; tail -5 gpurun_out/${TAG}_prof_$n.log; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/${TAG}_refab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'].split('/')[-1], d['variant'], d['ms_per_step'], d['kernels'])
"
