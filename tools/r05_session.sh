# round-5 GPU session script (the command of one gpurun call)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r05c}
( while true; do date >> gpurun_out/${TAG}_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "$TESTS" ]; then
  eval "timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS" > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
if [ -n "$AB" ]; then
  # library A/B, alternated: AB="lib1 lib2 ..." ABARGS="ab_step.py args"
  for i in 1 2; do
    for lib in $AB; do
      GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py ${ABARGS:---variants skip,keep90 --rounds 1 --steps 100} >> gpurun_out/${TAG}_ab.log 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/${TAG}_ab.log; exit 1; }
    done
  done
  python3 -c "
import json,sys
for l in open('gpurun_out/${TAG}_ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'].split('/')[-1], d['variant'], d['trees'], d['ms_per_step'], {k: v for k, v in d['kernels'].items() if k in ('gru_bwd','wgrad','prop_bwd','state_io','fwd_fused')})
"
fi
if [ -n "$PROFILE" ]; then
  bash tools/profile_round.sh $TAG || { echo PROFILE_FAILED; tail -20 gpurun_out/${TAG}_*.log; exit 1; }
  grep -h '^{' gpurun_out/${TAG}_trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('TRACE LEG', d['value'], d['ms_per_step'], {k: (round(v['avg_launch_ms'],4), round(v['frac'],4)) for k, v in d['roofline']['kernels'].items()})"
  grep -h '^{' gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'], d['dropout_on']['ms_per_step'], d['kernel_breakdown'])"
  tail -2 gpurun_out/${TAG}_smoke.log
fi
