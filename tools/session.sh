# GPU session script (rounds 5-6) (the command of one gpurun call)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r06x}
( while true; do date >> gpurun_out/${TAG}_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "$TESTS" ]; then
  eval "timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS" > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
if [ -n "$TESTS2" ]; then
  # a second selection, e.g. TESTS2="GGNN_LIB=tools/lib_x.so tests/test_gpu_parity.py -s"
  eval "$TESTS2_ENV timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS2" > gpurun_out/${TAG}_tests2.log 2>&1 || { echo TESTS2_FAILED; tail -40 gpurun_out/${TAG}_tests2.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests2.log
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
if [ -n "$E2EAB" ]; then
  # run_epoch at the reference defaults per library, alternated (no profiler):
  # E2EAB="lib1 lib2 ..."
  for i in 1 2; do
    for lib in $E2EAB; do
      echo "== $lib" >> gpurun_out/${TAG}_e2eab.log
      GGNN_LIB=$lib timeout -k 10 300 python3 tools/e2e_profile.py --no-cprofile >> gpurun_out/${TAG}_e2eab.log 2>&1 || { echo E2EAB_FAILED; tail -20 gpurun_out/${TAG}_e2eab.log; exit 1; }
    done
  done
  grep -E "^==|inst/s|per kind" gpurun_out/${TAG}_e2eab.log
fi
if [ -n "$E2E" ]; then
  # run_epoch at the reference defaults under a kernel + memory-copy trace;
  # per-batch kernel time, idle split (inside the graph / between steps), copies
  export TMPDIR=/tmp
  rm -rf /tmp/${TAG}_e2etrace
  timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/${TAG}_e2etrace -o run -- python3 tools/e2e_profile.py --no-cprofile > gpurun_out/${TAG}_e2etrace.log 2>&1 || { echo E2E_FAILED; tail -20 gpurun_out/${TAG}_e2etrace.log; exit 1; }
  python3 tools/trace_batch.py "$(find /tmp/${TAG}_e2etrace -name '*kernel_trace.csv' | head -1)" --copies "$(find /tmp/${TAG}_e2etrace -name '*memory_copy_trace.csv' | head -1)" --split k_slab_reduce,k_gemm_ring,k_gemm_ks > gpurun_out/${TAG}_e2e_train_batch_kernels.txt 2>&1
  head -12 gpurun_out/${TAG}_e2e_train_batch_kernels.txt
  grep -E "inst/s" gpurun_out/${TAG}_e2etrace.log
fi
if [ -n "$PROFILE" ]; then
  bash tools/profile_round.sh $TAG || { echo PROFILE_FAILED; tail -20 gpurun_out/${TAG}_*.log; exit 1; }
  grep -h '^{' gpurun_out/${TAG}_trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('TRACE LEG', d['value'], d['ms_per_step'], {k: (round(v['avg_launch_ms'],4), round(v['frac'],4)) for k, v in d['roofline']['kernels'].items()})"
  grep -h '^{' gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'], d['dropout_on']['ms_per_step'], d['kernel_breakdown'])"
  tail -2 gpurun_out/${TAG}_smoke.log
fi
