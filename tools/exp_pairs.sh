#!/bin/bash
# general-path experiment libraries (ggnn_amd/exp/lib_*.so), same box: the
# reference configuration (tools/pairs_probe.py) and the run_epoch line;
# EXP_TEST names the library the general-path GPU tests run against first
set -e
T=${EXP_TEST:-ggnn_amd/exp/lib_wpe2.so}
if [ "$T" != none ]; then
  GGNN_LIB=$T timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py tests/test_gpu_graphs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp_tests.log 2>&1
fi
for L in ggnn_amd/exp/lib_*.so; do
  n=$(basename $L .so)
  GGNN_LIB=$L timeout -k 10 200 python3 tools/pairs_probe.py > gpurun_out/pp_$n.log 2>&1
  GGNN_LIB=$L timeout -k 10 300 python3 bench.py --e2e-only --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/e2e_$n.log 2>&1
done
