#!/bin/bash
# fma_mix limb residuals: bit check, GPU suite on the in-tree library, then
# A/B against the pre-change build (ggnn_amd/exp/lib_base.so) on one box
set -e
timeout -k 10 60 ./tools/limb_mix_test > gpurun_out/mix_check.log 2>&1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mix_tests.log 2>&1
A="--no-cpu-baseline --no-side --steps 100 --warmup 10"
for rep in 1 2; do
  for n in base mix; do
    GGNN_LIB=ggnn_amd/exp/lib_$n.so timeout -k 10 200 python3 bench.py $A > gpurun_out/exp_${n}_$rep.log 2>&1
  done
done
for n in base mix; do
  GGNN_LIB=ggnn_amd/exp/lib_$n.so timeout -k 10 200 python3 tools/pairs_probe.py > gpurun_out/pp_$n.log 2>&1
done
