#!/bin/bash
# 4-slot ring for under-filled 128-row grids (GGNN_RING_DEEP = max workgroups), A/B on one box
set -e
export GGNN_LIB=ggnn_amd/exp/lib_deep.so
for D in 0 256 512; do
  for sh in "7680 800 800 0 0" "7680 400 800 0 0" "7680 800 400 0 1" "7680 400 400 0 0" "15360 800 800 0 0" "32768 800 400 0 0"; do
    GGNN_RING_DEEP=$D timeout -k 10 60 python3 tools/gemm_ring_probe.py $sh fp32 2 50 | sed "s/^/deep=$D /" >> gpurun_out/deep_probe.log 2>&1
  done
  GGNN_RING_DEEP=$D timeout -k 10 200 python3 tools/pairs_probe.py > gpurun_out/pp_deep$D.log 2>&1
done
