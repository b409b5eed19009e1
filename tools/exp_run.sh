#!/bin/bash
# bench kernel breakdown of the in-tree library and of each experiment library
# under ggnn_amd/exp (GPU box); EXP_ARGS overrides the bench arguments
ARGS=${EXP_ARGS:---no-cpu-baseline --no-side --steps 10 --warmup 3}
for f in ggnn_amd/exp/lib_*.so; do
  n=$(basename $f .so)
  GGNN_LIB=$f timeout -k 10 200 python3 bench.py $ARGS > gpurun_out/exp_$n.log 2>&1 || { echo "fail $n"; exit 1; }
done
timeout -k 10 200 python3 bench.py $ARGS > gpurun_out/exp_base.log 2>&1
python3 tools/bench_summary.py gpurun_out/exp_*.log
