set -e
A="--no-cpu-baseline --no-side --steps 100 --warmup 10"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c_gputests.log 2>&1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/r03c_bench.log 2>&1
timeout -k 10 200 python bench.py $A > gpurun_out/exp_base.log 2>&1
GGNN_GRU_BWD_RT=1 timeout -k 10 200 python bench.py $A > gpurun_out/exp_rt1.log 2>&1
GGNN_GRU_BWD_RT=1 GGNN_LIB=ggnn_amd/exp/lib_du.so timeout -k 10 200 python bench.py $A > gpurun_out/exp_du_rt1.log 2>&1
GGNN_LIB=ggnn_amd/exp/lib_du.so timeout -k 10 200 python bench.py $A > gpurun_out/exp_du_rt2.log 2>&1
python tools/bench_summary.py gpurun_out/exp_*.log
