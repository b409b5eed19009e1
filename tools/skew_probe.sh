set -e
for k in 0 4 8 16 28 0; do
  GGNN_FWD_SKEW=$k timeout -k 10 200 python bench.py --no-cpu-baseline --no-side --dropout-keep 1 > gpurun_out/skew_$k.log 2>&1
  grep '^{' gpurun_out/skew_$k.log | tail -1 > gpurun_out/skew_${k}_$(date +%s).json
done
