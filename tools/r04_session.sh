# Round-4 GPU session 12: config-3 step (ab_step default: b = 256, v = 128,
# hidden 256, C = 8, T = 5) with the round-3 library (tools/lib_r03.so) against
# the current one, alternated twice: did round 4 move the headline kernels?
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/lib_r03.so ggnn_amd/libggnn.so; do
    GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py --variants skip --rounds 2 --steps 100 >> gpurun_out/r04r_ab_cfg3.log 2>&1
  done
done
