# Round-4 GPU session (run from the repo root on the GPU box):
#   A/B of the current library against tools/lib_pack.so (before k_pair_reduce_x's
#   batched lookups and the batch-aware pack) on the reference configuration,
#   the e2e kernel trace of run_epoch, the GPU suite and the bench line.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for lib in tools/lib_pack.so ggnn_amd/libggnn.so; do
  GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py --reference --variants skip,keep9 --rounds 1 --steps 50 >> gpurun_out/r04h_ab.log 2>&1
done
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04h_e2etrace -o run -- python3 tools/e2e_profile.py --no-cprofile > gpurun_out/r04h_e2etrace.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 400 --timeout-method thread > gpurun_out/r04h_gputests.log 2>&1
timeout -k 10 700 python bench.py > gpurun_out/r04h_bench.log 2>&1
