# A/B on one box (the reference configuration, dropout off / on):
#   tools/lib_before.so  the library before the two re-applied round-3 commits
#   tools/lib_pack.so    + 16-byte masked pack copies, one-launch staging clears
#   ggnn_amd/libggnn.so  + k_pair_reduce_x's batched pair lookups
set -e
for rep in 1 2; do
for lib in tools/lib_before.so tools/lib_pack.so ggnn_amd/libggnn.so; do
  GGNN_LIB=$lib timeout -k 10 200 python tools/ab_step.py --reference --variants skip,keep9 --rounds 1 --steps 50
done
done
timeout -k 10 300 python -u -m pytest -q --timeout 200 tests/test_gpu_generic.py
