# The 32-row ring-tile products of a 20-sentence batch (hidden 400, ~600 rows):
# how their time scales with M, N, K, and a 4-slot ring (kernel 3) beside the
# shipped 2-slot one (kernel 2).  tools/gemm_ring_probe.py: M N K a_layout b_layout prec kernel reps
for k in 2; do
for s in "700 800 800" "700 800 400" "700 800 200" "700 800 100" "700 400 800" "700 128 800" "32 800 800" "2800 800 800" "700 800 800 0 1"; do
  set -- $s
  timeout -k 5 60 python tools/gemm_ring_probe.py $1 $2 $3 ${4:-0} ${5:-0} fp32 $k 50 | sed "s/^/kernel $k layout ${4:-0}${5:-0}: /" || exit 1
done
done
