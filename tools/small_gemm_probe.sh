# The 32-row ring-tile products of a 20-sentence batch (hidden 400, ~600-700 rows):
# how one launch's time scales with M, N and K (tools/gemm_ring_probe.py:
# M N K a_layout b_layout prec kernel reps).  "2800 800 200" is the same work as
# "700 800 800" cut into 4 K chunks (what a split-K launch would run: 532 workgroups).
for s in "700 800 800" "700 800 400" "700 800 200" "700 800 100" "700 400 800" "700 128 800" "32 800 800" \
         "2800 800 800" "2800 800 200" "1400 800 400" "700 800 800 0 1"; do
  set -- $s
  timeout -k 5 60 python tools/gemm_ring_probe.py $1 $2 $3 ${4:-0} ${5:-0} fp32 2 50 | sed "s/^/layout ${4:-0}${5:-0}: /" || exit 1
done
