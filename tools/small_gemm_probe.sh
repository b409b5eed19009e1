for s in "700 800 800" "700 800 400" "700 800 200" "700 800 100" "700 400 800" "700 128 800" "32 800 800" "2800 800 800" "11200 800 800"; do
  timeout -k 5 60 python tools/gemm_ring_probe.py $s 0 0 fp32 2 50 || exit 1
done
