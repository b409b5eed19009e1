# Kernel durations (rocprofv3 kernel trace, not host-paced event timing) of one
# 32-row ring product per shape: whether a small product's time is its K walk
# (per-slice latency) or a per-launch constant.  Writes <out>/summary.txt.
#   bash tools/small_gemm_trace.sh <out dir> [kernel: 2 ring (default), 3 K split]
set -e
out=${1:-/tmp/sgt}
kern=${2:-2}
mkdir -p "$out"
: > "$out/summary.txt"
for s in "700 800 800" "700 800 400" "700 800 200" "700 800 100" "700 800 32" "32 800 800" "2800 800 200" \
         "2800 800 800" "700 128 800" "700 800 800 0 1"; do
  set -- $s
  tag="m$1_n$2_k$3_l${4:-0}${5:-0}_k$kern"
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$tag" -o run -- \
    python3 tools/gemm_ring_probe.py $1 $2 $3 ${4:-0} ${5:-0} fp32 $kern 200 > "$out/$tag.log" 2>&1
  f=$(find "$out/$tag" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$tag" "$(tail -1 $out/$tag.log)" >> "$out/summary.txt" <<'EOF'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_gemm_' in r['Name']]
for r in rows:
    print("%-22s %-48s calls %5s avg %8.2f us min %8.2f us max %8.2f us | event-timed: %s" % (
        sys.argv[2], r['Name'].replace('void ', '')[:40], r['Calls'], float(r['AverageNs']) / 1e3, float(r['MinNs']) / 1e3, float(r['MaxNs']) / 1e3,
        sys.argv[3]))
EOF
done
cat "$out/summary.txt"
