"""Print the headline numbers of bench.py JSON logs: python tools/bench_summary.py log..."""
import json
import sys

for path in sys.argv[1:]:
    try:
        lines = [l for l in open(path).read().splitlines() if l.startswith("{")]
        d = json.loads(lines[-1])
    except Exception as e:  # noqa: BLE001
        print(path, "unreadable:", e)
        continue
    print("%s: %s %.1f %s  %.3f ms/step  dtype=%s  roofline %s %.1f TF (%.1f%%)" % (
        path, d["metric"][:22], d["value"], d["unit"], d["ms_per_step"], d["dtype"],
        d["roofline"]["kernel"], d["roofline"]["achieved"] or 0, 100 * (d["roofline"]["frac"] or 0)))
    print("   ", {k: round(v["ms_per_step"], 3) for k, v in d.get("kernel_breakdown", {}).items()})
    if "cpu_baseline" in d:
        print("    cpu:", d["cpu_baseline"])
