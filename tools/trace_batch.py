"""Per-kernel time per training batch from a rocprofv3 kernel trace of
tools/e2e_profile.py: the window of the last `--batches` training steps
(delimited by the optimizer's k_opt_adam launches).

    python tools/trace_batch.py gpurun_out/<dir>/run_kernel_trace.csv [--batches 102]
"""
import collections
import csv
import sys


def main(path, nb=102):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "k_opt_adam" in r["Kernel_Name"]]
    lo, hi = adam[-(nb + 1)], adam[-1]
    win = rows[lo + 1:hi + 1]
    t0, t1 = int(rows[lo]["End_Timestamp"]), int(rows[hi]["End_Timestamp"])
    tot, cnt = collections.defaultdict(float), collections.Counter()
    busy = 0.0
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = r["Kernel_Name"].split("(")[0][:90]
        tot[k] += d
        cnt[k] += 1
        busy += d
    print("window wall %.3f ms/batch, kernels busy %.3f ms/batch, %.1f launches/batch"
          % ((t1 - t0) / 1e6 / nb, busy / 1e3 / nb, len(win) / nb))
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:30]:
        print("%8.1f us/batch  %5.1f/batch  avg %6.1f us  %s" % (v / nb, cnt[k] / nb, v / cnt[k], k))


if __name__ == "__main__":
    a = sys.argv[1:]
    nb = int(a[a.index("--batches") + 1]) if "--batches" in a else 102
    main(a[0], nb)
