"""Per-kernel time per training batch from a rocprofv3 kernel trace of
tools/e2e_profile.py: the window of the last `--batches` training steps
(delimited by the optimizer's k_opt_adam launches), and where the window's
idle time sits: between the kernels of one step (inside the replayed graph)
or between two steps (the host's share: scoring the previous batch, staging
the next one's inputs, the graph launch), with the H2D copies a
--memory-copy-trace CSV shows in those gaps.

    python tools/trace_batch.py <dir>/run_kernel_trace.csv [--batches 102] [--copies <dir>/run_memory_copy_trace.csv]
        [--split k_slab_reduce,k_gemm_ring] [--untraced-ms 1.38]

Round 6: the traced window's wall is longer than the untraced run's (the
kernel tracer adds host work at every graph launch), and that extra time shows
up as ONE long gap per step in front of its first kernel.  Each step's longest
gap is therefore reported as the launch gap (host + tracer), not as idle time
inside the step's graph; with --untraced-ms (the same run's wall per batch
without the tracer, e.g. from its instances/s) the tracer's share is printed
as window wall - untraced wall.
"""
import collections
import csv
import sys


def main(path, nb=102, copies=None, split=(), untraced_ms=None):
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
    # idle time: gaps between consecutive kernels, split at the step boundaries;
    # a step starts at the first kernel after the optimizer that is not one of
    # the runtime's copy blits (the previous batch's fetch of the loss and the
    # heads' probabilities runs as __amd_rocclr_copyBuffer right after Adam):
    # every gap from Adam's end to that kernel is the host's
    starts = set()
    for i in adam[-(nb + 1):-1]:
        j = i + 1
        while j < hi and rows[j]["Kernel_Name"].startswith("__amd_rocclr"):
            starts.add(j)
            j += 1
        starts.add(j)
    inter, intra, launch, big = 0.0, 0.0, 0.0, collections.Counter()
    steps = [a for a in adam[-(nb + 1):]]
    prev_end = t0
    gaps = []          # (gap us, row index)
    for i in range(lo + 1, hi + 1):
        s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
        gaps.append((max(0, s - prev_end) / 1e3, i))
        prev_end = max(prev_end, e)
    # each step's longest gap: the graph launch (host work + the tracer's own)
    longest = set()
    for a0, a1 in zip(steps[:-1], steps[1:]):
        g = [x for x in gaps if a0 < x[1] <= a1]
        if g:
            longest.add(max(g)[1])
    for gap, i in gaps:
        if i in longest and i not in starts:
            launch += gap
        elif i in starts:
            inter += gap
        else:
            intra += gap
            if gap > 5.0:
                big[rows[i]["Kernel_Name"].split("(")[0][:60]] += gap
    wall = (t1 - t0) / 1e3
    print("window wall %.3f ms/batch, kernels busy %.3f ms/batch, %.1f launches/batch"
          % (wall / 1e3 / nb, busy / 1e3 / nb, len(win) / nb))
    print("idle %.1f us/batch: between steps %.1f us/batch (host: scoring, staging, graph launch), each step's "
          "longest gap %.1f us/batch (the graph launch under the tracer), the rest inside the step's graph "
          "%.1f us/batch (%.2f us per launch boundary)"
          % ((inter + intra + launch) / nb, inter / nb, launch / nb, intra / nb, intra / max(len(win) - 2 * nb, 1)))
    if untraced_ms:
        print("untraced wall %.3f ms/batch: the tracer adds %.3f ms/batch (window wall - untraced wall); kernels "
              "busy %.3f of the untraced wall" % (untraced_ms, wall / 1e3 / nb - untraced_ms, busy / 1e3 / nb))
    if big:
        print("  gaps > 5 us inside the step, before:", ", ".join("%s %.1f us/batch" % (k, v / nb)
                                                                   for k, v in big.most_common(6)))
    if copies:
        cr = list(csv.DictReader(open(copies)))
        h2d = [r for r in cr if "HOST_TO_DEVICE" in r.get("Direction", "") + r.get("Operation", "")
               and t0 <= int(r["Start_Timestamp"]) <= t1]
        d2h = [r for r in cr if "DEVICE_TO_HOST" in r.get("Direction", "") + r.get("Operation", "")
               and t0 <= int(r["Start_Timestamp"]) <= t1]
        for name, rs in (("H2D", h2d), ("D2H", d2h)):
            dur = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
            print("%s copies: %.1f per batch, %.1f us/batch" % (name, len(rs) / nb, dur / nb))
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:30]:
        print("%8.1f us/batch  %5.1f/batch  avg %6.1f us  %s" % (v / nb, cnt[k] / nb, v / cnt[k], k))
    # kernels named by --split: per launch grid (the same kernel serves
    # different products, e.g. k_slab_reduce)
    for name in split:
        g, gc = collections.defaultdict(float), collections.Counter()
        for r in win:
            if name not in r["Kernel_Name"]:
                continue
            key = "%s grid %s x %s" % (r["Kernel_Name"].split("(")[0][:60], r.get("Grid_Size_X", r.get("Grid_Size", "?")),
                                     r.get("Grid_Size_Y", "1"))
            g[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            gc[key] += 1
        for k, v in sorted(g.items(), key=lambda x: -x[1]):
            print("    %8.1f us/batch  %5.1f/batch  avg %6.1f us  %s" % (v / nb, gc[k] / nb, v / gc[k], k))


if __name__ == "__main__":
    a = sys.argv[1:]
    nb = int(a[a.index("--batches") + 1]) if "--batches" in a else 102
    cp = a[a.index("--copies") + 1] if "--copies" in a else None
    sp = a[a.index("--split") + 1].split(",") if "--split" in a else ()
    um = float(a[a.index("--untraced-ms") + 1]) if "--untraced-ms" in a else None
    main(a[0], nb, cp, sp, um)
