"""Inter-kernel gap distribution of training steps from a rocprofv3 kernel_trace.csv: eager
launches vs HIP-graph replay (bench.py --graph on), same batch.

    python tools/gap_stats.py trace.csv [steps=5] [boundary=adam_kernel]

A step is the kernels after one optimizer kernel up to and including the next.  For each
of the last `steps` steps: wall (previous optimizer kernel's end to the last end), kernel-busy (union of kernel
intervals, so overlapping side-stream kernels count once), and the idle time between
consecutive kernel intervals bucketed by length.  Printed: per-step lines and the mean.
"""
import csv
import sys


def union_busy(iv):
    iv = sorted(iv)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e in iv:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s <= cur_e:
            cur_e = max(cur_e, e)
        else:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
    if cur_e is not None:
        busy += cur_e - cur_s
    return busy, gaps


BUCKETS = [(0, 1e3), (1e3, 2e3), (2e3, 5e3), (5e3, 10e3), (10e3, 50e3), (50e3, float("inf"))]


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    marker = sys.argv[3] if len(sys.argv) > 3 else "adam_kernel"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(ends) < 2:
        sys.exit("need at least two '%s' launches" % marker)
    sel = list(zip(ends[:-1], ends[1:]))[-nsteps:]
    tot = {"wall": 0.0, "busy": 0.0, "n": 0, "k": 0}
    hist_tot = [0.0] * len(BUCKETS)
    cnt_tot = [0] * len(BUCKETS)
    for a, b in sel:
        step = rows[a + 1:b + 1]
        # from the previous optimizer kernel's end: the idle time between steps (host
        # enqueue or replay launch) counts as a gap of this step
        t0 = int(rows[a]["End_Timestamp"])
        iv = [(t0, t0)] + [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step]
        wall = max(e for _, e in iv) - t0
        busy, gaps = union_busy(iv)
        hist = [0.0] * len(BUCKETS)
        cnt = [0] * len(BUCKETS)
        for g in gaps:
            for i, (lo, hi) in enumerate(BUCKETS):
                if lo <= g < hi:
                    hist[i] += g
                    cnt[i] += 1
        print("step: %d kernels, wall %.1f us, busy %.1f us, idle %.1f us in %d gaps | %s" % (
            len(step), wall / 1e3, busy / 1e3, (wall - busy) / 1e3, len(gaps),
            "  ".join("%s:%d/%.0fus" % (_lab(lo, hi), c, h / 1e3)
                      for (lo, hi), c, h in zip(BUCKETS, cnt, hist))))
        tot["wall"] += wall
        tot["busy"] += busy
        tot["n"] += 1
        tot["k"] += len(step)
        for i in range(len(BUCKETS)):
            hist_tot[i] += hist[i]
            cnt_tot[i] += cnt[i]
    n = max(tot["n"], 1)
    print("mean over %d steps: %.0f kernels, wall %.1f us, busy %.1f us, idle %.1f us | %s" % (
        n, tot["k"] / n, tot["wall"] / n / 1e3, tot["busy"] / n / 1e3,
        (tot["wall"] - tot["busy"]) / n / 1e3,
        "  ".join("%s:%.1f/%.0fus" % (_lab(lo, hi), c / n, h / n / 1e3)
                  for (lo, hi), c, h in zip(BUCKETS, cnt_tot, hist_tot))))


def _lab(lo, hi):
    return ("<%gus" % (hi / 1e3)) if lo == 0 else (">%gus" % (lo / 1e3) if hi == float("inf")
                                                   else "%g-%gus" % (lo / 1e3, hi / 1e3))


if __name__ == "__main__":
    main()
