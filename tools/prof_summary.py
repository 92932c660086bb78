"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total GPU time %.2f ms  (%.2f ms per step over %g steps)" % (tot / 1e6, tot / 1e6 / steps, steps))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print("%6.2f%% %9.3f ms/step n/step=%6.1f avg=%8.1f us  %s" % (
        100 * float(r["TotalDurationNs"]) / tot, float(r["TotalDurationNs"]) / 1e6 / steps,
        float(r["Calls"]) / steps, float(r["AverageNs"]) / 1e3, r["Name"][:100]))
