"""Print the kernel sequence of one training step from a rocprofv3 kernel_trace.csv, in
launch order, with durations and the idle gap before each kernel.  Steps are delimited by
the fused optimizer kernel (one per step).

    python tools/prof_sequence.py out/r18_kernel_trace.csv [step_index_from_end=1] [boundary=adam_kernel]
"""
import csv
import sys

path = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
marker = sys.argv[3] if len(sys.argv) > 3 else "adam_kernel"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(ends) < back + 1:
    sys.exit("need at least %d '%s' launches, found %d" % (back + 1, marker, len(ends)))
lo, hi = ends[-back - 1] + 1, ends[-back] + 1
step = rows[lo:hi]
t0 = int(step[0]["Start_Timestamp"])
prev_end = int(rows[lo - 1]["End_Timestamp"])
busy = 0
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print("%9.1f us  +%6.1f gap  %8.1f us  %s" % ((s - t0) / 1e3, (s - prev_end) / 1e3,
                                                 (e - s) / 1e3, r["Kernel_Name"][:110]))
    prev_end = max(prev_end, e)
wall = int(step[-1]["End_Timestamp"]) - t0
print("step: %d kernels, wall %.1f us, kernel-busy %.1f us (%.1f%%)" % (
    len(step), wall / 1e3, busy / 1e3, 100.0 * busy / wall))
