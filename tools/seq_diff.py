"""Per-kernel step-time diff of two prof_sequence.py outputs (kernels above a threshold).

    python tools/seq_diff.py before.txt after.txt [min_us]
"""
import collections
import re
import sys


def load(path):
    d = collections.defaultdict(list)
    for line in open(path):
        m = re.match(r"\s*[\d.]+ us\s+\+\s*-?[\d.]+ gap\s+([\d.]+) us\s+(.*)", line)
        if m:
            d[m.group(2)[:64]].append(float(m.group(1)))
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
lim = float(sys.argv[3]) if len(sys.argv) > 3 else 50
ta = sum(sum(v) for v in a.values())
tb = sum(sum(v) for v in b.values())
print("%9s %9s %8s  kernel" % ("before", "after", "delta"))
for k in sorted(set(a) | set(b), key=lambda k: -max(sum(a.get(k, [0])), sum(b.get(k, [0])))):
    sa, sb = sum(a.get(k, [0])), sum(b.get(k, [0]))
    if max(sa, sb) >= lim:
        print("%9.1f %9.1f %+8.1f  %s" % (sa, sb, sb - sa, k))
print("%9.1f %9.1f %+8.1f  total" % (ta, tb, tb - ta))
