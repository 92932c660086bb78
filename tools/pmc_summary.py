"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (one or more files),
plus derived ratios (VALU/SALU instructions per MFMA, MFMA-busy share of wave time).
    python tools/pmc_summary.py run1/p_counter_collection.csv [run2/...csv]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if k.startswith("void at::") or k.startswith("at::"):
            continue
        k = k.replace("void ", "").split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(agg):
    v = {c: agg[k][c] / max(len(disp[k][c]), 1) for c in agg[k]}
    print(k)
    print("    " + "  ".join("%s=%.3g" % (c, x) for c, x in sorted(v.items())))
    mf = v.get("SQ_INSTS_MFMA", 0)
    if mf:
        print("    VALU/MFMA=%.2f  SALU/MFMA=%.2f  LDS/MFMA=%.2f" % (
            v.get("SQ_INSTS_VALU", 0) / mf, v.get("SQ_INSTS_SALU", 0) / mf,
            v.get("SQ_INSTS_LDS", 0) / mf))
    if v.get("SQ_WAVE_CYCLES"):
        w = v["SQ_WAVE_CYCLES"]
        print("    wave time: active %.0f%%  waiting %.0f%%  issue-stalled %.0f%%" % (
            100 * v.get("SQ_ACTIVE_INST_ANY", 0) / w, 100 * v.get("SQ_WAIT_ANY", 0) / w,
            100 * v.get("SQ_WAIT_INST_ANY", 0) / w))
