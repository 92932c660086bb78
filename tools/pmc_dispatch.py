"""Per-DISPATCH hardware counters from rocprofv3 --pmc counter_collection.csv files, joined
with a kernel trace for durations, and the derived per-kernel rates.

    python tools/pmc_dispatch.py [--trace kernel_trace.csv] [--flops name=GFLOP ...]
                                 pass1/..._counter_collection.csv [pass2/...csv ...]

Each pass is its own rocprofv3 run (the counter slots of one pass are limited), so a
dispatch is identified across passes by (kernel name, its ordinal among that kernel's
dispatches in the run): the same bench.py steps launch the same sequence every run.
Rows: one per dispatch (name, ordinal, grid, duration, raw counters), then derived:

* MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
  (SQ_VALU_MFMA_BUSY_CYCLES sums the matrix-pipe busy cycles of every SIMD;
  GRBM_GUI_ACTIVE sums the active cycles of the 8 XCDs - MI355X_MICROARCH.md "rocprofv3
  PMC slots" / "DVFS give-back");
* effective clock = GRBM_GUI_ACTIVE / 8 / duration;
* HBM bytes = 2 x FETCH_SIZE (gfx950 reports half of a wide streaming read) + WRITE_SIZE,
  both in KiB as rocprofv3 reports them;
* LDS bank-conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* wave-time split = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES.
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    return name.replace("void ", "").split("(")[0].replace("mpa::", "")


def load_pass(path):
    """-> {(kernel, ordinal): {"grid":..., "counters": {name: value}, "disp": id}}"""
    by_disp = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        e = by_disp.setdefault(d, {"name": r["Kernel_Name"], "grid": r.get("Grid_Size", ""),
                                   "counters": collections.defaultdict(float)})
        e["counters"][r["Counter_Name"]] += float(r["Counter_Value"])
    seen = collections.Counter()
    out = {}
    for d in sorted(by_disp, key=int):
        e = by_disp[d]
        k = short(e["name"])
        out[(k, seen[k])] = e
        seen[k] += 1
    return out


def load_trace(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seen = collections.Counter()
    out = {}
    for r in rows:
        k = short(r["Kernel_Name"])
        out[(k, seen[k])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        seen[k] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default=None)
    ap.add_argument("--match", default="", help="regex on the kernel name")
    ap.add_argument("passes", nargs="+")
    a = ap.parse_args()
    merged = collections.OrderedDict()
    for p in a.passes:
        for key, e in load_pass(p).items():
            m = merged.setdefault(key, {"grid": e["grid"], "c": {}})
            m["c"].update(e["counters"])
    dur = load_trace(a.trace) if a.trace else {}
    rx = re.compile(a.match) if a.match else None
    cols = sorted({c for m in merged.values() for c in m["c"]})
    print("# per dispatch: kernel #ordinal grid | duration us | derived | raw counters")
    for (k, i), m in merged.items():
        if rx and not rx.search(k):
            continue
        c = m["c"]
        d = []
        us = dur.get((k, i))
        if us:
            d.append("%.1f us" % us)
        ga = c.get("GRBM_GUI_ACTIVE")
        if ga and c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
            d.append("mfma %.1f%%" % (100.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (ga / 8 * 1024)))
        if ga and us:
            d.append("clk %.2f GHz" % (ga / 8 / (us * 1e3)))
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            hb = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024
            d.append("hbm %.0f MB" % (hb / 1e6) + (" (%.2f TB/s)" % (hb / us / 1e6) if us else ""))
        if c.get("SQ_LDS_IDX_ACTIVE"):
            d.append("lds-conf %.1f%%" % (100.0 * c.get("SQ_LDS_BANK_CONFLICT", 0)
                                          / c["SQ_LDS_IDX_ACTIVE"]))
        if c.get("SQ_WAVE_CYCLES"):
            w = c["SQ_WAVE_CYCLES"]
            d.append("wait %.0f%% stall %.0f%% active %.0f%%" % (
                100 * c.get("SQ_WAIT_ANY", 0) / w, 100 * c.get("SQ_WAIT_INST_ANY", 0) / w,
                100 * c.get("SQ_ACTIVE_INST_ANY", 0) / w))
        print("%s #%d grid=%s | %s" % (k, i, m["grid"], " | ".join(d)))
        print("    " + "  ".join("%s=%.4g" % (n, c[n]) for n in cols if n in c))


if __name__ == "__main__":
    main()
