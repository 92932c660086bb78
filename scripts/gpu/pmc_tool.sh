#!/bin/bash
# One rocprofv3 PMC pass (plus kernel trace/stats) over a python tool, summarised per kernel:
#   bash scripts/gpu/pmc_tool.sh TAG "COUNTERS" tools/x.py ARGS...
# -> gpurun_out/TAG_pmc/ and gpurun_out/TAG_pmc.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
TAG=$1; CTRS=$2; shift 2
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
  -d $R/gpurun_out/${TAG}_pmc -o p -- python3 "$@" > gpurun_out/${TAG}_pmc.log 2>&1 || {
  tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
f=$(find gpurun_out/${TAG}_pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" > gpurun_out/${TAG}_pmc.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))[:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    n = max(cnt[(k, c)] for c in d)
    print(k, "dispatches", n)
    for c, v in sorted(d.items()):
        print("   %-32s %.4g (per dispatch %.4g)" % (c, v, v / n))
PY
cat gpurun_out/${TAG}_pmc.txt | head -60
find gpurun_out/${TAG}_pmc -name "*.csv" -size +20M -delete
