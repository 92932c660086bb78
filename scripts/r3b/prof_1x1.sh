#!/bin/bash
# kernel trace of DenseNet's small 3x3 growth convs in isolation
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; R=$(pwd)
cd /tmp
ZOO_ONLY="${ZOO_ONLY}" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p1x1 -o run -- python3 $R/tools/bench_zoo_convs.py densenet 256 5 > $R/$O/p1x1.log 2>&1 || exit 1
cd $R
cat $O/p1x1.log | tail -3
f=$(find $O/p1x1 -name "*kernel_stats.csv" | head -1); head -20 $f
f=$(find $O/p1x1 -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=sorted(csv.DictReader(open(sys.argv[1])), key=lambda r:int(r["Start_Timestamp"]))
for r in rows[-45:]:
    print("%8.1f us grid %s wg %s %s"%((int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3, r.get("Grid_Size",""), r.get("Workgroup_Size",""), r["Kernel_Name"][:90]))
PY
rm -f $f
