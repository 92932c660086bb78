#!/bin/bash
# Alternating whole-step A/B of a baseline tree copy (abtree/: package + bench.py, built from
# the previous commit) against the working tree: bash scripts/gpu/ab_tree.sh TAG REPS [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=$1; REPS=$2; shift 2
export MPA_ALLOW_STALE=1
for i in $(seq 1 $REPS); do
  (cd abtree && timeout -k 10 300 python bench.py --small-batch 0 "$@" > ../gpurun_out/${TAG}_base_$i.json 2>/dev/null) || exit 1
  timeout -k 10 300 python bench.py --small-batch 0 "$@" > gpurun_out/${TAG}_new_$i.json 2>/dev/null || exit 1
  python - "$TAG" "$i" <<'PY'
import json, sys
t, i = sys.argv[1], sys.argv[2]
v = [json.loads(open("gpurun_out/%s_%s_%s.json" % (t, k, i)).read().strip().splitlines()[-1])["value"]
     for k in ("base", "new")]
print("rep", i, "base %.1f new %.1f" % tuple(v), flush=True)
PY
done
