"""Per-category time of ONE training step from a rocprofv3 kernel_trace.csv (the step
before the last optimizer kernel, or ``back`` steps from the end): convolution forward /
dgrad / wgrad, BN forward / backward, concat, pools, loss, optimizer, ATen / runtime
kernels.  Used for the zoo models' profiles (profiles/*_step_breakdown_r3.txt).

    python tools/step_breakdown.py prof/run_kernel_trace.csv [back=1] [top=12]
"""
import csv
import re
import sys
from collections import defaultdict

CATS = [
    ("aten/runtime", r"at::native|__amd_rocclr"),
    ("optimizer", r"adam_kernel|sgd_kernel|transpose_krsc|zero_f32|step_inc"),
    ("conv wgrad", r"wgrad|splitk_finalize"),
    ("conv (stem)", r"conv_stem"),
    ("conv fwd/dgrad (halo)", r"conv3_halo_kernel|conv3_strip_kernel"),
    ("conv/GEMM fwd/dgrad (igemm)", r"igemm_rows|igemm_kernel|igemm_dma|gemm"),
    ("conv1 dgrad + norm1 bwd (dense_gacc)", r"dense_gacc"),
    ("BN backward", r"bn_bwd|maxpool_bn_bwd|slab_reduce|act_bwd|bn_defer"),
    ("BN forward + stats", r"bn_fwd|bn_stats|slab_stats|slab_fold|bn_relu_maxpool|relu_kernel"),
    ("concat / channel copy", r"concat|chan_accum|chan_extract"),
    ("pooling", r"pool|adaptive"),
    ("loss", r"ce_|argmax"),
    ("preprocess", r"preprocess"),
]


def category(name: str) -> str:
    for cat, pat in CATS:
        if re.search(pat, name):
            return cat
    return "other"


def main():
    path = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"] or
            "sgd_kernel" in r["Kernel_Name"]]
    if len(ends) < back + 1:
        sys.exit("need %d optimizer launches, found %d" % (back + 1, len(ends)))
    step = rows[ends[-back - 1] + 1: ends[-back] + 1]
    wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    per = defaultdict(float)
    cnt = defaultdict(int)
    kern = defaultdict(float)
    kcnt = defaultdict(int)
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c = category(r["Kernel_Name"])
        per[c] += d
        cnt[c] += 1
        k = r["Kernel_Name"].split("(")[0][:90]
        kern[k] += d
        kcnt[k] += 1
    busy = sum(per.values())
    print("step: %d kernels, wall %.1f us, kernel-busy %.1f us" % (len(step), wall, busy))
    for c, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print("  %-30s %9.1f us  %5.1f%%  %4d launches" % (c, v, 100 * v / busy, cnt[c]))
    print("top kernels:")
    for k, v in sorted(kern.items(), key=lambda kv: -kv[1])[:top]:
        print("  %9.1f us %4d x  %s" % (v, kcnt[k], k))


if __name__ == "__main__":
    main()
