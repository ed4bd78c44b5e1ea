"""Kernel-time breakdown of ONE replayed training iteration from a rocprofv3 --kernel-trace CSV
(the kernels between two consecutive SGD launches), grouped by kernel family, with the replay's wall
time (first start to last end) - the sum exceeds the wall time when streams overlap.

    python scripts/replay_breakdown.py <kernel_trace.csv> [replay index, default 3]
"""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
idx = [i for i, r in enumerate(rows) if "k_sgd" in r["Kernel_Name"]]
seg = rows[idx[k] + 1: idx[k + 1] + 1]
fam = defaultdict(lambda: [0, 0.0])
for r in seg:
    n = r["Kernel_Name"]
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    if "k_igemm_fwd_sk2" in n:
        t = [x.strip() for x in n.split("<", 1)[1].rstrip(">").split(",")]  # BM BN G ST WM WN PW MT ACC [BD]
        pw, acc, bd = t[6] == "true", t[8] == "true", len(t) > 9 and t[9] == "true"
        n = ("fwd-form GEMM " + ("fp16 " if t[7] == "8" else "f16x3 ") + ("pointwise" if pw else "3x3") +
             (" acc" if acc else "") + (" (B in registers)" if bd else ""))
    elif "k_igemm_fwd_sk<" in n:
        n = "fwd-form GEMM exact-f32 " + n.split("<")[1].split(",")[0] + "-row"
    elif "elementwise" in n:
        n = "torch elementwise"
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    fam[n][0] += 1
    fam[n][1] += d
wall = (max(int(r["End_Timestamp"]) for r in seg) - int(seg[0]["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in fam.values())
print(f"replay {k}: {len(seg)} kernels, kernel time {tot / 1e3:.2f} ms, wall {wall / 1e3:.2f} ms")
for n, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
    print(f"{t / 1e3:8.3f} ms {c:5d}  {t / c:8.1f} us  {n[:100]}")
