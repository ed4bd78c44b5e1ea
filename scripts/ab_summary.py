"""Summarises a same-box A/B log of scripts/gpu_ab.sh: per op and build, the timings of both rounds."""
import collections
import json
import re
import sys

cur = None
d = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1]):
    if line.startswith("==="):
        cur = line.split()[1].split("/")[-2]
        continue
    if line.startswith("{"):
        r = json.loads(line)
        for k in ("fwd_us", "dgrad_us", "wgrad_us"):
            d[r["op"] + " " + k][cur].append(r[k])
    m = re.search(r'"ms_per_step": ([0-9.]+)', line)
    if m:
        d["step_ms"][cur].append(float(m.group(1)))
for k, v in d.items():
    print(f"{k:32s}", "  ".join(f"{lib}:{'/'.join(str(x) for x in xs)}" for lib, xs in v.items()))
