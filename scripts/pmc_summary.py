"""Mean per-dispatch rocprofv3 counters by kernel (name filter), from one or more counter_collection.csv."""
import csv
import sys
from collections import defaultdict


def load(paths, filt):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for row in csv.DictReader(open(p)):
            name = row["Kernel_Name"]
            if filt and not any(f in name for f in filt):
                continue
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


if __name__ == "__main__":
    paths = [a for a in sys.argv[1:] if a.endswith(".csv")]
    filt = [a for a in sys.argv[1:] if not a.endswith(".csv")]
    for name, cs in load(paths, filt).items():
        print(name[:110])
        vals = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(vals):
            print(f"   {c:28s} {vals[c]:16.0f}  (n={len(cs[c])})")
        if "GRBM_GUI_ACTIVE" in vals and "SQ_VALU_MFMA_BUSY_CYCLES" in vals:
            kc = vals["GRBM_GUI_ACTIVE"] / 8
            print(f"   kernel cycles {kc:.0f}; MFMA busy / (cycles x 1024 SIMDs) = {vals['SQ_VALU_MFMA_BUSY_CYCLES'] / kc / 1024:.3f}")
        if "SQ_WAVE_CYCLES" in vals:
            wc = vals["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in vals:
                    print(f"   {c} / SQ_WAVE_CYCLES = {vals[c] / wc:.3f}")
