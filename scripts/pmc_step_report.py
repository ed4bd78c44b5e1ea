"""Per-kernel counter report of the UDA step from scripts/gpu_pmc_step.sh's three passes.

Kernels are grouped by (name, grid, workgroup) - one group per shape.  Columns: launches,
mean duration under the counter pass, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8
XCDs x 1024 SIMDs), fraction of wave time waiting to issue (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES),
memory-side bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; FETCH_SIZE doubled per the gfx950
correction of MI355X_MICROARCH.md; Infinity-Cache hits are counted, so this is fabric traffic, an
upper bound on HBM bytes) and those bytes / duration.
Only each pass's last `last` dispatches are kept (the timed steps: the warmup iteration runs
MIOpen's solver search, whose trial kernels would otherwise dominate).
usage: pmc_step_report.py <dir with pmcs_<tag>_{sq,f,w}> <tag> [top N] [last]"""
import csv
import os
import sys
from collections import defaultdict


def load(path, last):
    d = {}
    for r in csv.DictReader(open(path)):
        k = r["Dispatch_Id"]
        e = d.setdefault(k, {"name": r["Kernel_Name"], "grid": r["Grid_Size"], "wg": r["Workgroup_Size"],
                             "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "c": {}})
        e["c"][r["Counter_Name"]] = float(r["Counter_Value"])
    keep = sorted(d, key=int)[-last:]
    return {k: d[k] for k in keep}


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n[:60]


def main():
    root, tag = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
    last = int(sys.argv[4]) if len(sys.argv) > 4 else 3200
    sq = load(os.path.join(root, f"pmcs_{tag}_sq", "sq_counter_collection.csv"), last)
    f = load(os.path.join(root, f"pmcs_{tag}_f", "f_counter_collection.csv"), last)
    w = load(os.path.join(root, f"pmcs_{tag}_w", "w_counter_collection.csv"), last)
    g = defaultdict(lambda: defaultdict(list))
    for src, keys in ((sq, ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES")),
                      (f, ("FETCH_SIZE",)), (w, ("WRITE_SIZE",))):
        for e in src.values():
            key = (short(e["name"]), e["grid"], e["wg"])
            for k in keys:
                if k in e["c"]:
                    g[key][k].append(e["c"][k])
            g[key]["dur_sq" if src is sq else "dur_fw"].append(e["dur"])
    mean = lambda v: sum(v) / len(v) if v else float("nan")  # noqa: E731
    rows = []
    for key, c in g.items():
        n = len(c["dur_sq"])
        d = mean(c["dur_fw"]) if c["dur_fw"] else mean(c["dur_sq"])
        kc = mean(c["GRBM_GUI_ACTIVE"]) / 8
        mf = mean(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / (kc * 1024) if kc > 0 else float("nan")
        wi = mean(c["SQ_WAIT_INST_ANY"]) / mean(c["SQ_WAVE_CYCLES"]) if c["SQ_WAVE_CYCLES"] and mean(c["SQ_WAVE_CYCLES"]) > 0 else float("nan")
        by = 2 * mean(c["FETCH_SIZE"]) * 1024 + mean(c["WRITE_SIZE"]) * 1024
        rows.append((n * d, key, n, d, mf, wi, by, by / (d * 1e-6) / 1e9 if d > 0 else float("nan")))
    rows.sort(reverse=True)
    print(f"{'kernel':60s} {'grid':>9s} {'wg':>5s} {'n':>5s} {'us':>8s} {'mfma':>6s} {'wait':>6s} {'MB':>8s} {'GB/s':>7s}")
    for tot, key, n, d, mf, wi, by, bw in rows[:top]:
        print(f"{key[0]:60s} {key[1]:>9s} {key[2]:>5s} {n:5d} {d:8.1f} {mf:6.3f} {wi:6.3f} {by / 1e6:8.1f} {bw:7.0f}")


if __name__ == "__main__":
    main()
