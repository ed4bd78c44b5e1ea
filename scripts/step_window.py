"""Per-iteration kernel time from a rocprofv3 kernel trace of bench.py: iterations are delimited by
the SGD kernel (one launch per step); prints, per iteration, the wall span, the summed kernel
time and the launch count, then the per-kernel totals of the last iteration.
usage: step_window.py <kernel_trace.csv> [top N]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cut = [i for i, r in enumerate(rows) if "k_sgd" in r["Kernel_Name"]]
    for a, b in zip(cut, cut[1:]):
        seg = rows[a + 1:b + 1]
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e6
        wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
        print(f"iteration: wall {wall:7.2f} ms  kernel-busy {busy:7.2f} ms  launches {len(seg)}")
    seg = rows[cut[-2] + 1:cut[-1] + 1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:90]
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("last iteration, per kernel:")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / 1e3:8.3f} ms {n:5d} x {t / n:8.1f} us  {k}")


if __name__ == "__main__":
    main()
