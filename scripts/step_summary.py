"""Per-kernel summary of a rocprofv3 --kernel-trace --stats run of bench.py: ms per step, calls
per step, average duration (usage: step_summary.py <kernel_stats.csv> <steps> [top N])."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"kernel-busy {tot / 1e6 / steps:.2f} ms/step over {steps} steps (incl. warmup)")
    for r in rows[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) / steps:6.1f} calls/step "
              f"avg {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:110]}")


if __name__ == "__main__":
    main()
