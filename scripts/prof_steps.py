"""Summarise a rocprofv3 kernel trace over the timed bench steps (after `--skip` SGD launches)."""
import csv, sys, collections
path = sys.argv[1]; skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
sgd = [i for i, r in enumerate(rows) if 'k_sgd' in r['Kernel_Name']]
start = sgd[skip - 1] + 1
steps = len(sgd) - skip
sel = rows[start:sgd[-1] + 1]
wall = (int(sel[-1]['End_Timestamp']) - int(sel[0]['Start_Timestamp'])) / 1e6
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in sel) / 1e6
agg = collections.defaultdict(lambda: [0, 0.0])
for r in sel:
    n = r['Kernel_Name']
    agg[n][0] += 1
    agg[n][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
print(f"steps {steps}  wall {wall/steps:.2f} ms/step  kernel-busy {busy/steps:.2f} ms/step  launches/step {len(sel)/steps:.0f}")
cat = collections.defaultdict(float)
for n, (c, t) in agg.items():
    k = ('msl:' + n.split('(')[0].replace('void ', '').replace('msl::', '')) if 'msl::' in n else ('torch-elementwise' if 'at::native' in n else ('MIOpen/BLAS:' + n[:40]))
    cat[k] += t
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{t/steps:8.3f} ms/step {c/steps:6.1f} calls/step avg {t/c*1e3:8.1f} us  {n[:100]}")
