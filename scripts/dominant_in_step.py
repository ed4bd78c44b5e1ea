"""The bench's dominant op inside the profiled training step: the layer3 dilated 3x3 conv in its
forward form (fwd and dgrad of Bottleneck.conv2, 256->256, 65x129, d=2), i.e. the stream-K
launches of that shape and the piece reduce after each (the bf16x6 weight planes are split at
pack time, once per SGD step, not per call).  The layer3 shape is the
only one of those kernels in the 40-160 us band at 1024x512 (layer2 ~25 us, layer4 ~300 us).
Usage: dominant_in_step.py <rocprofv3 kernel_trace.csv> [kernel-substring]"""
import csv
import sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_igemm_fwd_sk<128, 128"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
main, red = [], []
for i, r in enumerate(rows):
    if name in r["Kernel_Name"] and 40.0 <= dur(r) <= 160.0:
        main.append(dur(r))
        nxt = rows[i + 1] if i + 1 < len(rows) else None
        if nxt is not None and "k_sk_reduce" in nxt["Kernel_Name"]:
            red.append(dur(nxt))
avg = lambda v: sum(v) / max(len(v), 1)
print(f"layer3 forward-form launches: {len(main)}  stream-K kernel avg {avg(main):.1f} us  reduce avg "
      f"{avg(red):.1f} us  op avg {avg(main) + avg(red):.1f} us")
