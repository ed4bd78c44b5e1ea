"""Instruction mix per basic block (blocks that contain MFMAs) of one kernel in a hipcc -S file."""
import collections
import sys

path, sym = sys.argv[1], sys.argv[2]
s = open(path).read()
i = s.index(sym + ":")
body = s[i:s.index(".Lfunc_end", i)]
lines = [l.split(";")[0].strip() for l in body.split("\n")]
lines = [l for l in lines if l and (l.endswith(":") or not l.startswith("."))]
blocks, cur = [], None
for l in lines:
    if l.endswith(":"):
        cur = [l]
        blocks.append(cur)
    elif cur is not None:
        cur.append(l)
for b in blocks:
    k = collections.Counter()
    for x in b[1:]:
        op = x.split()[0]
        if "mfma" in op:
            k["mfma"] += 1
        elif op.startswith("v_"):
            k["valu"] += 1
        elif op.startswith("s_waitcnt"):
            k["waitcnt"] += 1
        elif op.startswith("s_barrier"):
            k["barrier"] += 1
        elif op.startswith("s_"):
            k["salu"] += 1
        elif op.startswith("ds_"):
            k["lds"] += 1
        elif op.startswith(("buffer_", "global_")):
            k["vmem"] += 1
        else:
            k[op] += 1
    if len(sys.argv) > 3 or k["mfma"] or len(b) > 150:
        print(b[0], len(b) - 1, dict(k))
