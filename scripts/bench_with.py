"""Run bench.py with module switches set first (same-box A/B of a host-side switch, rocprofv3-friendly:
the program after rocprofv3's `--` is this script itself, no exec):

    python scripts/bench_with.py ops.BN_MASK_BITS=False [-- bench.py args]

Each NAME=VALUE sets maxsquareloss_amd.<module>.<attr> to the Python literal VALUE."""
import ast
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
args = sys.argv[1:]
rest = args[args.index("--") + 1:] if "--" in args else []
for a in args[: args.index("--")] if "--" in args else args:
    name, value = a.split("=", 1)
    mod, attr = name.rsplit(".", 1)
    m = importlib.import_module("maxsquareloss_amd." + mod)
    if not hasattr(m, attr):
        raise SystemExit(f"bench_with: maxsquareloss_amd.{mod} has no {attr}")
    setattr(m, attr, ast.literal_eval(value))
sys.argv = [os.path.join(ROOT, "bench.py")] + rest
os.chdir(ROOT)
runpy.run_path(sys.argv[0], run_name="__main__")
