"""Full-step A/B of 1x1 dispatch rules on one box: runs bench.py in this process with
ops.conv1x1_plan replaced by a variant.  Usage: bench_plan_ab.py VARIANT [bench.py args...]
  new   the current ops.conv1x1_plan
  old   the rules before the hybrid schedule (fwd HIP only with cin >= 512, 1024->256 residual dgrad
        on MIOpen + add, 1024-input wgrads on hipBLASLt)
  wgold current rules with the 256 -> 1024 and 512 -> 1024 weight gradients on hipBLASLt
  fwdm  "new" with the 256 -> 1024 forward on MIOpen (adopted after this A/B: profiles/r02_plan_ab.txt)"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from maxsquareloss_amd import ops  # noqa: E402

variant = sys.argv[1]
cur = ops.conv1x1_plan


def old(cin, cout, p, form="bf16x6", residual=False):
    x6 = form == "bf16x6"
    big = p > 16384
    fwd = "hip" if x6 and ((big and cout <= 64) or (not big and cin >= 512 and max(cin, cout) >= 1024)) else "miopen"
    if x6 and not big and max(cin, cout) >= 1024 and min(cin, cout) >= 256 and not (cin > cout and cout < 512):
        dgrad = "hip"
    elif cout > cin or big:
        dgrad = "hipblaslt"
    else:
        dgrad = "miopen"
    wgrad = "hip" if big or (x6 and max(cin, cout) >= 2048) else "hipblaslt"
    return fwd, dgrad, wgrad


def fwdm(cin, cout, p, form="bf16x6", residual=False):
    plan = cur(cin, cout, p, form, residual)
    return (("miopen",) + plan[1:]) if (cin, cout) == (256, 1024) else plan


def wgold(cin, cout, p, form="bf16x6", residual=False):
    plan = cur(cin, cout, p, form, residual)
    return (plan[:2] + ("hipblaslt",)) if (cin, cout) in ((256, 1024), (512, 1024)) else plan


ops.conv1x1_plan = {"new": cur, "old": old, "fwdm": fwdm, "wgold": wgold}[variant]
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"),
               run_name="__main__")
