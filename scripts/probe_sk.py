"""Drive the diagnostic stamp build (scripts/probe_sk.hip): the layer3 3x3 d=2 forward over the 1024x512
pair, f16x3 BD form; checks the output against the library's own call, times the stamped and the plain
kernel, and prints where a K-step of a wave goes (shares of the stamped build's cycles per phase)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from maxsquareloss_amd import hip, ops  # noqa: E402

lib = hip.load()
so = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe_sk.so"))
c_p, c_i, c_sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
so.probe_bd_fwd.argtypes = [c_p, c_p, c_p] + [c_i] * 6 + [c_p, c_i, c_p, c_sz, c_p, c_i, c_p]
so.probe_workers.argtypes = [c_i] * 5
cin, cout, h, w, nimg, d = [int(v) for v in (sys.argv[1:7] if len(sys.argv) > 6 else (256, 256, 65, 129, 2, 2))]
g = torch.Generator().manual_seed(1)
x = torch.relu(torch.randn(1, cin, nimg, h, w, generator=g)).cuda()
wt = (torch.randn(cout, cin, 3, 3, generator=g) * 0.02).cuda()
cache = ops.PackCache()
packed = cache.get([wt], cin, cout, 0)
xpart = ops._parts(x)
wsb = max(lib.msl_dconv_fwd_workspace(1, cin, cout, h, w, nimg), 768 * 2 * 128 * 128 * 4 + 4096)
ws = hip.workspace(wsb, "cuda")
y_ref = torch.empty(1, cout, nimg, h, w, device="cuda")
hip.check(lib.msl_dconv_fwd_sc(x.data_ptr(), packed.data_ptr(), None, y_ref.data_ptr(), 1, cin, cout, h, w, nimg, d, 0,
                               hip.forms(), ws.data_ptr(), wsb, hip.stream_ptr(), *ops._pp(xpart)),
          "ref")
nw = so.probe_workers(cin, cout, h, w, nimg)
prof = torch.zeros(nw * 4 * 8, dtype=torch.int64, device="cuda")
y = torch.empty_like(y_ref)


def run(p):
    hip.check(so.probe_bd_fwd(x.data_ptr(), packed.data_ptr(), y.data_ptr(), cin, cout, h, w, nimg, d, xpart[0].data_ptr(),
                              xpart[1], ws.data_ptr(), wsb, prof.data_ptr(), p, hip.stream_ptr()), "probe")


def timed(p, reps=20):
    for _ in range(3):
        run(p)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run(p)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


t_plain, t_prof = timed(0), timed(1)
abl = {name: round(timed(v), 1) for v, name in ((16, "BN apply in the split (identity table)"), (2, "no B loads"), (4, "no A DMA"), (6, "no B loads, no A DMA"),
                                                (8, "no barrier"), (14, "no loads, no DMA, no barrier"))}
ok_plain = None
run(0)
torch.cuda.synchronize()
ok_plain = torch.equal(y, y_ref)
run(16)
torch.cuda.synchronize()
ok_apply = torch.equal(y, y_ref)
prof.zero_()
run(1)
torch.cuda.synchronize()
ph = prof.view(nw * 4, 8)[:, :6].double().cpu()
steps = ph[:, 5].sum().item()
tot = ph[:, :5].sum(0)
names = ["wait A pieces (vmcnt)", "barrier", "frag reads + split + MFMA issue + next issue", "lgkmcnt(0)", "epilogue"]
out = {"shape": [cin, cout, h, w, nimg, d], "workers": nw, "us_plain": round(t_plain, 1), "us_stamped": round(t_prof, 1), "us_ablations": abl,
       "plain_output_bitexact_vs_library": ok_plain, "apply_output_bitexact_vs_library": ok_apply, "kstep_waves": steps,
       "cycles_per_kstep": {n: round(tot[i].item() / steps, 1) for i, n in enumerate(names)},
       "shares": {n: round(tot[i].item() / tot.sum().item(), 3) for i, n in enumerate(names)}}
print(json.dumps(out))
