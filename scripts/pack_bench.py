"""Weight-pack kernels A/B (msl_conv_set_pack_form 0: k_pack + k_split_pack, 1: k_pack_split) on
the model's conv shapes; run under rocprofv3 --kernel-trace for the per-kernel durations."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from maxsquareloss_amd import hip

lib = hip.load()
SHAPES = [("d", 1, 256, 256), ("d", 1, 512, 512), ("d", 2, 2048, 19), ("p", 1, 1024, 256), ("p", 1, 256, 1024)]
for form in (0, 1):
    lib.msl_conv_set_pack_form(form)
    for kind, nb, cin, cout in SHAPES:
        k = 3 if kind == "d" else 1
        w = torch.randn(nb, cout, cin, k, k, device="cuda")
        for fd in (0, 1):
            n = lib.msl_dconv_packed_elems(nb, cin, cout, fd) if kind == "d" else lib.msl_pconv_packed_elems(cin, cout, fd)
            buf = torch.empty(n, device="cuda")
            for _ in range(20):
                if kind == "d":
                    lib.msl_dconv_pack(w.data_ptr(), cout * cin * 9, nb, cin, cout, fd, buf.data_ptr(), hip.stream_ptr())
                else:
                    lib.msl_pconv_pack(w.data_ptr(), cin, cout, fd, buf.data_ptr(), hip.stream_ptr())
torch.cuda.synchronize()
lib.msl_conv_set_pack_form(1)
print("done")
