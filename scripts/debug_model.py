import sys; sys.path.insert(0, ".")
import torch, torch.nn.functional as F
from maxsquareloss_amd.graphs.models.deeplab_multi import DeeplabMulti, DilatedConv3x3, Classifier_Module
from maxsquareloss_amd.utils.synthetic import init_weights, synthetic_image
for (H, W, ng) in [(256, 512, True), (256, 512, False), (128, 256, True)]:
    m = init_weights(DeeplabMulti(19, False), 12345).cuda()
    worst = []
    def hook(mod, inp, out, name=None):
        x = inp[0].detach()
        if isinstance(mod, DilatedConv3x3):
            ref = F.conv2d(x, mod.weight.detach(), padding=mod.dilation[0], dilation=mod.dilation[0])
        else:
            c0, c1 = mod.conv2d_list[0], mod.conv2d_list[1]
            ref = F.conv2d(x, c0.weight, c0.bias, padding=6, dilation=6) + F.conv2d(x, c1.weight, c1.bias, padding=12, dilation=12)
        err = ((out.detach() - ref).abs().max() / ref.abs().max()).item()
        worst.append((err, name, tuple(x.shape)))
    for n, mod in m.named_modules():
        if isinstance(mod, (DilatedConv3x3, Classifier_Module)):
            mod.register_forward_hook(lambda mo, i, o, n=n: hook(mo, i, o, n))
    x = synthetic_image(H, W, 0).cuda()
    if ng:
        with torch.no_grad(): m(x)
    else:
        m(x)
    torch.cuda.synchronize()
    worst.sort(reverse=True)
    print(H, W, "no_grad" if ng else "grad", worst[:4], flush=True)
