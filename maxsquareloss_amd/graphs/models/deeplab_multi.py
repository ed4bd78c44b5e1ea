"""DeepLabv2 / ResNet-101 "multi" model with the MI355X hot path.

Drop-in for graphs/models/deeplab_multi.py of the reference:
  - same constructor `DeeplabMulti(num_classes=21, pretrained=True)` (:174),
  - same module tree and state_dict keys (`layer3.5.conv2.weight`,
    `layer6.conv2d_list.1.bias`, ...),
  - same `forward(x) -> (x2, x1)` (layer6 head, layer5 head) (:113-130),
  - same `optim_parameters(args)` groups, duplicates included (:132-171, Q2).

What runs where (no library kernel is left on the step, so it is bit-reproducible run to run):
  - every stride-1 3x3 Bottleneck.conv2 (dilation 2 in layer3, 4 in layer4, and
    1 in layers 1-2) -> `DilatedConv3x3`, HIP implicit-GEMM kernels (fwd, dgrad,
    wgrad; fp32 in the f16x3 form by default);
  - the ASPP heads (live branches d=6 and d=12 only, quirk Q1) -> one fused
    two-branch HIP conv with both biases;
  - bilinear upsampling (align_corners=True) -> HIP kernel; the result keeps a
    handle on the low-res logits for the fused losses;
  - every BatchNorm (train mode, batch statistics of the one image, Q9) fused with the
    following ReLU and, for bn3, the residual add -> HIP kernels with fp64-accumulated
    statistics (MIOpen's single-pass variance is not accurate enough at bs=1);
  - every 1x1 conv -> `PointwiseConv`: the HIP pointwise GEMMs, weight gradients accumulated in
    place into the flat gradient buffer, conv1's data gradient summing in the identity
    residual's gradient (ops.ResidualGrad); layer2.0's stride-2 conv1 and downsample read one
    shared x[:, :, ::2, ::2] (ops.subsample);
  - the stem 7x7/2 conv -> `StemConv` (im2col + the pointwise GEMM), the ceil-mode maxpool ->
    `MaxPool` (csrc/stem.hip, gather-form backward).
"""
import torch
import torch.nn as nn

from ... import ops

affine_par = True


class DilatedConv3x3(nn.Conv2d):
    """nn.Conv2d(c, c, 3, stride=1, padding=d, dilation=d, bias=False) on the HIP kernels."""

    def __init__(self, in_channels, out_channels, dilation=1):
        super().__init__(in_channels, out_channels, kernel_size=3, stride=1, padding=dilation,
                         dilation=dilation, bias=False)
        self._pack = ops.PackCache()

    def forward(self, x):
        return ops.dconv3x3(x, self.weight, self.dilation[0], self._pack)


# Bottleneck blocks with an identity residual let conv1's data-gradient GEMM sum in the residual's
# gradient (ops.ResidualGrad) instead of autograd's separate add; False restores the add (tests).
FUSE_RESIDUAL_GRAD = True
# r05: a downsample block's conv1 also sums the downsample conv's data gradient (no accumulation kernel)
FUSE_DOWNSAMPLE_GRAD = True


class PointwiseConv(nn.Conv2d):
    """nn.Conv2d(cin, cout, 1, stride, bias=False) on the HIP pointwise GEMMs (ops.pconv).  A strided
    one reads x[:, :, ::stride, ::stride]; `presampled` says the caller already passed that."""

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__(in_channels, out_channels, kernel_size=1, stride=stride, bias=False)
        self._pack = ops.PackCache(pointwise=True)

    def forward(self, x, residual_grad=None, presampled=False, grad_to=None):
        if self.stride[0] != 1 and not presampled:
            x = ops.subsample(x, self.stride[0])
        return ops.pconv(x, self.weight, self._pack, residual_grad, grad_to)


class StemConv(nn.Conv2d):
    """ResNetMulti.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False) (deeplab_multi.py:73):
    im2col + the HIP pointwise GEMM (ops.stem_conv)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding):
        super().__init__(in_channels, out_channels, kernel_size=kernel_size, stride=stride, padding=padding,
                         bias=False)
        self._pack = ops.PackCache(pointwise=True)

    def forward(self, x):
        return ops.stem_conv(x, self.weight, self.stride[0], self.padding[0], self._pack)


class MaxPool(nn.MaxPool2d):
    """nn.MaxPool2d(3, 2, 1, ceil_mode=True) (deeplab_multi.py:77) on HIP (ops.maxpool2d)."""

    def forward(self, x):
        return ops.maxpool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode)


def conv1x1(inplanes, planes, stride):
    return PointwiseConv(inplanes, planes, stride)


class Bottleneck(nn.Module):
    """deeplab_multi.py:8-48 (Caffe-style: the stride sits on conv1)."""

    expansion = 4

    def __init__(self, inplanes, planes, stride=1, dilation=1, downsample=None, bn_momentum=0.1):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes, affine=affine_par)
        self.conv2 = DilatedConv3x3(planes, planes, dilation=dilation)
        self.bn2 = nn.BatchNorm2d(planes, affine=affine_par)
        self.conv3 = conv1x1(planes, planes * 4, 1)
        self.bn3 = nn.BatchNorm2d(planes * 4, affine=affine_par)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # identity residual: its gradient is summed into x's gradient by conv1's data-gradient
        # GEMM (ops.ResidualGrad) rather than by autograd's accumulation kernel; r05: likewise the
        # downsample conv's data gradient (both read xs)
        fuse = (FUSE_RESIDUAL_GRAD and torch.is_grad_enabled() and
                (self.downsample is None or FUSE_DOWNSAMPLE_GRAD))
        hold = ops.ResidualGrad() if fuse else None
        # a strided block (layer2.0): conv1 and the downsample read one shared x[:, :, ::s, ::s]
        xs = ops.subsample(x, self.stride) if self.stride != 1 else x
        out = ops.bn_act(self.bn1, self.conv1(xs, hold, presampled=True), relu=True)
        out = ops.bn_act(self.bn2, self.conv2(out), relu=True)
        if self.downsample is not None:
            residual = ops.bn_act(self.downsample[1], self.downsample[0](xs, presampled=True, grad_to=hold))
            hold_bn3 = None
        else:
            residual = x.detach() if fuse else x
            hold_bn3 = hold
        # bn3 + residual add + ReLU in one kernel (deeplab_multi.py:38-46)
        return ops.bn_act(self.bn3, self.conv3(out), residual=residual, relu=True, residual_grad=hold_bn3)


class Classifier_Module(nn.Module):
    """ASPP head (deeplab_multi.py:51-66).

    The reference returns inside its loop, so only conv2d_list[0] (d=6) and
    conv2d_list[1] (d=12) ever run (quirk Q1); branches 2 and 3 exist for
    state_dict compatibility and never receive gradients.
    """

    def __init__(self, inplanes, dilation_series, padding_series, num_classes):
        super().__init__()
        self.conv2d_list = nn.ModuleList()
        for dilation, padding in zip(dilation_series, padding_series):
            self.conv2d_list.append(nn.Conv2d(inplanes, num_classes, kernel_size=3, stride=1,
                                              padding=padding, dilation=dilation, bias=True))
        for m in self.conv2d_list:
            m.weight.data.normal_(0, 0.01)
        self._pack = ops.PackCache()

    def forward(self, x):
        c0, c1 = self.conv2d_list[0], self.conv2d_list[1]
        return ops.aspp2(x, c0.weight, c0.bias, c1.weight, c1.bias, c0.dilation[0], c1.dilation[0],
                         self._pack)


class ResNetMulti(nn.Module):
    """deeplab_multi.py:69-171."""

    def __init__(self, block, layers, num_classes):
        self.inplanes = 64
        super().__init__()
        self.conv1 = StemConv(3, 64, kernel_size=7, stride=2, padding=3)
        self.bn1 = nn.BatchNorm2d(64, affine=affine_par)
        for i in self.bn1.parameters():
            i.requires_grad = False
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = MaxPool(kernel_size=3, stride=2, padding=1, ceil_mode=True)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=1, dilation=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=1, dilation=4)
        self.layer5 = self._make_pred_layer(Classifier_Module, 1024, [6, 12, 18, 24], [6, 12, 18, 24], num_classes)
        self.layer6 = self._make_pred_layer(Classifier_Module, 2048, [6, 12, 18, 24], [6, 12, 18, 24], num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data.normal_(0, 0.01)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _make_layer(self, block, planes, blocks, stride=1, dilation=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion or dilation == 2 or dilation == 4:
            downsample = nn.Sequential(
                conv1x1(self.inplanes, planes * block.expansion, stride),
                nn.BatchNorm2d(planes * block.expansion, affine=affine_par))
        layers = [block(self.inplanes, planes, stride, dilation=dilation, downsample=downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, dilation=dilation))
        return nn.Sequential(*layers)

    def _make_pred_layer(self, block, inplanes, dilation_series, padding_series, num_classes):
        return block(inplanes, dilation_series, padding_series, num_classes)

    # With keep_split, _heads cuts the graph at layer3's output and after the layer3 blocks in split_cuts:
    # the points where a captured data-parallel step splits its backward into segments (utils/graph.py),
    # so the gradients each segment finishes (layer4 and the heads; then groups of layer3 blocks) are
    # exchanged while the next segments' backward runs.  split_out: the cuts' (x, leaf) pairs in forward
    # order.  r05: cuts after blocks 14, 6 and 2 leave 11.9 % of the live gradient bytes (layer3.0-2,
    # layer2, layer1, the stem) to the last segment.
    keep_split = False
    split_cuts = (14, 6, 2)
    split_out = None

    def split_params(self):
        """The trainable parameters whose gradients are final once the backward has reached layer3's
        output: layer4 and both heads."""
        return [p for m in (self.layer4, self.layer5, self.layer6) for p in m.parameters() if p.requires_grad]

    def valid_cuts(self):
        """split_cuts that lie inside this layer3 (a cut after block c needs blocks after it: 0 <= c <
        len(layer3) - 1), distinct, descending - the cuts _heads and split_segments use (the
        23-block defaults indexed past a shallower layer3)."""
        return sorted({int(c) for c in self.split_cuts if 0 <= int(c) < len(self.layer3) - 1}, reverse=True)

    def split_segments(self):
        """The trainable parameters each segment of the split backward finishes, in backward order:
        [layer4 + heads, layer3 blocks after the last cut, ..., after the first cut]; the last segment
        (layer3 up to the first cut, layer2, layer1, the stem) finishes the rest."""
        groups, hi = [self.split_params()], len(self.layer3)
        for c in self.valid_cuts():
            groups.append([p for b in range(c + 1, hi) for p in self.layer3[b].parameters() if p.requires_grad])
            hi = c + 1
        return groups

    def _cut(self, x):
        """A detached leaf standing in for x downstream: the backward of what reads it stops there
        (backward(inputs=[x]) would run x's own node, a BN), and its .grad seeds the next segment."""
        xd = x.detach().requires_grad_()
        if hasattr(x, "_msl_absmax"):
            xd._msl_absmax = x._msl_absmax  # the BN's absmax tag (same version counter)
        self.split_out.append((x, xd))
        return xd

    def _heads(self, x):
        """The trunk and both heads on (1,3,H,W) or an image batch (1,3,N,H,W): (layer6, layer5)
        low-resolution logits."""
        x = self.maxpool(ops.bn_act(self.bn1, self.conv1(x), relu=True))
        x = self.layer1(x)
        x = self.layer2(x)
        if self.keep_split:
            self.split_out = []
            cuts = set(self.valid_cuts())
            for i, blk in enumerate(self.layer3):
                x = blk(x)
                if i in cuts or i == len(self.layer3) - 1:
                    x = self._cut(x)
        else:
            x = self.layer3(x)
        x1 = self.layer5(x)
        x2 = self.layer4(x)
        x2 = self.layer6(x2)
        return x2, x1

    def forward(self, x):
        input_size = x.size()[2:]
        x2, x1 = self._heads(x)
        return ops.upsample_bilinear(x2, input_size), ops.upsample_bilinear(x1, input_size)

    def forward_pair(self, x_s, x_t):
        """forward(x_s), forward(x_t) as one image pair (not in the reference): every conv GEMM runs
        once over both images, while each image keeps its own bs=1 BatchNorm statistics (the
        running statistics are updated source first, then target, as two forwards would) and its
        own padding.  Returns [(x2_s, x1_s), (x2_t, x1_t)]."""
        if x_s.shape != x_t.shape:
            raise ValueError("forward_pair: source and target images must have the same size")
        input_size = x_s.size()[2:]
        x2, x1 = self._heads(ops.pair_join(x_s, x_t))
        return [(ops.upsample_bilinear(a, input_size), ops.upsample_bilinear(b, input_size))
                for a, b in zip(ops.pair_split(x2), ops.pair_split(x1))]

    def get_1x_lr_params_NOscale(self):
        """Backbone parameters, each yielded once per enclosing module (quirk Q2)."""
        b = [self.conv1, self.bn1, self.layer1, self.layer2, self.layer3, self.layer4]
        for i in range(len(b)):
            for j in b[i].modules():
                for k in j.parameters():
                    if k.requires_grad:
                        yield k

    def get_10x_lr_params(self):
        b = [self.layer5.parameters(), self.layer6.parameters()]
        for j in range(len(b)):
            for i in b[j]:
                yield i

    def optim_parameters(self, args):
        return [{'params': self.get_1x_lr_params_NOscale(), 'lr': args.lr},
                {'params': self.get_10x_lr_params(), 'lr': 10 * args.lr}]


def DeeplabMulti(num_classes=21, pretrained=True):
    """deeplab_multi.py:174-187.  `pretrained=True` needs the reference's ImageNet
    checkpoint (an absent /data path); load it with `load_pretrained`."""
    model = ResNetMulti(Bottleneck, [3, 4, 23, 3], num_classes)
    if pretrained:
        raise FileNotFoundError(
            "DeeplabMulti(pretrained=True): the reference's ImageNet init checkpoint "
            "(DeepLab_resnet_pretrained_init-f81d91e8.pth) is not available offline; pass "
            "pretrained=False or call load_pretrained(model, path)")
    return model


def load_pretrained(model, restore_from):
    """Load the reference's init checkpoint, skipping layer5 like deeplab_multi.py:177-186."""
    saved_state_dict = torch.load(restore_from, map_location="cpu", weights_only=True)
    new_params = model.state_dict().copy()
    for i in saved_state_dict:
        i_parts = i.split('.')
        if not i_parts[1] == 'layer5':
            new_params['.'.join(i_parts[1:])] = saved_state_dict[i]
    model.load_state_dict(new_params)
    return model
