"""Deterministic synthetic weights and inputs.

The datasets and checkpoints of the reference are not available offline, so
every run (bench, parity tests, golden generation) uses:
  - weights from a counter-based generator (splitmix64 + Box-Muller) keyed on
    (seed, parameter name), independent of torch's RNG and version, with the
    reference's init distributions (quirk Q10): conv weights N(0, 0.01), BN
    weight 1 / bias 0, ASPP biases U(+-1/sqrt(fan_in));
  - images: uint8 RGB U[0,255] -> BGR - IMG_MEAN, CHW fp32, the
    cityscapes_Dataset.py:14,245-251 preprocessing; seed 1000*rank + iter;
  - source labels: int64 uniform over {-1, ..., C-1}.
"""
import zlib

import numpy as np
import torch

IMG_MEAN = np.array((104.00698793, 116.66876762, 122.67891434), dtype=np.float32)

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _key(seed, name):
    return _splitmix64(np.uint64(seed) * np.uint64(0x100000001B3) ^ np.uint64(zlib.crc32(name.encode())))


def counter_uniform(seed, name, n):
    """n uniforms in (0, 1) as float64 (24-bit resolution)."""
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) + _key(seed, name)
        z = _splitmix64(ctr)
    return ((z >> np.uint64(40)).astype(np.float64) + 0.5) / float(1 << 24)


def counter_normal(seed, name, n, std=1.0):
    u1 = counter_uniform(seed, name + "#u1", n)
    u2 = counter_uniform(seed, name + "#u2", n)
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2) * std).astype(np.float32)


def init_weights(model, seed=12345):
    """Reference init (Q10) from the counter generator, in place, for any module tree with the
    DeeplabMulti parameter names (this package's model or the reference's)."""
    with torch.no_grad():
        for name, p in model.named_parameters():
            n = p.numel()
            if name.endswith("weight") and p.dim() == 4:
                v = counter_normal(seed, name, n, 0.01)
            elif name.endswith("bias") and "conv2d_list" in name:
                fan_in = int(np.prod(model.get_parameter(name.replace("bias", "weight")).shape[1:]))
                bound = 1.0 / np.sqrt(fan_in)
                v = ((counter_uniform(seed, name, n) * 2.0 - 1.0) * bound).astype(np.float32)
            elif name.endswith("weight"):  # BatchNorm gamma
                v = np.ones(n, np.float32)
            else:  # BatchNorm beta
                v = np.zeros(n, np.float32)
            p.copy_(torch.from_numpy(v).view_as(p))
        for name, b in model.named_buffers():
            if name.endswith("running_mean"):
                b.zero_()
            elif name.endswith("running_var"):
                b.fill_(1)
            elif name.endswith("num_batches_tracked"):
                b.zero_()
    return model


def synthetic_rgb(h, w, seed):
    """(h, w, 3) uint8 RGB, U[0, 255]."""
    return np.floor(counter_uniform(seed, "image", h * w * 3) * 256.0).astype(np.uint8).reshape(h, w, 3)


def synthetic_image(h, w, seed):
    """(1, 3, h, w) fp32: uint8 RGB -> BGR - IMG_MEAN, CHW (host form of utils/preprocess.image_transform)."""
    rgb = synthetic_rgb(h, w, seed)
    img = rgb.astype(np.float32)[:, :, ::-1] - IMG_MEAN
    return torch.from_numpy(img.transpose(2, 0, 1).copy()).unsqueeze(0)


def synthetic_labels(h, w, num_classes, seed):
    """(1, h, w) int64 uniform over {-1, ..., C-1}."""
    u = counter_uniform(seed, "label", h * w)
    lab = np.floor(u * (num_classes + 1)).astype(np.int64) - 1
    return torch.from_numpy(lab.reshape(1, h, w))


class SyntheticDomain:
    """A GTA5/Cityscapes-shaped dataset of `n` synthetic (image, label, id) items."""

    def __init__(self, h, w, num_classes, n, rank=0, offset=0):
        self.h, self.w, self.c, self.n, self.rank, self.offset = h, w, num_classes, n, rank, offset

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        seed = 1000 * self.rank + i + self.offset
        return synthetic_image(self.h, self.w, seed), synthetic_labels(self.h, self.w, self.c, seed), i
