"""Loss modules with the reference's signatures (utils/loss.py) on HIP kernels.

`MaxSquareloss.forward(pred, prob)` / `IW_MaxSquareloss.forward(pred, prob, label)`
behave exactly like loss.py:69-119 when given an explicit probability tensor.
Passing `prob=None` selects the fused path: the loss is computed straight
from the logits behind `pred` (the low-res ASPP output when `pred` came from
this package's DeeplabMulti), with softmax, upsampling and the loss fused into
one forward and one backward kernel pair.
"""
import torch.nn as nn

from .. import ops


def _fused_source(pred):
    low = ops.low_of(pred)
    if low is None:  # a plain hi-res logits tensor: identity interpolation
        low = pred
    return low, tuple(pred.shape[2:])


class MaxSquareloss(nn.Module):
    """loss = -sum(p^2) / (2*N*C*H*W) (loss.py:104-119; the `prob != -1` mask is a no-op, Q5)."""

    def __init__(self, ignore_index=-1, num_class=19):
        super().__init__()
        self.ignore_index = ignore_index
        self.num_class = num_class

    def forward(self, pred, prob=None):
        if prob is None:
            low, hw = _fused_source(pred)
            return ops.maxsquare_up(low, hw)
        return ops.maxsquare_prob(prob)


class IW_MaxSquareloss(nn.Module):
    """Image-wise class-balanced MaxSquare (loss.py:69-102).

    hist = per-class pixel count of argmax(prob) (or of `label`), weights
    w_c = 1/max(hist_c^ratio * (sum hist)^(1-ratio), 1),
    loss = -sum_px w[argmax] * sum_c p^2 / (N*C).  The last histogram and
    weights are kept on the module (`last_hist`, `last_weights`, device tensors).
    """

    def __init__(self, ignore_index=-1, num_class=19, ratio=0.2):
        super().__init__()
        self.ignore_index = ignore_index
        self.num_class = num_class
        self.ratio = ratio
        self.last_hist = None
        self.last_weights = None

    def forward(self, pred, prob=None, label=None):
        if prob is None:
            if label is not None:
                raise NotImplementedError("fused IW_MaxSquareloss counts argmax(prob); pass prob with label")
            low, hw = _fused_source(pred)
            loss, hist, w = ops.iw_maxsquare_up(low, hw, self.ratio)
        else:
            loss, hist, w = ops.iw_maxsquare_prob(prob, label, self.ratio)
        self.last_hist, self.last_weights = hist, w
        return loss


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss(ignore_index=-1) on (1,C,H,W) logits and (1,H,W) int64 labels
    (train_source.py:128).  Mean over non-ignored pixels; nan when none (quirk Q8)."""

    def __init__(self, weight=None, ignore_index=-1):
        super().__init__()
        if weight is not None or ignore_index != -1:
            raise NotImplementedError("only weight=None, ignore_index=-1 (the reference's setting)")
        self.ignore_index = ignore_index

    def forward(self, pred, target):
        low, hw = _fused_source(pred)
        return ops.ce_up(low, target.reshape(-1), hw)


def multi_level_guidance_ce(pred, pred_2, threshold):
    """CE(pred_2, label_2) with label_2 = (max P > thr | max P2 > thr) ? argmax((P+P2)/2) : -1,
    P = softmax(pred), P2 = softmax(pred_2)  (solve_gta5.py:206-213).  Gradient flows to pred_2 only."""
    low1, hw = _fused_source(pred_2)
    low2, hw2 = _fused_source(pred)
    if hw != hw2:
        raise ValueError("both heads must be upsampled to the same size")
    return ops.multi_ce_up(low1, low2.detach(), hw, threshold)
