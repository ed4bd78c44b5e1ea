"""Segmentation metrics of the reference's `Eval` (utils/eval.py:13-118), confusion matrix on device.

The reference bins `num_class * gt + argmax(pred)` with np.bincount after copying the
prediction and label to the host every iteration (tools/train_source.py:280-283); here
`add_batch(label, pred)` takes the device tensors and runs `msl_confusion_accumulate`
(csrc/eval.hip: fused argmax + exact integer counts), and the matrix only crosses to the host
when a metric is read.  The metric definitions follow utils/eval.py: per-class accuracy / IoU /
precision with NaN for absent classes, nan-means over classes (`ignore_index` slicing),
16/13-class SYNTHIA subsets, and FWIoU as the frequency-weighted sum of the non-NaN IoUs.
"""
import numpy as np
import torch

from .. import hip

# utils/eval.py:9-11
synthia_set_16 = [0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 15, 17, 18]
synthia_set_13 = [0, 1, 2, 6, 7, 8, 10, 11, 12, 13, 15, 17, 18]
synthia_set_16_to_13 = [0, 1, 2, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15]


def _ratio(num, den):
    with np.errstate(divide="ignore", invalid="ignore"):
        return num / den


class Eval:
    def __init__(self, num_class):
        self.num_class = num_class
        self.ignore_index = None
        self.synthia = num_class == 16
        self._dev = None  # int64 [C*C] on the GPU, accumulated by add_batch
        self._host = np.zeros((num_class, num_class))

    # ------------------------------------------------------------------ accumulation
    def add_batch(self, gt_image, pre_image):
        """gt_image: int64 labels [N, H, W] (or [H, W]); pre_image: fp32 logits [N, C, H, W] on
        the GPU (argmax taken on device), same H, W.  Pixels with gt outside [0, C) are skipped."""
        if not (torch.is_tensor(pre_image) and pre_image.is_cuda and pre_image.dim() == 4):
            raise hip.MSLError("Eval.add_batch: expects device logits [N, C, H, W]")
        c = pre_image.size(1)
        if c != self.num_class:
            raise hip.MSLError(f"Eval.add_batch: {c} classes, Eval built for {self.num_class}")
        gt = gt_image.to(device=pre_image.device, dtype=torch.int64).reshape(pre_image.size(0), -1).contiguous()
        pred = pre_image.detach().float().contiguous()
        p = pred.size(2) * pred.size(3)
        if gt.size(1) != p:
            raise hip.MSLError("Eval.add_batch: label and prediction sizes differ")
        if self._dev is None or self._dev.device != pred.device:
            self._dev = torch.zeros(c * c, dtype=torch.int64, device=pred.device)
        lib = hip.load()
        for n in range(pred.size(0)):
            hip.check(lib.msl_confusion_accumulate(pred[n].data_ptr(), gt[n].data_ptr(), c, p,
                                                   self._dev.data_ptr(), None, hip.stream_ptr()),
                      "msl_confusion_accumulate")

    def reset(self):
        self._host = np.zeros((self.num_class,) * 2)
        if self._dev is not None:
            self._dev.zero_()

    @property
    def confusion_matrix(self):
        """[gt][pred] counts as float64 (the reference's dtype); syncs the device matrix."""
        m = self._host
        if self._dev is not None:
            m = m + self._dev.view(self.num_class, self.num_class).cpu().numpy().astype(np.float64)
        return m

    @confusion_matrix.setter
    def confusion_matrix(self, value):
        self._host = np.asarray(value, dtype=np.float64).copy()
        if self._dev is not None:
            self._dev.zero_()

    # ------------------------------------------------------------------ metrics
    def _reduce(self, per_class, out_16_13):
        if self.synthia:
            return np.nanmean(per_class[:self.ignore_index]), np.nanmean(per_class[synthia_set_16_to_13])
        if out_16_13:
            return np.nanmean(per_class[synthia_set_16]), np.nanmean(per_class[synthia_set_13])
        return np.nanmean(per_class[:self.ignore_index])

    def Pixel_Accuracy(self):
        m = self.confusion_matrix
        total = m.sum()
        if total == 0:
            print("Attention: pixel_total is zero!!!")
            return 0
        return np.trace(m) / total

    def _iou(self, m):
        d = np.diag(m)
        return _ratio(d, m.sum(axis=1) + m.sum(axis=0) - d)

    def Mean_Pixel_Accuracy(self, out_16_13=False):
        m = self.confusion_matrix
        return self._reduce(_ratio(np.diag(m), m.sum(axis=1)), out_16_13)

    def Mean_Intersection_over_Union(self, out_16_13=False):
        return self._reduce(self._iou(self.confusion_matrix), out_16_13)

    def Mean_Precision(self, out_16_13=False):
        m = self.confusion_matrix
        return self._reduce(_ratio(np.diag(m), m.sum(axis=0)), out_16_13)

    def Frequency_Weighted_Intersection_over_Union(self, out_16_13=False):
        m = self.confusion_matrix
        fw = m.sum(axis=1) * self._iou(m)
        total = m.sum()

        def part(v):
            return float(v[~np.isnan(v)].sum()) / total

        if self.synthia:
            return part(fw), part(fw[synthia_set_16_to_13])
        if out_16_13:
            return part(fw[synthia_set_16]), part(fw[synthia_set_13])
        return part(fw)
