"""Device-side input pipeline: the reference loaders' final transforms as HIP kernels (§8f row 4).

The reference converts every image and label on the host in numpy
(datasets/cityscapes_Dataset.py:245-264) and ships fp32 CHW images and fp32
labels; here the uint8 image / id map is copied as is (4x / 8x fewer PCIe
bytes) and converted on the GPU (csrc/preprocess.hip), bit-exact:
  image_transform:  RGB uint8 HWC -> BGR - IMG_MEAN fp32 (1,3,H,W)   (_img_transform, :245-251)
  label_transform:  ids uint8 HW  -> trainIds int64 (1,H,W), -1 = ignore
                    (id2trainId + the 16 / 13-class remaps, :124-155, 260-264)
both with the optional horizontal mirror of the random_mirror augmentation.
"""
import numpy as np
import torch

from .. import hip
from .synthetic import IMG_MEAN

# id -> trainId tables of the three loaders (values not listed map to the ignore label -1)
CITYSCAPES_ID_TO_TRAINID = {7: 0, 8: 1, 11: 2, 12: 3, 13: 4, 17: 5, 19: 6, 20: 7, 21: 8, 22: 9, 23: 10,
                            24: 11, 25: 12, 26: 13, 27: 14, 28: 15, 31: 16, 32: 17, 33: 18}  # cityscapes_Dataset.py:124-130
GTA5_ID_TO_TRAINID = dict(CITYSCAPES_ID_TO_TRAINID)  # gta5_Dataset.py:73-75 (the same 19 labelled ids)
SYNTHIA_ID_TO_TRAINID = {1: 10, 2: 2, 3: 0, 4: 1, 5: 4, 6: 8, 7: 5, 8: 13, 9: 7, 10: 11, 11: 18, 12: 17,
                         15: 6, 16: 9, 17: 12, 18: 14, 19: 15, 20: 16, 21: 3}  # synthia_Dataset.py:56-58
SET_16 = [0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 15, 17, 18]  # cityscapes_Dataset.py:132
SET_13 = [0, 1, 2, 6, 7, 8, 10, 11, 12, 13, 15, 17, 18]            # cityscapes_Dataset.py:136


def build_lut(dataset, class_16=False, class_13=False):
    """int32[256]: uint8 label id -> the trainId the reference's id2trainId produces."""
    table = {"cityscapes": CITYSCAPES_ID_TO_TRAINID, "gta5": GTA5_ID_TO_TRAINID,
             "synthia": SYNTHIA_ID_TO_TRAINID}[dataset.lower()]
    lut = np.full(256, -1, np.int32)
    for k, v in table.items():
        lut[k] = v
    for on, sub in ((class_16, SET_16), (class_13, SET_13)):
        if on:
            remap = {t: i for i, t in enumerate(sub)}
            lut = np.array([remap.get(int(t), -1) for t in lut], np.int32)
    return lut


def image_transform(rgb, mirror=False, mean=IMG_MEAN):
    """rgb: uint8 (H, W, 3) on the GPU -> (1, 3, H, W) fp32 BGR - mean."""
    if not rgb.is_cuda or rgb.dtype != torch.uint8 or rgb.dim() != 3 or rgb.size(2) != 3:
        raise hip.MSLError(f"image_transform: expected a CUDA uint8 (H, W, 3) tensor, got {tuple(rgb.shape)} "
                           f"{rgb.dtype} {rgb.device}")
    rgb = rgb.contiguous()
    h, w = rgb.shape[:2]
    out = torch.empty((1, 3, h, w), dtype=torch.float32, device=rgb.device)
    m = [float(np.float32(v)) for v in mean]
    hip.check(hip.load().msl_image_transform(rgb.data_ptr(), h, w, int(bool(mirror)), m[0], m[1], m[2],
                                             out.data_ptr(), hip.stream_ptr()), "msl_image_transform")
    return out


_LUTS = {}


def label_transform(ids, lut, mirror=False):
    """ids: uint8 (H, W) on the GPU, lut: int32[256] (build_lut) -> (1, H, W) int64 trainIds."""
    if not ids.is_cuda or ids.dtype != torch.uint8 or ids.dim() != 2:
        raise hip.MSLError(f"label_transform: expected a CUDA uint8 (H, W) tensor, got {tuple(ids.shape)} "
                           f"{ids.dtype} {ids.device}")
    ids = ids.contiguous()
    key = (ids.device.index, np.asarray(lut, np.int32).tobytes())
    dlut = _LUTS.get(key)
    if dlut is None:
        dlut = torch.from_numpy(np.asarray(lut, np.int32).copy()).to(ids.device)
        if dlut.numel() != 256:
            raise hip.MSLError("label_transform: the table must have 256 entries")
        _LUTS[key] = dlut
    h, w = ids.shape
    out = torch.empty((1, h, w), dtype=torch.int64, device=ids.device)
    hip.check(hip.load().msl_label_transform(ids.data_ptr(), h, w, int(bool(mirror)), dlut.data_ptr(),
                                             out.data_ptr(), hip.stream_ptr()), "msl_label_transform")
    return out
