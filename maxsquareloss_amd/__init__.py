"""MI355X-native DeepLabv2/ResNet-101 MaxSquare domain-adaptation training step.

Mirrors the reference's layout for the hot path only:
  graphs/models/deeplab_multi.py  - DeeplabMulti with HIP dilated convs / ASPP / upsample
  utils/loss.py                   - MaxSquareloss, IW_MaxSquareloss, CrossEntropyLoss (fused HIP)
  utils/optim.py                  - SGD with the reference's duplicated-parameter semantics
  utils/dist.py                   - bucketed RCCL all-reduce overlapped with the backward
  tools/solve_gta5.py, tools/train_source.py - the trainer entry points
Native code: csrc/*.hip -> _lib/libmsl_hip.so (C-ABI in include/msl_hip.h).
"""
__version__ = "0.1.0"
