"""Checkpoint format of the reference trainers (tools/train_source.py:662-704).

save:  {'epoch': current_epoch + 1, 'iteration': current_iter, 'state_dict': model weights,
        'optimizer': optimizer.state_dict(), 'best_MIou': best}            (:662-678)
load:  the weights (a 'module.' prefix - the reference saves its one-GPU nn.DataParallel
       wrapper's state_dict, train_source.py:133-136, 671-674 - is accepted and stripped), then,
       when the file holds an optimizer state, the optimizer and the epoch / iteration / best
       counters (:680-704).  A missing file is logged and skipped, as the reference does.

Files are read with torch.load(weights_only=True): a checkpoint is data, never code.
"""
import logging
import os

import torch

log = logging.getLogger(__name__)


def save_checkpoint(path, model, optimizer, epoch, iteration, best_MIou, module_prefix=False):
    """Write the reference's checkpoint dict to `path`.  module_prefix=True writes the keys as the
    reference's nn.DataParallel(model, device_ids=[0]) wrapper names them ('module.conv1.weight')."""
    sd = model.state_dict()
    if module_prefix:
        sd = {"module." + k: v for k, v in sd.items()}
    state = {"epoch": epoch, "iteration": iteration, "state_dict": sd,
             "optimizer": optimizer.state_dict(), "best_MIou": best_MIou}
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    torch.save(state, path)


def load_checkpoint(path, model, optimizer=None, map_location=None):
    """Restore `model` (and `optimizer`) from `path`.  Returns None when the file does not exist,
    {} when it holds weights only, else {'epoch', 'iteration', 'best_MIou'}."""
    try:
        ckpt = torch.load(path, map_location=map_location, weights_only=True)
    except OSError:
        log.info("No checkpoint exists from '%s'. Skipping...", path)
        return None
    sd = ckpt["state_dict"] if "state_dict" in ckpt else ckpt
    sd = {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}
    model.load_state_dict(sd)
    if "optimizer" not in ckpt:
        return {}
    if optimizer is not None:
        optimizer.load_state_dict(ckpt["optimizer"])
    return {"epoch": ckpt["epoch"], "iteration": ckpt["iteration"], "best_MIou": ckpt["best_MIou"]}
