"""Evaluation path: utils/eval.py's metrics vs the oracle restatement of the
reference's utils/eval.py:25-115 (CPU), and the device argmax + confusion kernel vs numpy
argmax/bincount (GPU)."""
import numpy as np
import pytest
import torch

from maxsquareloss_amd import hip
from maxsquareloss_amd.utils.eval import Eval
from oracle import msl_oracle as orc


def _close(a, b):
    a, b = np.atleast_1d(np.asarray(a, dtype=np.float64)), np.atleast_1d(np.asarray(b, dtype=np.float64))
    return a.shape == b.shape and np.allclose(a, b, rtol=1e-12, atol=0, equal_nan=True)


@pytest.mark.parametrize("num_class,out_16_13,empty", [(19, False, False), (19, True, False), (19, False, True),
                                                       (16, False, False), (16, False, True), (13, False, False)])
def test_metrics_match_reference_formulas(num_class, out_16_13, empty):
    rng = np.random.default_rng(num_class + 3 * out_16_13 + 7 * empty)
    cm = rng.integers(0, 5000, size=(num_class, num_class)).astype(np.float64)
    if empty:  # a class never in the label and never predicted: NaN entries, nan-means
        cm[3, :] = 0
        cm[:, 3] = 0
        cm[5, :] = 0
    ev = Eval(num_class)
    ev.confusion_matrix = cm
    ref = orc.eval_metrics(cm, out_16_13)
    assert _close(ev.Pixel_Accuracy(), ref["PA"])
    assert _close(ev.Mean_Pixel_Accuracy(out_16_13), ref["MPA"])
    assert _close(ev.Mean_Intersection_over_Union(out_16_13), ref["MIoU"])
    assert _close(ev.Frequency_Weighted_Intersection_over_Union(out_16_13), ref["FWIoU"])
    assert _close(ev.Mean_Precision(out_16_13), ref["Precision"])


def test_zero_matrix_pixel_accuracy():
    ev = Eval(19)
    assert ev.Pixel_Accuracy() == 0


def test_add_batch_has_no_cpu_path():
    ev = Eval(19)
    with pytest.raises(hip.MSLError):
        ev.add_batch(torch.zeros(1, 4, 4, dtype=torch.long), torch.zeros(1, 19, 4, 4))


@pytest.mark.gpu
@pytest.mark.parametrize("c,h,w", [(19, 512, 1024), (16, 65, 129), (13, 7, 9)])
def test_device_confusion_matches_bincount(c, h, w):
    g = torch.Generator().manual_seed(c * h)
    # quantised logits: many exact ties (lowest index must win), a few NaNs, ignored labels
    pred = (torch.randint(0, 6, (2, c, h, w), generator=g).float() * 0.5)
    pred[0, 4, 0, :3] = float("nan")
    pred[1, 0, 1, :2] = float("nan")
    label = torch.randint(-1, c + 1, (2, h, w), generator=g)
    label[0, 0, :5] = 255
    ev = Eval(c)
    ev.add_batch(label.cuda(), pred.cuda())
    ref = sum(orc.confusion(label[n].numpy(), pred[n].numpy(), c)[0] for n in range(2))
    assert np.array_equal(ev.confusion_matrix, ref.astype(np.float64))
    # per-pixel argmax output of the C-ABI entry point
    lib = hip.load()
    arg = torch.empty(h * w, dtype=torch.int32, device="cuda")
    cm = torch.zeros(c * c, dtype=torch.int64, device="cuda")
    pc, lc = pred[0].cuda().contiguous(), label[0].cuda().contiguous()
    hip.check(lib.msl_confusion_accumulate(pc.data_ptr(), lc.data_ptr(), c, h * w, cm.data_ptr(), arg.data_ptr(),
                                           hip.stream_ptr()), "msl_confusion_accumulate")
    torch.cuda.synchronize()
    ref0, arg0 = orc.confusion(label[0].numpy(), pred[0].numpy(), c)
    assert np.array_equal(arg.cpu().numpy(), arg0)
    assert np.array_equal(cm.view(c, c).cpu().numpy(), ref0)
    ev.reset()
    assert ev.confusion_matrix.sum() == 0


@pytest.mark.gpu
def test_source_epoch_fills_eval_on_device():
    """Trainer.train_one_epoch (train_source.py:241-283): every iteration's argmax lands in the
    device confusion matrix; its total is the epoch's count of labelled pixels."""
    import argparse
    from maxsquareloss_amd.tools.train_source import Trainer, add_train_args, init_args
    argv = ["--crop_size", "256,128", "--target_crop_size", "256,128", "--imagenet_pretrained", "False",
            "--save_dir", "", "--synthetic_images", "2", "--iter_max", "200000"]
    args, _, _ = init_args(add_train_args(argparse.ArgumentParser()).parse_args(argv))
    tr = Trainer(args, cuda=True)
    tr.train_one_epoch()
    torch.cuda.synchronize()
    c = args.num_classes
    n = sum(int(((y >= 0) & (y < c)).sum()) for y in (tr.dataloader[i][1] for i in range(tr.dataloader.num_iterations)))
    cm = tr.Eval.confusion_matrix
    assert cm.shape == (c, c) and cm.sum() == n
    assert 0.0 <= tr.Eval.Pixel_Accuracy() <= 1.0 and np.isfinite(tr.Eval.Mean_Intersection_over_Union())
