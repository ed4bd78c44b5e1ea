"""Source-only trainer (tools/train_source.py of the reference), MI355X path.

Same flags (add_train_args, :726-829), same `init_args` parsing (:832-883),
same `Trainer` surface (`train()`, `train_one_epoch()`, `poly_lr_scheduler`,
`save_checkpoint` / `load_checkpoint` dict format).  Differences, all outside
the training arithmetic:
  - data is synthetic (the GTA5/Cityscapes/SYNTHIA files are not available):
    utils/synthetic.py reproduces the reference preprocessing on generated
    uint8 images; the dataset flags are accepted and only set shapes/classes;
  - one process per GPU: under torchrun (WORLD_SIZE > 1) the model is
    replicated and gradients are all-reduced over RCCL (utils/dist.py);
  - loss scalars stay on the device (no per-iteration .cpu().item() sync);
    the NaN check of :277-278 runs on the accumulated value at epoch end;
  - the per-iteration argmax + Eval confusion matrix (:280-283) run on the
    device (utils/eval.py, csrc/eval.hip), no D2H copy of the prediction;
    tensorboard logging is out of scope.
"""
import argparse
import logging
import os
import random

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..utils.dist import GradReducer
from ..utils.checkpoint import load_checkpoint, save_checkpoint
from ..utils.eval import Eval
from ..utils.loss import CrossEntropyLoss
from ..utils.optim import SGD
from ..utils.synthetic import SyntheticDomain, init_weights
from ..utils.train_helper import get_model

ITER_MAX = 5000


def str2bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true", "t", "y", "1"):
        return True
    if v.lower() in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError("Unsupported value encountered.")


def dist_env():
    """(rank, world, local_rank) from torchrun's environment, (0, 1, 0) otherwise."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def _free_port():
    """A TCP port free on 127.0.0.1 now (the one-rank group's rendezvous)."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


class Trainer:
    def __init__(self, args, cuda=None, train_id="None", logger=None):
        self.args = args
        self.rank, self.world, self.local_rank = dist_env()
        self.cuda = bool(cuda) and torch.cuda.is_available()
        if not self.cuda:
            raise RuntimeError("the MI355X trainer needs a GPU (no CPU fallback)")
        torch.cuda.set_device(self.local_rank)
        self.device = torch.device("cuda", self.local_rank)
        dp = self.world > 1 or bool(getattr(args, "dp_exchange", False))
        if dp and not dist.is_initialized():
            if self.world == 1:
                # --dp_exchange on a plain single-process launch: a one-rank group on this host
                # instead of env:// failing on the variables torchrun would have set
                for k, v in (("MASTER_ADDR", "127.0.0.1"), ("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
                    os.environ.setdefault(k, v)
                os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("nccl", device_id=self.device)
        self.train_id = train_id
        self.logger = logger or logging.getLogger(__name__)
        self.current_MIoU = self.best_MIou = self.best_FWIou = self.best_source_MIou = 0
        self.current_epoch = 0
        self.current_iter = 0

        self.loss = CrossEntropyLoss(weight=None, ignore_index=-1)
        self.Eval = Eval(self.args.num_classes)  # train_source.py:93, confusion matrix on device
        ops.set_conv_math(getattr(self.args, "conv_math", "fp32"))
        if getattr(self.args, "f32_form", None):
            ops.set_f32_form(self.args.f32_form)

        self.model, self.params = get_model(self.args)
        init_weights(self.model, seed=self.args.seed)
        self.model.to(self.device)

        if self.args.optim != "SGD":
            raise NotImplementedError("only --optim SGD (the reference default) is on the MI355X path")
        self.optimizer = SGD(lr=self.args.lr, params=self.params, momentum=self.args.momentum,
                             weight_decay=self.args.weight_decay)
        self.reducer = GradReducer(self.optimizer, always=self.world == 1) if dp else None
        self.packer = ops.PackBatch(self.model)  # every weight pack of a step in two launches

        h, w = self.args.crop_size[1], self.args.crop_size[0]
        self.dataloader = SyntheticDomain(h, w, self.args.num_classes, self.args.synthetic_images,
                                          rank=self.rank)
        self.dataloader.num_iterations = min(len(self.dataloader), ITER_MAX)
        iters = self.args.iter_stop if self.args.iter_stop is not None else self.args.iter_max
        self.epoch_num = -(-iters // self.dataloader.num_iterations)

    # ------------------------------------------------------------------ loop
    def main(self):
        """train_source.py:161-173: restore --checkpoint_dir whenever it is given; the counters
        restart unless --continue_training."""
        if self.args.checkpoint_dir is not None:
            self.load_checkpoint(self.args.checkpoint_dir)
        if not self.args.continue_training:
            self.current_epoch = 0
        self.train()

    def train(self):
        for epoch in range(self.current_epoch, self.epoch_num):
            self.train_one_epoch(epoch)
            self.current_epoch += 1
        self.save_checkpoint(self.train_id + "final.pth")

    def train_one_epoch(self, epoch=None):
        # train_source.py:225-229: --freeze_bn keeps BN on its running statistics
        self.model.eval() if self.args.freeze_bn else self.model.train()
        iter_num = self.dataloader.num_iterations
        loss_sum = torch.zeros((), device=self.device)
        self.Eval.reset()
        for i in range(iter_num):
            x, y, _ = self.dataloader[i]
            self.poly_lr_scheduler(self.optimizer, init_lr=self.args.lr, iter=self.current_iter,
                                   max_iter=self.args.iter_max, power=self.args.poly_power)
            x = x.to(self.device, non_blocking=True)
            y = y.to(self.device, dtype=torch.long, non_blocking=True)
            loss_sum += self.source_step(x, y).detach()
            self.Eval.add_batch(y, self.last_pred)  # train_source.py:280-283, argmax on device
            self.current_iter += 1
        mean = float(loss_sum) / max(iter_num, 1)
        if np.isnan(mean):
            raise ValueError("Loss is nan during training...")
        self.logger.info("The average loss of train epoch-%d-:%f", self.current_epoch, mean)
        self.logger.info("Epoch:%d, PA:%.3f, MPA:%.3f, MIoU:%.3f, FWIoU:%.3f", self.current_epoch,
                         self.Eval.Pixel_Accuracy(), self.Eval.Mean_Pixel_Accuracy() if not self.Eval.synthia
                         else self.Eval.Mean_Pixel_Accuracy()[0], self.Eval.Mean_Intersection_over_Union()
                         if not self.Eval.synthia else self.Eval.Mean_Intersection_over_Union()[0],
                         self.Eval.Frequency_Weighted_Intersection_over_Union() if not self.Eval.synthia
                         else self.Eval.Frequency_Weighted_Intersection_over_Union()[0])

    def source_step(self, x, y):
        """train_source.py:248-264: CE(x2,y) + lambda_seg*CE(x1,y); zero_grad; backward; step."""
        pred = self.model(x)
        pred, pred_2 = pred if isinstance(pred, tuple) else (pred, None)
        self.last_pred = pred.detach()
        cur_loss = self.loss(pred, y)
        if self.args.multi:
            cur_loss = cur_loss + self.args.lambda_seg * self.loss(pred_2, y)
        self.optimizer.zero_grad()
        if self.reducer:
            self.reducer.prepare_for_backward()
        cur_loss.backward()
        if self.reducer:
            self.reducer.finish()
        self.optimizer.step()
        self.packer.run()
        return cur_loss

    # ------------------------------------------------------------------ checkpoints
    def save_checkpoint(self, filename=None):
        """train_source.py:662-678 (utils/checkpoint.py)."""
        if self.rank != 0 or not self.args.save_dir:
            return
        save_checkpoint(os.path.join(self.args.save_dir, filename), self.model, self.optimizer,
                        self.current_epoch + 1, self.current_iter, self.best_MIou)

    def load_checkpoint(self, filename):
        """train_source.py:680-704 (utils/checkpoint.py): weights, then optimizer + counters."""
        got = load_checkpoint(filename, self.model, self.optimizer, map_location=self.device)
        if got:
            self.current_epoch = got["epoch"]
            self.current_iter = got["iteration"]
            self.best_MIou = got["best_MIou"]

    # ------------------------------------------------------------------ LR
    def poly_lr_scheduler(self, optimizer, init_lr=None, iter=None, max_iter=None, power=None):
        """train_source.py:706-717."""
        init_lr = self.args.lr if init_lr is None else init_lr
        iter = self.current_iter if iter is None else iter
        max_iter = self.args.iter_max if max_iter is None else max_iter
        power = self.args.poly_power if power is None else power
        new_lr = init_lr * (1 - float(iter) / max_iter) ** power
        optimizer.param_groups[0]["lr"] = new_lr
        if len(optimizer.param_groups) == 2:
            optimizer.param_groups[1]["lr"] = 10 * new_lr
        if len(optimizer.param_groups) == 3:
            optimizer.param_groups[2]["lr"] = new_lr


def add_train_args(arg_parser):
    """The reference's flags (train_source.py:726-829) plus --synthetic_images."""
    a = arg_parser.add_argument
    a("--data_root_path", type=str, default=None)
    a("--list_path", type=str, default=None)
    a("--checkpoint_dir", default=None)
    a("--save_dir", default="./log/train")
    a("--backbone", default="deeplabv2_multi")
    a("--bn_momentum", type=float, default=0.1)
    a("--imagenet_pretrained", type=str2bool, default=True)
    a("--pretrained_ckpt_file", type=str, default=None)
    a("--continue_training", type=str2bool, default=False)
    a("--show_num_images", type=int, default=2)
    a("--seed", default=12345, type=int)
    a("--gpu", type=str, default="0")
    a("--batch_size", default=1, type=int)
    a("--exp_tag", type=str, default="test")
    a("--dataset", default="Cityscapes", type=str)
    a("--base_size", default="1856,928", type=str)
    a("--crop_size", default="928,464", type=str)
    a("--target_base_size", default="1856,928", type=str)
    a("--target_crop_size", default="928,464", type=str)
    a("--seg_size", default=(1280, 640))
    a("--num_classes", default=19, type=int)
    a("--data_loader_workers", default=0, type=int)
    a("--pin_memory", default=2, type=int)
    a("--split", type=str, default="train")
    a("--random_mirror", default=True, type=str2bool)
    a("--random_crop", default=False, type=str2bool)
    a("--resize", default=True, type=str2bool)
    a("--gaussian_blur", default=False, type=str2bool)
    a("--numpy_transform", default=True, type=str2bool)
    a("--freeze_bn", type=str2bool, default=False)
    a("--optim", default="SGD", type=str)
    a("--momentum", type=float, default=0.9)
    a("--weight_decay", type=float, default=5e-4)
    a("--lr", type=float, default=2.5e-4)
    a("--iter_max", type=int, default=200000)
    a("--iter_stop", type=int, default=80000)
    a("--poly_power", type=float, default=0.9)
    a("--rectification", type=bool, default=False)
    a("--crop_trans", type=bool, default=False)
    a("--client", type=bool, default=False)
    a("--DA", type=bool, default=False)
    a("--multi", default=True, type=str2bool)
    a("--lambda_seg", type=float, default=0.1)
    a("--synthetic_images", type=int, default=4, help="synthetic items per domain (no datasets offline)")
    a("--conv_math", default="fp32", choices=["fp32", "fp16", "bf16"],
      help="conv MFMA precision (not in the reference, which is fp32): fp16 = BASELINE config 5's "
           "fp16 MFMA path (scaled fp16 operands, fp32 sums), bf16 = bf16 products, fp32 sums; BN, "
           "losses, SGD stay fp32")
    a("--f32_form", default=None, choices=["mfma_f32", "bf16x6", "f16x3"],
      help="matrix-core form of the fp32 convs; default f16x3 (the library's default): each operand "
           "scaled by a power of two and split into two fp16 terms, three v_mfma_f32_32x32x16_f16 "
           "products with fp32 sums (fp32-accurate); mfma_f32 = v_mfma_f32_32x32x2_f32 (exact fp32 "
           "FMA chains); bf16x6 = three-way bf16 split, six products, fp32-accurate")
    return arg_parser


def init_args(args):
    """train_source.py:832-883 without the log-file handler."""
    train_id = args.exp_tag

    def pair(s):
        parts = str(s).split(",")
        return int(parts[0]) if len(parts) == 1 else (int(parts[0]), int(parts[1]))

    args.crop_size, args.base_size = pair(args.crop_size), pair(args.base_size)
    args.target_crop_size, args.target_base_size = pair(args.target_crop_size), pair(args.target_base_size)
    if isinstance(args.crop_size, int):
        args.crop_size = (args.crop_size, args.crop_size)
    if isinstance(args.target_crop_size, int):
        args.target_crop_size = (args.target_crop_size, args.target_crop_size)
    args.class_16 = args.num_classes == 16
    args.class_13 = args.num_classes == 13
    logger = logging.getLogger()
    logger.setLevel(logging.INFO)
    random.seed(args.seed)
    np.random.seed(args.seed)
    torch.random.manual_seed(args.seed)
    return args, train_id, logger


if __name__ == "__main__":
    parser = add_train_args(argparse.ArgumentParser())
    args, train_id, logger = init_args(parser.parse_args())
    Trainer(args=args, cuda=True, train_id=train_id, logger=logger).main()
