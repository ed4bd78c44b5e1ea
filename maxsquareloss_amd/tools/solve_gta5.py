"""GTA5/SYNTHIA -> Cityscapes UDA trainer (tools/solve_gta5.py of the reference), MI355X path.

One iteration (solve_gta5.py:335-387), with the same method names:
    poly_lr_scheduler
    pred = model(x_src);  train_source(pred, y)   # CE(x2,y) [+ lambda_seg*CE(x1,y)]; backward
    pred = model(x_tgt);  train_target(pred)      # lambda_t*MaxSquare|IW-MaxSquare(x2)
                                                  # [+ lambda_seg*lambda_t*CE(x1, label_2)]; backward
    optimizer.step(); optimizer.zero_grad()
Gradients of the two backward passes accumulate; with WORLD_SIZE > 1 the
bucketed RCCL all-reduce is armed for the target backward and overlaps it.

With --pair (default) the two forwards run as one image pair (model.forward_pair:
every conv GEMM once over both images, each image with its own bs=1 BatchNorm
statistics) and the two losses share one backward pass; the gradients are the
same sums, added inside the weight-gradient GEMMs instead of by a second pass.

The losses run fused from the low-resolution logits (utils/loss.py), so the
two softmax tensors of the reference (:182-183) are never materialised.
Style-transfer augmentation (exp_tag source_aug/target_aug) and the
validation/eval path are out of scope.
"""
import argparse
import os

import numpy as np
import torch

from .. import ops
from ..utils.loss import IW_MaxSquareloss, MaxSquareloss, multi_level_guidance_ce
from ..utils.graph import GraphedStep
from ..utils.synthetic import SyntheticDomain
from .train_source import Trainer, add_train_args, init_args, str2bool


class UDATrainer(Trainer):
    def __init__(self, args, cuda=None, train_id="None", logger=None):
        super().__init__(args, cuda, train_id, logger)
        h, w = self.args.crop_size[1], self.args.crop_size[0]
        th, tw = self.args.target_crop_size[1], self.args.target_crop_size[0]
        self.source_dataloader = SyntheticDomain(h, w, self.args.num_classes, self.args.synthetic_images,
                                                 rank=self.rank)
        self.target_dataloader = SyntheticDomain(th, tw, self.args.num_classes, self.args.synthetic_images,
                                                 rank=self.rank, offset=500)
        self.ignore_index = -1
        mode = self.args.target_mode
        if mode == "maxsquare":
            self.target_loss = MaxSquareloss(ignore_index=-1, num_class=self.args.num_classes)
        elif mode == "IW_maxsquare":
            self.target_loss = IW_MaxSquareloss(ignore_index=-1, num_class=self.args.num_classes,
                                                ratio=self.args.IW_ratio)
        else:
            raise NotImplementedError(f"target_mode {mode!r} is outside the MI355X hot path "
                                      "(maxsquare, IW_maxsquare)")
        self.current_round = self.args.init_round
        self.round_num = self.args.round_num
        self.threshold = self.args.threshold
        self.iter_num = 1
        self._reset_meters()
        self.use_graph = bool(getattr(self.args, "graph", False))
        self._graphed = None
        self.overlap = bool(getattr(self.args, "overlap", True))
        self.pair = bool(getattr(self.args, "pair", True))
        self._side = None

    def _reset_meters(self):
        # zeroed in place once they exist: a captured step (utils/graph.py) adds into these tensors
        if getattr(self, "loss_seg_value", None) is not None:
            for t in (self.loss_seg_value, self.loss_seg_value_2, self.loss_target_value, self.loss_target_value_2):
                t.zero_()
            return
        z = lambda: torch.zeros((), device=self.device)  # noqa: E731
        self.loss_seg_value, self.loss_seg_value_2 = z(), z()
        self.loss_target_value, self.loss_target_value_2 = z(), z()

    # ---------------------------------------------------------------- the two halves
    def source_loss(self, pred, y):
        """The source objective of solve_gta5.py:220-235 (meters updated), without its backward."""
        if isinstance(pred, tuple):
            pred_2 = pred[1]
            pred = pred[0]
        y = torch.squeeze(y, 1)
        self.loss_val = self.loss(pred, y)
        loss_ = self.loss_val
        if self.args.multi:
            loss_2 = self.args.lambda_seg * self.loss(pred_2, y)
            loss_ = loss_ + loss_2
            self.loss_seg_value_2 += loss_2.detach() / self.iter_num
        self.loss_seg_value += self.loss_val.detach() / self.iter_num
        return loss_

    def target_loss_total(self, pred):
        """The target objective of solve_gta5.py:178-218 (maxsquare / IW_maxsquare target modes; meters
        updated), without its backward."""
        pred_2 = None
        if isinstance(pred, tuple):
            pred_2 = pred[1]
            pred = pred[0]
        self.loss_target = self.args.lambda_target * self.target_loss(pred)
        loss_target_ = self.loss_target
        if self.args.multi:
            self.loss_target_2 = (self.args.lambda_seg * self.args.lambda_target *
                                  multi_level_guidance_ce(pred, pred_2, self.threshold))
            loss_target_ = loss_target_ + self.loss_target_2
            self.loss_target_value_2 += self.loss_target_2.detach() / self.iter_num
        self.loss_target_value += self.loss_target.detach() / self.iter_num
        return loss_target_

    def train_source(self, pred, y):
        """solve_gta5.py:220-235."""
        self.source_loss(pred, y).backward()

    def train_target(self, pred):
        """solve_gta5.py:178-218 (maxsquare / IW_maxsquare target modes)."""
        loss_target_ = self.target_loss_total(pred)
        if self.reducer:
            self.reducer.prepare_for_backward()
        loss_target_.backward()

    def uda_step(self, x_s, y_s, x_t):
        """One iteration of the hot loop (solve_gta5.py:336-383), inputs already on the device.
        With use_graph, iterations after the first replay captured hipGraphs (utils/graph.py): one
        graph for the whole iteration on a single process; with a data-parallel reducer, a graph of
        the two forward/backward passes, the gradient all-reduce, then a graph of the SGD step."""
        self.poly_lr_scheduler(optimizer=self.optimizer, init_lr=self.args.lr)
        if self.use_graph:
            if self._graphed is None:
                if self.reducer is None:
                    self._graphed = GraphedStep(self, self._uda_body)
                elif self._split_ok():
                    # the backward captured in segments split at layer3's output and inside layer3 (the
                    # model's split_cuts): the gradients each segment finished are exchanged while the
                    # next segments replay.  Pair mode: the pair's one backward is cut; two-pass mode (r06,
                    # the reference's order): the source pass runs whole in the first segment (it only
                    # accumulates), and the target backward - the one that finishes the gradients - is cut
                    ends = list(np.cumsum([len(g) for g in self.model.split_segments()]))
                    self.reducer.set_breaks(ends)
                    red = self.reducer
                    between = [lambda n=ends[0]: red.reduce_early(n)]
                    between += [lambda n=n: red.reduce_more(n) for n in ends[1:]]
                    self._graphed = GraphedStep(
                        self, self._uda_grads, update=self._uda_update,
                        segments=[self._uda_grads_head] + [self._uda_grads_trunk] * len(ends),
                        between=between + [red.reduce_rest])
                else:
                    self._graphed = GraphedStep(self, self._uda_grads, exchange=self.reducer.reduce_all,
                                                update=self._uda_update)
            self._graphed(x_s, y_s, x_t)
        else:
            self._uda_body(x_s, y_s, x_t)
        self.current_iter += 1

    def _uda_grads(self, x_s, y_s, x_t):
        if self.pair and x_s.shape != x_t.shape and not getattr(self, "_pair_warned", False):
            #  --pair needs equal source and target crops; say so once instead of silently
            # running the two-pass step (bench.py's pair-mode step time applies to equal crops only)
            import warnings
            warnings.warn(f"--pair: source {tuple(x_s.shape)} and target {tuple(x_t.shape)} crops differ; "
                          "running the two-pass step", RuntimeWarning)
            self._pair_warned = True
        if self.pair and x_s.shape == x_t.shape:
            # one image pair through the network, one backward pass for both objectives
            pred_s, pred_t = self.model.forward_pair(x_s, x_t)
            loss_s = self.source_loss(pred_s, y_s)
            loss_t = self.target_loss_total(pred_t)
            if self.reducer:
                self.reducer.prepare_for_backward()
            torch.autograd.backward([loss_s, loss_t])
            ops.wgrad_join(self.device)
            return
        if not self.overlap:
            pred = self.model(x_s)
            self.train_source(pred, y_s)
            pred = self.model(x_t)
            self.train_target(pred)
            ops.wgrad_join(self.device)  # the side-stream weight gradients (ops.ASYNC_WGRAD) rejoin
            return
        # The target forward depends on neither the source backward nor its gradients (the weights
        # change only at the optimizer step; BN running statistics are updated by the forwards, in
        # the reference's order: source, then target), so it runs on a side stream concurrently with
        # the source backward.  The target backward (autograd runs it on the stream of its forward)
        # accumulates into the same gradient buffer: it waits for the source backward first, and the
        # main stream waits for it before the optimizer step.  Same kernels, same operands, same
        # order per buffer: the results are bit-identical to the sequential order.
        main = torch.cuda.current_stream(self.device)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
            # the ASPP parameters' AccumulateGrad nodes were made on the main stream: their
            # accumulation after the side-stream target backward syncs to it, as intended
            torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        side = self._side
        pred = self.model(x_s)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            pred_t = self.model(x_t)
        self.train_source(pred, y_s)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self.train_target(pred_t)
        main.wait_stream(side)
        ops.wgrad_join(self.device)  # the side-stream weight gradients (ops.ASYNC_WGRAD) rejoin

    def _split_ok(self):
        """Whether the parameters each backward segment finishes (model.split_segments) lead the flat
        gradient buffer (its backward order) in segment order, so the buckets launched after a segment
        hold final gradients only (False for a model without the split, or a cut list that leaves a
        segment empty)."""
        if not hasattr(self.model, "split_segments"):
            return False
        order = [id(p) for p in self.optimizer.grads.params]
        k = 0
        try:
            segments = self.model.split_segments()
        except (IndexError, AttributeError):
            return False
        for grp in segments:
            ids = {id(p) for p in grp}
            if not ids or set(order[k:k + len(ids)]) != ids:
                return False
            k += len(ids)
        return True

    def _uda_grads_head(self, x_s, y_s, x_t):
        """The pair's forward and the backward through the heads and layer4, stopping at layer3's
        output (the cuts kept for _uda_grads_trunk): the first segment of a captured data-parallel step
        (utils/graph.py).  The segments run exactly the kernels of _uda_grads, in its order.
        Two-pass mode (r06): the source forward and backward whole (they only accumulate), then the target
        forward with the cuts kept and its backward through the heads and layer4 - _uda_grads' order with
        the target backward cut (without the side-stream overlap of the target forward: one stream)."""
        m = self.model
        if not (self.pair and x_s.shape == x_t.shape):
            self.train_source(m(x_s), y_s)
            m.keep_split = True
            try:
                pred_t = m(x_t)
            finally:
                m.keep_split = False
            split, m.split_out = m.split_out, None
            loss_t = self.target_loss_total(pred_t)
            self.reducer.prepare_for_backward()
            loss_t.backward()  # ends at the heads' detached input (its .grad)
            ops.wgrad_join(self.device)
            self._split = split
            return
        m.keep_split = True
        try:
            pred_s, pred_t = m.forward_pair(x_s, x_t)
        finally:
            m.keep_split = False
        split, m.split_out = m.split_out, None
        loss_s = self.source_loss(pred_s, y_s)
        loss_t = self.target_loss_total(pred_t)
        self.reducer.prepare_for_backward()
        torch.autograd.backward([loss_s, loss_t])  # ends at the heads' detached input (its .grad)
        ops.wgrad_join(self.device)
        self._split = split

    def _uda_grads_trunk(self):
        """The next segment of the backward: from the last remaining cut back to the one before it (the
        last segment: through layer3's first blocks .. the stem)."""
        x, xd = self._split.pop()
        g, xd.grad = xd.grad, None
        torch.autograd.backward([x], [g])
        ops.wgrad_join(self.device)

    def _uda_update(self):
        self.optimizer.step()
        self.optimizer.zero_grad()
        self.packer.run()  # the next iteration's weight packs, batched (ops.PackBatch)

    def _uda_body(self, x_s, y_s, x_t):
        self._uda_grads(x_s, y_s, x_t)
        if self.reducer:
            self.reducer.finish()
        self._uda_update()

    # ---------------------------------------------------------------- loop
    def main(self):
        """solve_gta5.py:237-267: start from --pretrained_ckpt_file (the source-trained model); the
        counters restart unless --continue_training, which resumes from --checkpoint_dir; iter_max
        covers the rounds still to run."""
        if self.args.pretrained_ckpt_file is not None:
            path = self.args.pretrained_ckpt_file
            if os.path.isdir(path):
                path = self.args.checkpoint_dir
            self.load_checkpoint(path)
        if not self.args.continue_training:
            self.best_MIou = 0
            self.current_iter = 0
            self.current_epoch = 0
        else:
            self.load_checkpoint(self.args.checkpoint_dir)
        self.args.iter_max = self.current_iter + self.dataloader.num_iterations * \
            self.args.epoch_each_round * self.round_num
        self.optimizer.zero_grad()
        for _ in range(self.current_round, self.round_num):
            self.epoch_num = self.current_epoch + (self.current_round + 1) * self.args.epoch_each_round
            self.train()
            self.current_round += 1

    def train(self):
        for epoch in range(self.current_epoch, self.epoch_num):
            self.train_one_epoch(epoch)
            self.current_epoch += 1
        self.save_checkpoint(self.train_id + "final.pth")

    def train_one_epoch(self, epoch=0):
        self.model.eval() if self.args.freeze_bn else self.model.train()
        self.iter_num = self.dataloader.num_iterations
        self.Eval.reset()  # solve_gta5.py:294 (the UDA loop resets but never fills it)
        self._reset_meters()
        for i in range(self.iter_num):
            x_s, y_s, _ = self.source_dataloader[i % len(self.source_dataloader)]
            x_t, _, _ = self.target_dataloader[i % len(self.target_dataloader)]
            self.uda_step(x_s.to(self.device), y_s.to(self.device, dtype=torch.long), x_t.to(self.device))
        self.logger.info("epoch %d: source loss %.6f target loss %.6f", self.current_epoch,
                         float(self.loss_seg_value), float(self.loss_target_value))


def add_UDA_train_args(arg_parser):
    """solve_gta5.py:407-432."""
    a = arg_parser.add_argument
    a("--source_dataset", default="gta5", type=str, choices=["gta5", "synthia"])
    a("--source_split", default="train", type=str)
    a("--init_round", type=int, default=0)
    a("--round_num", type=int, default=1)
    a("--epoch_each_round", type=int, default=2)
    a("--target_mode", type=str, default="maxsquare",
      choices=["maxsquare", "IW_maxsquare", "entropy", "IW_entropy", "hard"])
    a("--lambda_target", type=float, default=1)
    a("--gamma", type=float, default=0)
    a("--IW_ratio", type=float, default=0.2)
    a("--threshold", type=float, default=0.95)
    a("--target_solo_epoch", type=int, default=0)
    a("--pair", type=str2bool, default=True,
      help="run the source and target images of an iteration as one image pair (per-image BatchNorm "
           "statistics, one backward pass; not in the reference, which runs two forward/backward passes)")
    a("--overlap", type=str2bool, default=True,
      help="with --pair False: run the target forward on a side stream concurrently with the source "
           "backward (same results; not in the reference, whose loop is sequential)")
    a("--graph", type=str2bool, default=False,
      help="replay each iteration after the first as one captured hipGraph (single process; not in the "
           "reference, whose loop is eager)")
    a("--dp_exchange", type=str2bool, default=False,
      help="run the data-parallel gradient exchange (RCCL process group + GradReducer) even at one rank, "
           "where the all-reduce is the identity: the multi-GPU code path on one GPU (not in the reference)")
    return arg_parser


def build_parser():
    return add_UDA_train_args(add_train_args(argparse.ArgumentParser()))


if __name__ == "__main__":
    args, train_id, logger = init_args(build_parser().parse_args())
    args.target_dataset = args.dataset
    train_id = str(args.source_dataset) + "2" + str(args.target_dataset) + "_" + args.target_mode
    UDATrainer(args=args, cuda=True, train_id=train_id, logger=logger).main()
