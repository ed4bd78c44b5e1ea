"""The captured step (utils/graph.py) against the eager step, and the step's run-to-run bit identity
(GPU only).

Every kernel of the training step is a HIP kernel with a fixed summation order (no library GEMM or
conv, no float atomics: the stem, maxpool and the stride-2 1x1 convs run on csrc/stem.hip + the
pointwise GEMMs since r03), so two trainers from the same counter-generated init fed the same images
must agree bit for bit - eagerly, and when one of them replays a captured hipGraph (the graph
replays the poly learning rate from device memory and repacks the weights the previous replay
updated).  Between replays the test edits weights eagerly in both trainers (an in-place scale of
several conv weights): the graphed trainer must notice and repack before its replay reads the packs
(GraphedStep.versions), or its losses would differ.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from maxsquareloss_amd.tools.solve_gta5 import UDATrainer, build_parser  # noqa: E402
from maxsquareloss_amd.tools.train_source import init_args  # noqa: E402
from maxsquareloss_amd.utils.synthetic import synthetic_image, synthetic_labels  # noqa: E402

H, W = 256, 512


def _trainer(graph, mode="IW_maxsquare", multi="True"):
    argv = ["--crop_size", f"{W},{H}", "--target_crop_size", f"{W},{H}", "--imagenet_pretrained", "False",
            "--save_dir", "", "--target_mode", mode, "--multi", multi, "--lambda_target", "0.09",
            "--iter_max", "1000", "--graph", str(graph)]
    args, _, _ = init_args(build_parser().parse_args(argv))
    tr = UDATrainer(args, cuda=True)
    tr.optimizer.zero_grad()
    return tr


def _inputs(it):
    return (synthetic_image(H, W, 40 + it).cuda(), synthetic_labels(H, W, 19, 40 + it).cuda(),
            synthetic_image(H, W, 540 + it).cuda())


def _state(tr):
    return ([p.detach().clone() for p in tr.model.parameters()] + [b.detach().clone() for b in tr.model.buffers()] +
            [tr.optimizer.state[p]["momentum_buffer"].detach().clone() for p in tr.optimizer._uniq
             if p in tr.optimizer.state])


def _first_diff(a, b, names):
    for i, (x, y) in enumerate(zip(a, b)):
        if not torch.equal(x, y):
            return names[i] if i < len(names) else i
    return None


def test_eager_step_is_bit_reproducible():
    """Two eager trainers, same init and images, three UDA iterations: every loss, the IW histogram,
    every parameter, BN buffer and momentum buffer identical bit for bit."""
    a, b = _trainer(False), _trainer(False)
    names = [n for n, _ in a.model.named_parameters()] + [n for n, _ in a.model.named_buffers()]
    for it in range(3):
        for tr in (a, b):
            tr.uda_step(*_inputs(it))
        torch.cuda.synchronize()
        for name in ("loss_val", "loss_target", "loss_target_2"):
            assert getattr(a, name).item() == getattr(b, name).item(), (it, name)
        assert torch.equal(a.target_loss.last_hist, b.target_loss.last_hist), it
        assert _first_diff(_state(a), _state(b), names) is None, (it, _first_diff(_state(a), _state(b), names))


def test_graph_replay_matches_eager_bit_for_bit():
    eager, graphed = _trainer(False), _trainer(True)
    assert graphed.use_graph and not eager.use_graph
    names = [n for n, _ in eager.model.named_parameters()] + [n for n, _ in eager.model.named_buffers()]
    edited = [eager.model.layer3[5].conv2.weight, eager.model.layer4[0].conv1.weight, eager.model.conv1.weight,
              eager.model.layer6.conv2d_list[1].weight]
    edited_g = [graphed.model.layer3[5].conv2.weight, graphed.model.layer4[0].conv1.weight,
                graphed.model.conv1.weight, graphed.model.layer6.conv2d_list[1].weight]
    losses = []
    for it in range(5):
        if it == 3:  # an eager edit between replays: the replay must see it (repack before replay)
            with torch.no_grad():
                for p, q in zip(edited, edited_g):
                    p.mul_(0.5)
                    q.mul_(0.5)
        xs, ys, xt = _inputs(it)
        for tr in (eager, graphed):
            tr.uda_step(xs, ys, xt)
        torch.cuda.synchronize()
        assert graphed._graphed is not None and graphed._graphed.replays == max(0, it)
        for name in ("loss_val", "loss_target", "loss_target_2"):
            a, b = getattr(graphed, name).item(), getattr(eager, name).item()
            assert a == b, (it, name, a, b)
        losses.append(eager.loss_val.item())
        assert torch.equal(graphed.target_loss.last_hist, eager.target_loss.last_hist), it
        d = _first_diff(_state(graphed), _state(eager), names)
        assert d is None, (it, d)
    assert graphed._graphed.eager_repacks == 1
    assert graphed.current_iter == eager.current_iter == 5
    # the poly learning rate moved every iteration (iter_max 1000): replays used the current one
    assert eager.optimizer.param_groups[0]["lr"] < 2.5e-4
    for name in ("loss_seg_value", "loss_target_value", "loss_target_value_2"):
        assert getattr(graphed, name).item() == getattr(eager, name).item()
    # after replays the packed-weight caches are stale for eager code: the version bump repacks
    x = synthetic_image(H, W, 77).cuda()
    with torch.no_grad():
        a2, a1 = graphed.model(x)
        b2, b1 = eager.model(x)
    assert torch.equal(a2, b2) and torch.equal(a1, b1)
