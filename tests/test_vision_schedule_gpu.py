"""Scheduling of the frozen image encoder (trainers/_vision.py) changes no result:

* CoOp / CoCoOp trained with the next-batch prefetch and the side-stream overlap on
  (NATIVE.PREFETCH_VISION / OVERLAP_VISION, the defaults) give bitwise the per-step losses,
  CoOp's post-step accuracy and the final prompt parameters of the inline schedule (the loop
  names the next batch as TrainerX.run_epoch does);
* a prefetched or remembered result is used only for the very tensor it was computed from,
  unmodified since: an in-place change of the images (their ``_version``) or another tensor
  with equal values forces a fresh image-encoder run.
Reference behaviour: image_encoder(image) inline in every forward (coop.py:356-363,
cocoop.py:238-251)."""
import pytest
import torch

from test_trainer_gpu import _init_like_fixture, _setup
from parity_util import load_fixture

pytestmark = pytest.mark.gpu


def _run(trainer, outdir, dev, on):
    _, ref = load_fixture(f"trainer_{trainer.lower()}")
    tr, _ = _setup(trainer, outdir, dev)
    tr.cfg.NATIVE["PREFETCH_VISION"] = on
    tr.cfg.NATIVE["OVERLAP_VISION"] = on
    _init_like_fixture(tr, trainer, ref)
    batches = tr.dm.train_loader_x
    tr.num_batches = len(batches)
    losses = []
    tr.set_model_mode("train")
    for step in range(2 * len(batches)):
        tr.batch_idx = step % len(batches)
        tr.next_batch = batches[(step + 1) % len(batches)]
        out = tr.forward_backward(batches[step % len(batches)])
        losses.append({k: float(v) for k, v in out.items()})
    params = [p.detach().clone() for p in tr.model.prompt_learner.parameters() if p.requires_grad]
    return losses, params


@pytest.mark.parametrize("trainer", ["CoOp", "CoCoOp"])
def test_schedule_is_bitwise_inline(dev, tmp_path, trainer):
    l_on, p_on = _run(trainer, tmp_path / "on", dev, True)
    l_off, p_off = _run(trainer, tmp_path / "off", dev, False)
    assert l_on == l_off, (l_on, l_off)
    assert len(p_on) == len(p_off) and all(torch.equal(a, b) for a, b in zip(p_on, p_off))


def test_features_only_for_the_same_unmodified_tensor(dev, tmp_path):
    tr, _ = _setup("CoCoOp", tmp_path / "out", dev)
    m = tr.model
    x = tr.dm.train_loader_x[0]["img"].to(dev).clone()
    inline = m.image_encoder(x)
    m.prefetch_image_features(x)
    same = m.cached_image_features(x)
    assert same is not None and torch.equal(same, inline)
    # the step's features are remembered for that tensor (CoOp's accuracy forward)
    assert m.cached_image_features(x) is same
    # equal values in another tensor: not reused
    y = x.clone()
    assert m.cached_image_features(y) is None
    # the same tensor modified in place: not reused, recomputed from the new values (the
    # write waits for the prefetch's reads of x: a prefetched tensor is not written in place
    # before the side stream is done with it, trainers/_vision.py)
    m.prefetch_image_features(x)
    m._side(x.device).synchronize()
    x.mul_(0.5)
    assert m.cached_image_features(x) is None
    fresh = m.image_features(x)
    assert torch.equal(fresh, m.image_encoder(x))
    assert not torch.equal(fresh, inline)
    # two prefetches in flight (the next batch's started before this one is consumed)
    a, b = x.clone(), y.clone()
    m.prefetch_image_features(a)
    m.prefetch_image_features(b)
    assert torch.equal(m.cached_image_features(a), m.image_encoder(a))
    assert torch.equal(m.cached_image_features(b), m.image_encoder(b))


def test_side_stream_runs_beside_main(dev):
    """The ViT prefetch's side stream is one whose work runs while the main stream is busy (a
    pool stream on the main stream's hardware queue would serialise the two: profiles/r05zb)."""
    from fsp_amd.trainers._vision import runs_beside, side_stream
    s = side_stream(dev)
    assert s is side_stream(dev), "one side stream per device"
    assert runs_beside(torch.cuda.current_stream(dev), s, dev)
