"""Scheduling of the frozen image encoder for the CoOp / CoCoOp CustomCLIPs.

The reference calls ``image_encoder(image)`` inline in every forward (coop.py:356-363,
cocoop.py:238-251). Its weights never train, so its output for a given image tensor is the
same whenever it is computed; this mixin uses that to move the ViT's small, latency-bound
launches next to the text encoder's:
* ``prefetch_image_features(image)`` starts it on a side stream for a batch the loop will pass
  later (NATIVE.PREFETCH_VISION; the loops name the next batch: TrainerX.run_epoch / test and
  bench.py keep one batch of lookahead), so it runs beside the current step's text encoder;
* ``image_features(image)`` returns the prefetched result when it was started for this very
  tensor (unmodified since), else the last result for it (CoOp's post-step accuracy forward of
  the same images, coop.py:464-469), else computes it now.
Results are bitwise the same as the inline call's.
Contract: a tensor passed to ``prefetch_image_features`` is read by the side stream until the
prefetch completes; the caller must not write it in place before then (consume the result with
``image_features`` first, or synchronise the side stream). A later in-place write is detected
(``_version``) and the stale result is not used."""
from __future__ import annotations

import time

import torch

# Side streams by device index, shared by every model of the process (they run one at a time).
_SIDE = {}


def runs_beside(main, side, device, timeout_s=2.0) -> bool:
    """Whether work queued on ``side`` runs while ``main`` is busy. HIP places each stream on one
    of a few hardware queues (GPU_MAX_HW_QUEUES, 4); a stream that shares the main stream's queue
    executes behind it in submission order, and a ViT "prefetched" there serialises with the
    text encoder (+0.5 ms at B = 8, +0.6 ms at B = 1: tools/lab/side_stream_ab.py,
    profiles/r05zb). Probe: ~4 ms of GEMMs on main, then a tiny op on side; on separate
    queues the tiny op completes first."""
    x = torch.zeros(1, device=device)
    with torch.cuda.stream(side):  # the stream's first use (its queue may be created lazily)
        x.add_(1)
    torch.cuda.synchronize(device)
    a = torch.randn(8192, 8192, device=device, dtype=torch.float16)
    with torch.cuda.stream(main):
        for _ in range(4):
            torch.mm(a, a)
        ev_main = torch.cuda.Event()
        ev_main.record(main)
    with torch.cuda.stream(side):
        x.add_(1)
        ev_side = torch.cuda.Event()
        ev_side.record(side)
    t0 = time.perf_counter()
    while not ev_side.query():
        if time.perf_counter() - t0 > timeout_s:
            break
    beside = ev_side.query() and not ev_main.query()
    torch.cuda.synchronize(device)
    return beside


def side_stream(device):
    """A pool stream that runs beside the current (main) stream, probed once per device (up to
    8 candidates; the last one if none passes)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    side = _SIDE.get(idx)
    if side is None:
        main = torch.cuda.current_stream(device)
        held = []  # keep rejected candidates referenced while probing the next ones
        for _ in range(8):
            side = torch.cuda.Stream(device)
            if runs_beside(main, side, device):
                break
            held.append(side)
        _SIDE[idx] = side
    return side


class ImageFeatureSchedule:
    def _side(self, device):
        side = getattr(self, "_side_stream", None)
        if side is None or side.device != device:
            side = self._side_stream = side_stream(device)
        return side

    def prefetch_image_features(self, image, after=None):
        """after: an event recorded on the main stream once `image` is ready there; the side
        stream waits for it instead of for everything queued on main so far (a caller may queue
        the current step's work first and start the prefetch behind it on the host)."""
        main = torch.cuda.current_stream(image.device)
        side = self._side(image.device)
        if after is not None:
            side.wait_event(after)
        else:
            side.wait_stream(main)
        with torch.cuda.stream(side):
            imf = self.image_encoder(image)
            done = torch.cuda.Event()
            done.record(side)
        image.record_stream(side)  # its memory is not reused while the side stream reads it
        # an event, not the stream: later work queued on the side stream (the next prefetch)
        # must not hold up the step that consumes this result. Two entries: a step may start
        # the next batch's prefetch before it consumes its own.
        pend = getattr(self, "_prefetched", None) or []
        self._prefetched = (pend + [(image, image._version, imf, done)])[-2:]

    def image_features_async(self, image):
        """The image encoder on the side stream for THIS step's images, beside work the caller
        queues next on the main stream; returns join() -> features (waits on the main stream)."""
        main = torch.cuda.current_stream(image.device)
        side = self._side(image.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            imf = self.image_encoder(image)
            done = torch.cuda.Event()
            done.record(side)
        image.record_stream(side)

        def join():
            main.wait_event(done)
            imf.record_stream(main)
            self._last_imf = (image, image._version, imf)
            return imf
        return join

    def cached_image_features(self, image):
        """The prefetched or last result for this very tensor, or None."""
        pend = getattr(self, "_prefetched", None) or []
        hit = [pf for pf in pend if pf[0] is image and pf[1] == image._version]
        if hit:
            self._prefetched = [pf for pf in pend if pf is not hit[0]]
            _, _, imf, done = hit[0]
            main = torch.cuda.current_stream(image.device)
            main.wait_event(done)
            imf.record_stream(main)
            self._last_imf = (image, image._version, imf)
            return imf
        last = getattr(self, "_last_imf", None)
        if last is not None and last[0] is image and last[1] == image._version:
            return last[2]
        return None

    def image_features(self, image):
        imf = self.cached_image_features(image)
        if imf is None:
            imf = self.image_encoder(image)
            self._last_imf = (image, image._version, imf)
        return imf
