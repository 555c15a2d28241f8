"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the CoOp/CoCoOp hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import anything from here, and only as the checker / the timed CPU baseline.
The product package (``fsp_amd``) never imports it and has no CPU fallback.

``clip_oracle`` restates the reference algorithm (``PromptSRC/clip/model.py`` and
``PromptSRC/trainers/{coop,cocoop}.py``) in plain fp32 PyTorch on the CPU with
explicit ops. Parity is pinned: ``tests/test_oracle_golden.py`` checks it against
golden vectors produced by running the reference itself in the survey container
(``tests/golden/make_golden.py``).
"""
