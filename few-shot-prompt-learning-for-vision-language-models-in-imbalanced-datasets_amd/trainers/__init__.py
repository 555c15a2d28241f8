"""CoOp / CoCoOp / ZeroshotCLIP / IVLP / MaPLe / PromptSRC trainers (registered in
fsp_amd.engine.TRAINER_REGISTRY)."""
from . import coop, cocoop, zsclip, deep  # noqa: F401
