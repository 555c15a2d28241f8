"""CoOp / CoCoOp / ZeroshotCLIP trainers (registered in fsp_amd.engine.TRAINER_REGISTRY)."""
from . import coop, cocoop, zsclip  # noqa: F401
