"""CoOp / CoCoOp trainers (registered in fsp_amd.engine.TRAINER_REGISTRY)."""
from . import coop, cocoop  # noqa: F401
