"""Minimal Dassl-compatible engine surface for the CoOp/CoCoOp path."""
from .registry import Registry, TRAINER_REGISTRY, build_trainer  # noqa: F401
