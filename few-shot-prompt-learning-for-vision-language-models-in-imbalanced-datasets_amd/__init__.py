"""MI355X-native CoOp/CoCoOp prompt-tuning hot path (import as ``fsp_amd``).

Layout:
  csrc/      hand-written HIP kernels for gfx950 + the C-ABI (libclipk.so)
  _native.py ctypes binding of the C-ABI (fails loudly if the library is missing)
  clip/      CLIP model host side: weight packing, encoders, tokenizer, synthetic weights
  trainers/  CoOp / CoCoOp (same registry names, cfg keys and module contract as the
             reference PromptSRC/trainers/{coop,cocoop}.py)
  engine/    minimal Dassl-compatible registry / trainer contract / optim / evaluator
"""
__version__ = "0.1.0"
