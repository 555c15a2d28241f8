"""ctypes binding of libclipk.so (the C-ABI in include/clipk.h).

There is no CPU fallback: if the library is missing or the device is not a gfx950
GPU, every op raises. Build with ``python __graft_entry__.py`` (``build()``) or
``make -C <pkg>/csrc``.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import sys

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CLIPK_LIB") or os.path.join(_PKG, "libclipk.so")  # override: A/B builds
_ROOT = os.path.dirname(_PKG)


def source_files():
    """The sources libclipk.so is built from, as (path relative to the repo root, absolute path):
    csrc/{*.hip, *.h, Makefile} and include/clipk.h, in name order."""
    csrc = os.path.join(_PKG, "csrc")
    names = sorted(n for n in os.listdir(csrc) if n.endswith((".hip", ".h")) or n == "Makefile")
    rel = [("csrc/" + n, os.path.join(csrc, n)) for n in names]
    return rel + [("include/clipk.h", os.path.join(_ROOT, "include", "clipk.h"))]


def source_digest():
    """sha256 (hex) of "<sha256 of content>  <relative path>\n" over source_files(): the value
    the Makefile compiles into the library (clipk_source_digest, include/clipk.h)."""
    h = hashlib.sha256()
    for rel, path in source_files():
        with open(path, "rb") as f:
            h.update(f"{hashlib.sha256(f.read()).hexdigest()}  {rel}\n".encode())
    return h.hexdigest()

F32, F16, BF16, F32S = 0, 1, 2, 3  # F32S: fp32 activations x split-packed weights (PREC fp32s)
PREFIX_CLS_GROUP0 = 1  # clipk_attention_prefix_*_ex flag
F32S16 = 4  # F32S for fp16-valued weights: B is the compact fp16 SPLIT_SCALE * W (clipk_split_hi16)
SPLIT_SCALE = 64.0  # CLIPK_SPLIT_SCALE: clipk_split_pack stores SPLIT_SCALE * W
EPI_BIAS, EPI_BIAS_RES, EPI_BIAS_QGELU, EPI_DQGELU, EPI_NONE = 0, 1, 2, 3, 4
A_QGELU = 0x100  # OR-ed into epi: the GEMM consumes quickgelu(A) (include/clipk.h)
QGELU_DERIV = 0x200  # OR-ed into epi: out2 = quickgelu' (EPI_BIAS_QGELU) / aux is quickgelu' (EPI_DQGELU)
OUT_SPLIT, A_SPLIT = 0x400, 0x800  # PREC fp32s pre-split operands (include/clipk.h)
PROF_NONE, PROF_GEMM_FC, PROF_GEMM_ALL, PROF_ATTN, PROF_LN, PROF_GEMM_DGELU = 0, 1, 2, 3, 4, 5

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_S = ctypes.c_size_t
_D = ctypes.c_double

# name -> (restype, argtypes); must match include/clipk.h exactly
SIGNATURES = {
    "clipk_version": (ctypes.c_char_p, []),
    "clipk_source_digest": (ctypes.c_char_p, []),
    "clipk_strerror": (ctypes.c_char_p, [_I]),
    "clipk_device_arch_ok": (_I, []),
    "clipk_gemm": (_I, [_I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P, _I, _P, _I, _P, _P, _I, _I, _P]),
    "clipk_gemm_auto_splits": (_I, [_I, _I, _I, _I]),
    "clipk_gemm_splitk_ws_bytes": (_S, [_I, _I, _I]),
    "clipk_gemm_splitk": (_I, [_I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P, _I, _P, _I, _P, _I, _P, _S, _P]),
    "clipk_gemm_set_config": (_I, [_I]),
    "clipk_split_pack": (_I, [_I, _I, _P, _I, _P, _P]),
    "clipk_split_lo_zero": (_I, [_I, _I, _P, _P, _P]),
    "clipk_split_hi16": (_I, [_I, _I, _P, _P, _P]),
    "clipk_gemm_ln": (_I, [_I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P]),
    "clipk_ln_stats_merge": (_I, [_I, _I, _P, _P, _P, _P, _P]),
    "clipk_gemm_ln_merge_fused": (_I, [_I, _I, _I, _I]),
    "clipk_gemm_ln_stats_split": (_I, [_I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P, _I, _P, _I, _P, _P, _P, _P]),
    "clipk_gemm_ln_gamma": (_I, [_I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P, _I, _P, _P, _P, _P, _P]),
    "clipk_gemm_ln_merge": (_I, [_I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "clipk_image_resample": (_I, [_I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P]),
    "clipk_gemm_stamps": (_I, [_P, _S]),
    "clipk_layernorm_fwd": (_I, [_I, _I, _I, _P, _I, _P, _P, _P, _P, _I, _P, _P, _P]),
    "clipk_layernorm_bwd": (_I, [_I, _I, _I, _P, _I, _P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _I, _P, _I, _P]),
    "clipk_layernorm_fwd_x": (_I, [_I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _I, _P, _P, _P]),
    "clipk_layernorm_bwd_x": (_I, [_I, _I, _I, _I, _P, _I, _P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _I, _P, _I, _P]),
    "clipk_layernorm_bwd_x2": (_I, [_I, _I, _I, _I, _P, _I, _P, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P, _I, _P, _I, _P]),
    "clipk_attention_fwd": (_I, [_I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "clipk_attention_bwd": (_I, [_I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _I, _P, _P, _I, _P]),
    "clipk_im2col": (_I, [_I, _I, _I, _I, _I, _P, _P, _P]),
    "clipk_vit_embed_ln": (_I, [_I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "clipk_prompt_assemble": (_I, [_I, _I, _I, _I, _P, _P, _P, _L, _L, _P, _P, _P, _P]),
    "clipk_ctx_grad": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "clipk_prompt_assemble_rows": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, _L, _L, _P, _P, _P, _P]),
    "clipk_ctx_grad_rows": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "clipk_ctx_bias_grad_rows": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "clipk_attention_prefix_fwd": (_I, [_I, _I, _I, _I, _I, _P, _P, _I, _P, _I, _P, _I, _P, _P]),
    "clipk_attention_prefix_ws_bytes": (_S, [_I, _I, _I]),
    "clipk_attention_prefix_bwd": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _I, _P, _I, _P, _I, _P, _I, _P, _P,
                                        _I, _P, _S, _P]),
    "clipk_attention_prefix_fwd_ex": (_I, [_I, _I, _I, _I, _I, _P, _P, _I, _P, _I, _P, _I, _P, _I, _P]),
    "clipk_attention_prefix_bwd_ex": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _I, _P, _I, _P, _I, _P, _I, _P, _P,
                                           _I, _P, _S, _I, _P]),
    "clipk_cosine_logits_fwd": (_I, [_I, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P]),
    "clipk_cosine_logits_bwd": (_I, [_I, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P, _P]),
    "clipk_ce_loss": (_I, [_I, _I, _P, _P, _P, _F, _I, _F, _P, _P, _P]),
    "clipk_ce_loss_reduce": (_I, [_I, _I, _P, _P, _P, _F, _I, _F, _I, _P, _P, _P, _P]),
    "clipk_meta_net_fwd": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "clipk_meta_net_fwd_norm": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "clipk_status_take": (_I, [_P, _P, _P]),
    "clipk_meta_net_bwd": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "clipk_sgd_step": (_I, [_L, _P, _P, _P, _F, _F, _F, _I, _P]),
    "clipk_sgd_step_multi": (_I, [_I, _P, _P, _P, _P, _P, _F, _F, _F, _P]),
    "clipk_sgd_step_multi_scaled": (_I, [_I, _P, _P, _P, _P, _P, _F, _F, _F, _F, _P]),
    "clipk_sgd_step_multi_if": (_I, [_I, _P, _P, _P, _P, _P, _F, _F, _F, _F, _P, _I, _P]),
    "clipk_cast": (_I, [_I, _L, _P, _P, _P]),
    "clipk_rows_copy": (_I, [_I, _I, _P, _P, _P, _P, _P]),
    "clipk_vit_embed_ln_vpt": (_I, [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "clipk_rows_inject": (_I, [_I, _I, _I, _I, _P, _P, _P, _I, _P]),
    "clipk_rows_collect": (_I, [_I, _I, _I, _I, _P, _I, _P, _I, _I, _P, _P, _I, _I, _P]),
    "clipk_encoder_set_deep_prompts": (_I, [_P, _I, _I, _I, _P, _P, _P]),
    "clipk_encoder_set_input_rows": (_I, [_P, _I]),
    "clipk_encoder_set_ln_fold": (_I, [_P, _P]),
    "clipk_encoder_set_split": (_I, [_P, _I]),
    "clipk_encoder_set_split_target": (_I, [_P, _I]),
    "clipk_encoder_set_status": (_I, [_P, _P]),
    "clipk_vit_prompted_saved_bytes": (_S, [_P, _I, _I]),
    "clipk_vit_prompted_ws_bytes": (_S, [_P, _I, _I]),
    "clipk_vit_forward_prompted": (_I, [_P, _I, _P, _I, _P, _P, _P, _S, _P, _S, _P]),
    "clipk_vit_backward_prompted": (_I, [_P, _I, _I, _P, _P, _P, _P, _S, _P, _P, _S, _P]),
    "clipk_encoder_create": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "clipk_encoder_destroy": (None, [_P]),
    "clipk_text_saved_bytes": (_S, [_P, _I, _I]),
    "clipk_text_ws_bytes": (_S, [_P, _I, _I]),
    "clipk_text_forward": (_I, [_P, _I, _I, _P, _P, _P, _P, _S, _P, _S, _P]),
    "clipk_text_bwd_ws_bytes": (_S, [_P, _I, _I]),
    "clipk_text_backward": (_I, [_P, _I, _I, _P, _P, _P, _S, _P, _P, _S, _P]),
    "clipk_text_packed_saved_bytes": (_S, [_P, _I, _I, _I]),
    "clipk_text_packed_ws_bytes": (_S, [_P, _I, _I, _I]),
    "clipk_text_packed_bwd_ws_bytes": (_S, [_P, _I, _I, _I, _I]),
    "clipk_text_forward_packed": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _S, _P, _S, _P]),
    "clipk_text_backward_packed": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _S, _P, _P, _S, _P]),
    "clipk_vision_create": (_I, [_I, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "clipk_vit_ws_bytes": (_S, [_P, _I]),
    "clipk_vit_forward": (_I, [_P, _I, _P, _P, _P, _S, _P]),
    "clipk_prof_enable": (_I, [_I]),
    "clipk_prof_read": (_I, [_P, _P, _P]),
    "clipk_prof_sites_enable": (_I, [_I]),
    "clipk_prof_sites_read": (_I, [_I, _P, _P, _P, _P, _P, _P]),
}

PROF_NAME_LEN = 32


def prof_sites_read(max_sites: int = 64):
    """{site: (total_ms, launches, flops, bytes)} accumulated since the last read / enable."""
    lib = load()
    names = ctypes.create_string_buffer(max_sites * PROF_NAME_LEN)
    ms = (ctypes.c_double * max_sites)()
    cnt = (ctypes.c_long * max_sites)()
    fl = (ctypes.c_double * max_sites)()
    by = (ctypes.c_double * max_sites)()
    n = ctypes.c_int()
    check(lib.clipk_prof_sites_read(max_sites, names, ms, cnt, fl, by, ctypes.byref(n)), "clipk_prof_sites_read")
    out = {}
    for i in range(n.value):
        nm = names.raw[i * PROF_NAME_LEN:(i + 1) * PROF_NAME_LEN].split(b"\0", 1)[0].decode()
        if cnt[i]:
            out[nm] = (ms[i], cnt[i], fl[i], by[i])
    return out

_lib = None


class ClipkError(RuntimeError):
    pass


def load():
    """Load libclipk.so and declare every C-ABI signature (no device calls)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise ClipkError(f"{LIB_PATH} is missing: the HIP extension is not built "
                         f"(run `python __graft_entry__.py` or `make -C csrc`). No CPU fallback exists.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    built = lib.clipk_source_digest().decode()
    tree = source_digest()
    if built != tree:
        raise ClipkError(f"{LIB_PATH} was built from other sources than this tree (library digest {built[:16]}, "
                         f"tree {tree[:16]}): rebuild it (`python __graft_entry__.py` or `make -C csrc`)")
    _lib = lib
    return lib


def library_digest():
    """clipk_source_digest() of the loaded library (== source_digest(): load() checks it)."""
    return load().clipk_source_digest().decode()


def strerror(rc: int) -> str:
    return load().clipk_strerror(rc).decode()


def check(rc: int, what: str):
    if rc != 0:
        raise ClipkError(f"{what} failed: {strerror(rc)} (status {rc})")


def call(name: str, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc


if __name__ == "__main__" and sys.argv[1:] == ["--digest-header"]:
    # csrc/Makefile: the digest compiled into the library
    print(f'#define CLIPK_SOURCE_DIGEST "{source_digest()}"')
