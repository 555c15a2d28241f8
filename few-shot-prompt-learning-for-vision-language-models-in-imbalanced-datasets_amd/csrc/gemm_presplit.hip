// PREC fp32s GEMMs with pre-split operands (include/clipk.h CLIPK_A_SPLIT / CLIPK_OUT_SPLIT /
// CLIPK_OUT2_SPLIT_GAMMA): the split loop's A fragments arrive as fp16 hi / lo parts a producer
// epilogue already formed, so the K loop issues no split VALU (the split sits in the ping-pong
// loop's memory segment, each A element split once per wave column: measured 23 % of every split
// GEMM's launch, tools/split_gemm_bench.py NOSPLIT, profiles/r06b/). Own translation unit: these
// instantiations compile beside gemm.hip's.
#include "gemm_kernel.h"

namespace clipk {

// (epi, lnm, spf) combinations the encoders launch; others CLIPK_EINVAL. lnm: 0 plain, 1 the
// LayerNorm-statistics producer, 2 the fold with W' in B, 4 the fold with gamma on A.
template <typename TS>
static int presplit_combo(int spf, int epi, int lnm, const GemmArgs& g, hipStream_t st) {
  constexpr bool H = __is_same(TS, f32h);
  const int key = (spf << 16) | (lnm << 8) | epi;
  auto K3 = [](int s, int l, int e) { return (s << 16) | (l << 8) | e; };
  // phase 1: c_fc -> c_proj (g), dgelu -> fc_dx (dh)
  if (key == K3(1, 0, CLIPK_EPI_NONE)) return launch_gemm_split<CLIPK_EPI_NONE, 0, TS, 1>(g, st);
  if (key == K3(1, 0, CLIPK_EPI_BIAS_RES)) return launch_gemm_split<CLIPK_EPI_BIAS_RES, 0, TS, 1>(g, st);
  if (key == K3(1, 1, CLIPK_EPI_BIAS_RES)) return launch_gemm_split<CLIPK_EPI_BIAS_RES, 1, TS, 1>(g, st);
  if (key == K3(2, 0, CLIPK_EPI_BIAS_QGELU)) return launch_gemm_split<CLIPK_EPI_BIAS_QGELU, 0, TS, 2>(g, st);
  if (key == K3(2, 0, EPI_QGELU_D)) return launch_gemm_split<EPI_QGELU_D, 0, TS, 2>(g, st);
  if (key == K3(2, 2, CLIPK_EPI_BIAS_QGELU)) return launch_gemm_split<CLIPK_EPI_BIAS_QGELU, 2, TS, 2>(g, st);
  if (key == K3(2, 2, EPI_QGELU_D)) return launch_gemm_split<EPI_QGELU_D, 2, TS, 2>(g, st);
  if (key == K3(2, 0, EPI_DMUL)) return launch_gemm_split<EPI_DMUL, 0, TS, 2>(g, st);
  if constexpr (H) {  // split mode 2 (fp16-valued weights, the LayerNorm weight on A)
    if (key == K3(2, 4, CLIPK_EPI_BIAS_QGELU)) return launch_gemm_split<CLIPK_EPI_BIAS_QGELU, 4, TS, 2>(g, st);
    if (key == K3(2, 4, EPI_QGELU_D)) return launch_gemm_split<EPI_QGELU_D, 4, TS, 2>(g, st);
    // the residual stream's split copy at the gamma of the next fold: out_proj (-> c_fc), c_proj
    // (-> the next layer's qkv) and those folds reading it
    if (key == K3(4, 1, CLIPK_EPI_BIAS_RES)) return launch_gemm_split<CLIPK_EPI_BIAS_RES, 1, TS, 4>(g, st);
    if (key == K3(5, 1, CLIPK_EPI_BIAS_RES)) return launch_gemm_split<CLIPK_EPI_BIAS_RES, 1, TS, 5>(g, st);
    if (key == K3(1, 4, CLIPK_EPI_BIAS)) return launch_gemm_split<CLIPK_EPI_BIAS, 4, TS, 1>(g, st);
    if (key == K3(3, 4, CLIPK_EPI_BIAS_QGELU)) return launch_gemm_split<CLIPK_EPI_BIAS_QGELU, 4, TS, 3>(g, st);
    if (key == K3(3, 4, EPI_QGELU_D)) return launch_gemm_split<EPI_QGELU_D, 4, TS, 3>(g, st);
    // dgelu reading the residual gradient's split copy and writing dh split
    if (key == K3(3, 0, EPI_DMUL)) return launch_gemm_split<EPI_DMUL, 0, TS, 3>(g, st);
    if (key == K3(1, 0, EPI_DMUL)) return launch_gemm_split<EPI_DMUL, 0, TS, 1>(g, st);
  }
  return CLIPK_EINVAL;
}

int presplit_launch(bool w16, int spf, int epi, int lnm, const GemmArgs& g, hipStream_t st) {
  return w16 ? presplit_combo<f32h>(spf, epi, lnm, g, st) : presplit_combo<f32s>(spf, epi, lnm, g, st);
}

}  // namespace clipk
