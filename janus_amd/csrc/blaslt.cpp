// The encoder's large-M projections on hipBLASLt — a COMPARISON point only
// (janus_gemm_lt_f16, tools/gemm_big_probe.py): the product path runs the hand-written
// gemm_big kernel (gemm_big.hip), at parity with the library over an encoder layer
// (954 vs 963 us at 64 x 1500 rows, base.en). The GELU projection uses the
// library's bias epilogue into fp16 followed by an exact-erf GELU pass in place (the
// library's GELU is not Whisper's erf form).
// Plans are restricted to workspace-free solutions and handles are per device, so
// concurrent callers on different streams or devices share no scratch memory.
//
// Row-major C[M][N] = A[M][K] W[N][K]^T is the column-major problem
// C^T[N x M] = op_T(W as [K x N], ld = ldw) * op_N(A as [K x M], ld = lda), bias per
// column-major row (= per output column n).
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "kernels.h"

namespace janus {

namespace {

#define LT_CHECK(x)                                                                    \
  do {                                                                                 \
    hipblasStatus_t st_ = (x);                                                         \
    if (st_ != HIPBLAS_STATUS_SUCCESS)                                                 \
      throw Error(std::string("hipBLASLt: ") + #x + " failed (" + std::to_string((int)st_) + ")"); \
  } while (0)

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool ok = false;
};

struct Lt {
  hipblasLtHandle_t h = nullptr;
  std::map<std::tuple<int, int, int, int, int64_t, int64_t, int64_t>, Plan> plans;
};

std::mutex g_lt_mu;  // guards the per-device map and every plan's descriptor

Lt& lt() {  // the calling thread's current device
  static std::map<int, Lt*> per_dev;
  int dev = 0;
  JANUS_HIP(hipGetDevice(&dev));
  Lt*& l = per_dev[dev];
  if (!l) {
    l = new Lt;
    LT_CHECK(hipblasLtCreate(&l->h));
  }
  return *l;
}

Plan& plan_for(Lt& L, int epi, int M, int N, int K, int64_t lda, int64_t ldw, int64_t ldc) {
  const auto key = std::make_tuple(epi, M, N, K, lda, ldw, ldc);
  auto it = L.plans.find(key);
  if (it != L.plans.end()) return it->second;
  Plan p;
  const bool f32out = epi == EPI_RESID_F32 || epi == EPI_F32;
  const hipDataType ct = f32out ? HIP_R_32F : HIP_R_16F;
  LT_CHECK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
  const hipDataType bt = HIP_R_32F;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16F, K, N, ldw));  // W as [K x N]
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16F, K, M, lda));  // A as [K x M]
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.lc, ct, N, M, ldc));         // C^T as [N x M]
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  const size_t no_ws = 0;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES,
                                                 &no_ws, sizeof(no_ws)));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(L.h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1,
                                                             res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st == HIPBLAS_STATUS_SUCCESS && n > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS) {
    p.algo = res[0].algo;
    p.ws = res[0].workspaceSize;
    p.ok = p.ws == 0;
  }
  return L.plans.emplace(key, p).first->second;
}

}  // namespace

// true when the library ran the GEMM; false = no plan for this shape (caller falls back
// to gemm_launch). Epilogues: EPI_F16 / EPI_F32 (bias), EPI_RESID_F32 (C == R in place,
// beta = 1), EPI_GELU_F16 (bias into C, then the erf GELU in place).
bool gemm_lt_launch(int epi, const GemmArgs& g, hipStream_t s) {
  if (!(epi == EPI_F16 || epi == EPI_F32 || epi == EPI_RESID_F32 || epi == EPI_GELU_F16)) return false;
  if (epi == EPI_RESID_F32 && (g.R != g.C || g.ldr != g.ldc)) return false;
  if (g.a_group_cols || g.lnin_x || g.ln_part || g.ln_out || g.kc) return false;
  std::lock_guard<std::mutex> lock(g_lt_mu);
  Lt& L = lt();
  Plan& p = plan_for(L, epi, g.M, g.N, g.K, g.lda, g.ldw, g.ldc);
  if (!p.ok) return false;
  const float alpha = 1.0f, beta = epi == EPI_RESID_F32 ? 1.0f : 0.0f;
  const void* bias = g.bias;
  float* zero_bias = nullptr;
  if (!bias) return false;  // (every encoder projection carries a bias)
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  (void)zero_bias;
  LT_CHECK(hipblasLtMatmul(L.h, p.desc, &alpha, g.W, p.la, g.A, p.lb, &beta, g.C, p.lc, g.C, p.lc,
                           &p.algo, nullptr, 0, s));
  if (epi == EPI_GELU_F16)
    gelu_inplace_f16_launch(static_cast<_Float16*>(g.C), g.ldc, g.M, g.N, s);
  return true;
}

}  // namespace janus
