// hipBLASLt for BERT-base's plain dense GEMMs (bf16 operands, fp32 accumulation): the projections' forward with a
// bias, the input gradients with a residual, the weight gradients into the fp32 gradient (reference: the
// nn.Linear layers of transformers' BertModel, model/lang/bert_hugface.py:20). The fused epilogues stay on the
// hand-written engine (GELU + pre-activation, GELU', BN epilogues, every convolution); this is the vendor library
// for the GEMMs that carry nothing but a bias or an addend, where it measured faster than the 128 x 128 LDS-DMA
// engine (profiles/r05_bert_lt_ab.txt). VCG_LT_GEMM=0 keeps every GEMM on the engine.
//
// Row-major C[M][N] = op(A) op(B)^T is the column-major C^T = op(B) op(A)^T: hipBLASLt's (m, n, k) = (N, M, K),
// its first operand our B, its second our A; the bias is per column of C = per row of C^T (the library's bias).
// One plan per shape (descriptors, layouts and the heuristic's first algorithm, chosen once: the same algorithm --
// the same summation order -- for every call of a shape) and one workspace per stream (BERT's GEMMs run on a side
// stream beside the trunk; two streams never share a workspace).
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "igemm.h"

namespace vcg {
namespace {

constexpr size_t LT_WS = 64ull << 20;

struct LtPlan {
  bool ok = false;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  std::vector<hipblasLtMatmulAlgo_t> cands;  // the heuristic's candidates in its order; algo = cands[0]
};
constexpr int LT_CANDS = 16;

struct LtState {
  std::mutex mu;
  std::map<int, hipblasLtHandle_t> handle;  // per device
  std::map<std::tuple<int, int, int, int, int, int, long long, long long, long long, long long, int, int, int>, LtPlan> plans;
  std::map<std::pair<int, hipStream_t>, void*> ws;  // per (device, stream)
};

LtState& lt_state() {
  static LtState* s = new LtState();  // (never destroyed: plans may be in use at exit)
  return *s;
}

}  // namespace

bool lt_gemm_enabled() {  // (read per call: tests compare both paths in one process)
  const char* e = getenv("VCG_LT_GEMM");
  return e == nullptr || e[0] != '0';
}

// D = op(A) op(B)^T (+ bias[n]) (+ beta C): A, B bf16 row-major (transA: A is [K][lda], else [M][lda]; transB: B is
// [K][ldb], else [N][ldb]); C / D bf16 or fp32 (d_f32) row-major with ldc / ldd (C may alias D). Returns VCG_OK,
// or VCG_ERR_UNSUPPORTED when the library has no algorithm for the shape (the caller runs the engine instead).
int lt_gemm(int transA, int transB, int M, int N, int K, const void* A, long long lda, const void* B, long long ldb,
            const void* C, long long ldc, void* D, long long ldd, int d_f32, const float* bias, float beta,
            hipStream_t stream) {
  LtState& st = lt_state();
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return VCG_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> lock(st.mu);
  auto hit = st.handle.find(dev);
  if (hit == st.handle.end()) {
    hipblasLtHandle_t h = nullptr;
    if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return VCG_ERR_UNSUPPORTED;
    hit = st.handle.emplace(dev, h).first;
  }
  const hipblasLtHandle_t h = hit->second;
  const bool has_c = C != nullptr && beta != 0.f;
  const auto key = std::make_tuple(dev, transA, transB, M, N, K, lda, ldb, has_c ? ldc : 0LL, ldd, d_f32,
                                   bias != nullptr ? 1 : 0, has_c ? 1 : 0);
  auto pit = st.plans.find(key);
  if (pit == st.plans.end()) {
    LtPlan p;
    const hipDataType dt = d_f32 ? HIP_R_32F : HIP_R_16BF;
    // first operand = our B: stored row-major [N][ldb] (= column-major [ldb x N], op T) or [K][ldb] (op N)
    const hipblasOperation_t op1 = transB ? HIPBLAS_OP_N : HIPBLAS_OP_T;
    const hipblasOperation_t op2 = transA ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    bool good = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
    good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &op1, sizeof(op1)) ==
                       HIPBLAS_STATUS_SUCCESS;
    good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &op2, sizeof(op2)) ==
                       HIPBLAS_STATUS_SUCCESS;
    if (good && bias) {
      const hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BIAS;
      const int32_t bt = HIP_R_32F;
      good = hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)) ==
                 HIPBLAS_STATUS_SUCCESS &&
             hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) ==
                 HIPBLAS_STATUS_SUCCESS;
    }
    // column-major layouts: first operand [rows x cols] as stored, second likewise, C / D [N x M]
    good = good && hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, transB ? N : K, transB ? K : N, ldb) ==
                       HIPBLAS_STATUS_SUCCESS;
    good = good && hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, transA ? M : K, transA ? K : M, lda) ==
                       HIPBLAS_STATUS_SUCCESS;
    good = good && hipblasLtMatrixLayoutCreate(&p.lc, dt, N, M, has_c ? ldc : ldd) == HIPBLAS_STATUS_SUCCESS;
    good = good && hipblasLtMatrixLayoutCreate(&p.ld, dt, N, M, ldd) == HIPBLAS_STATUS_SUCCESS;
    if (good) {
      hipblasLtMatmulPreference_t pref = nullptr;
      uint64_t wsb = LT_WS;
      hipblasLtMatmulHeuristicResult_t res[LT_CANDS];
      int n = 0;
      if (hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS &&
          hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)) ==
              HIPBLAS_STATUS_SUCCESS &&
          hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.lc, p.ld, pref, LT_CANDS, res, &n) ==
              HIPBLAS_STATUS_SUCCESS) {
        for (int i = 0; i < n; ++i)
          if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= LT_WS) p.cands.push_back(res[i].algo);
        if (!p.cands.empty()) {
          p.algo = p.cands[0];
          p.ok = true;
        }
      }
      if (pref) hipblasLtMatmulPreferenceDestroy(pref);
    }
    pit = st.plans.emplace(key, p).first;
  }
  LtPlan& p = pit->second;
  if (!p.ok) return VCG_ERR_UNSUPPORTED;
  void*& w = st.ws[{dev, stream}];
  if (w == nullptr && hipMalloc(&w, LT_WS) != hipSuccess) {
    w = nullptr;
    return VCG_ERR_UNSUPPORTED;
  }
  if (bias) {
    if (hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
        HIPBLAS_STATUS_SUCCESS)
      return VCG_ERR_UNSUPPORTED;
  }
  const float alpha = 1.f, b = has_c ? beta : 0.f;
  const hipblasStatus_t rc = hipblasLtMatmul(h, p.desc, &alpha, B, p.la, A, p.lb, &b, has_c ? C : D, p.lc, D, p.ld,
                                             &p.algo, w, LT_WS, stream);
  if (rc != HIPBLAS_STATUS_SUCCESS) {
    set_error("hipblasLtMatmul failed (" + std::to_string((int)rc) + ")");
    return VCG_ERR_HIP;
  }
  return VCG_OK;
}

// out = gelu(pre) over [rows][8 n8] bf16 with row pitch ld (elements): FFN1's activation after the library GEMM
// wrote the pre-activation (bias added, rounded to bf16) -- the bf16-autocast order of the reference's Linear ->
// GELU. fast: erf_fast (the bf16 epilogues' GELU, common.h), else erff.
__global__ __launch_bounds__(256) void lt_gelu_kernel(const bf16_t* __restrict__ pre, bf16_t* __restrict__ out,
                                                      long long rows, int n8, long long ld, int fast) {
  const long long total = rows * n8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long r = i / n8;
    const long long off = r * ld + 8 * (i - r * n8);
    const uint4 u = *reinterpret_cast<const uint4*>(pre + off);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = __uint_as_float(w[k] << 16), hi = __uint_as_float(w[k] & 0xffff0000u);
      const float glo = fast ? gelu_erf_fast(lo) : gelu_erf(lo), ghi = fast ? gelu_erf_fast(hi) : gelu_erf(hi);
      o[k] = (uint32_t)f2bf(glo) | ((uint32_t)f2bf(ghi) << 16);
    }
    *reinterpret_cast<uint4*>(out + off) = uint4{o[0], o[1], o[2], o[3]};
  }
}

// pre = op(A) op(B)^T + bias (bf16, the library), out = gelu(pre): VCG_OK / VCG_ERR_UNSUPPORTED (engine instead)
int lt_gemm_gelu(int transA, int transB, int M, int N, int K, const void* A, long long lda, const void* B,
                 long long ldb, const float* bias, void* pre, void* out, long long ld, int fast, hipStream_t stream) {
  if (N % 8 != 0 || ld % 8 != 0 || (((uintptr_t)pre | (uintptr_t)out) & 15) != 0) return VCG_ERR_UNSUPPORTED;
  const int rc = lt_gemm(transA, transB, M, N, K, A, lda, B, ldb, nullptr, 0, pre, ld, 0, bias, 0.f, stream);
  if (rc != VCG_OK) return rc;
  const long long total = (long long)M * (N / 8);
  const int grid = (int)std::min<long long>((total + 255) / 256, 256LL * 16);
  hipLaunchKernelGGL(lt_gelu_kernel, dim3(grid), dim3(256), 0, stream, (const bf16_t*)pre, (bf16_t*)out, (long long)M,
                     N / 8, ld, fast);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

}  // namespace vcg

using namespace vcg;

// Tuning aid (tools/lt_tune.py; not on the product path): time the heuristic's candidates for one vcg_gemm-shaped
// library GEMM on the caller's operands, each `reps` times on `stream` (D written, C read when beta != 0: pass scratch
// buffers). us[i] = average microseconds of candidate i (-1: the candidate failed). Returns the number of candidates.
VCG_API int vcg_lt_tune(int transA, int transB, int M, int N, int K, const void* A, long long lda, const void* B,
                        long long ldb, const void* C, long long ldc, void* D, long long ldd, int d_f32,
                        const float* bias, float beta, int reps, float* us, int max_out, hipStream_t stream) {
  // build (or find) the plan with one real call
  int rc = lt_gemm(transA, transB, M, N, K, A, lda, B, ldb, C, ldc, D, ldd, d_f32, bias, beta, stream);
  if (rc != VCG_OK) return rc;
  LtState& st = lt_state();
  int dev = 0;
  VCG_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(st.mu);
  const bool has_c = C != nullptr && beta != 0.f;
  LtPlan& p = st.plans[std::make_tuple(dev, transA, transB, M, N, K, lda, ldb, has_c ? ldc : 0LL, ldd, d_f32,
                                       bias != nullptr ? 1 : 0, has_c ? 1 : 0)];
  void* w = st.ws[{dev, stream}];
  hipEvent_t e0, e1;
  VCG_CHECK_HIP(hipEventCreate(&e0));
  VCG_CHECK_HIP(hipEventCreate(&e1));
  const int n = (int)p.cands.size() < max_out ? (int)p.cands.size() : max_out;
  const float alpha = 1.f, b = has_c ? beta : 0.f;
  for (int i = 0; i < n; ++i) {
    bool ok = hipblasLtMatmul(st.handle[dev], p.desc, &alpha, B, p.la, A, p.lb, &b, has_c ? C : D, p.lc, D, p.ld,
                              &p.cands[i], w, LT_WS, stream) == HIPBLAS_STATUS_SUCCESS;  // warm-up
    VCG_CHECK_HIP(hipEventRecord(e0, stream));
    for (int r = 0; ok && r < reps; ++r)
      ok = hipblasLtMatmul(st.handle[dev], p.desc, &alpha, B, p.la, A, p.lb, &b, has_c ? C : D, p.lc, D, p.ld,
                           &p.cands[i], w, LT_WS, stream) == HIPBLAS_STATUS_SUCCESS;
    VCG_CHECK_HIP(hipEventRecord(e1, stream));
    VCG_CHECK_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    VCG_CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
    us[i] = ok ? ms * 1000.f / reps : -1.f;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return n;
}
