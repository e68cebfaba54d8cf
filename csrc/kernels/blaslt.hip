// hipBLASLt GEMMs with fused epilogues, called directly (host code; the GEMM kernels are hipBLASLt's).
//
// What this build of hipBLASLt offers on gfx950 was probed per epilogue (scripts/bench_lt_epilogues.py,
// profiles/r2_hipblaslt_epilogue_probe.txt): BIAS, GELU_BIAS and BGRADB (B transposed) have algorithms;
// GELU_AUX_BIAS, DGELU and DGELU_BGRAD have none -- so the transformer MLP keeps the framework's own bias-GELU
// kernels, and what moves into the GEMM is the bias gradient of every biased Linear:
//   dW = dY^T X with BGRADB  ->  db = colsum(dY) reduced in the same GEMM, dY read once
// (replacing the 2-launch column-sum the backward otherwise runs per biased Linear).
//
// Row-major [N, K] = dY[M, N]^T X[M, K] is the column-major product D[K, N] = op(A) op(B) with A = X
// (column-major [K, M], op N) and B = dY (column-major [N, M], op T); the bias gradient runs along n = N.
// Plans (descriptors + the algorithm) are cached per shape; the first call of a shape outside graph capture
// times up to 8 (plain / bias: 16) heuristic candidates and keeps the fastest.  Workspace: one 64 MiB device buffer per device.
// The library resolves at run time to the libhipblaslt.so.1 torch already mapped (same soname).
#include "common.h"
#include <hipblaslt/hipblaslt.h>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

using namespace pdt;

namespace {

constexpr size_t WS_BYTES = 64ull << 20;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool tuned = false;
  std::vector<hipblasLtMatmulHeuristicResult_t> cands;
};

struct State {
  hipblasLtHandle_t handle = nullptr;
  void* ws = nullptr;
  std::map<std::tuple<int, int, int64_t, int64_t, int64_t, int, int, int>, Plan> plans;   // (..., C given)
};

std::mutex g_mu;
std::map<int, State> g_state;   // per device

State* state_for_device(int& err) {
  int dev = 0;
  err = (int)hipGetDevice(&dev);
  if (err) return nullptr;
  State& s = g_state[dev];
  if (!s.handle) {
    if (hipblasLtCreate(&s.handle) != HIPBLAS_STATUS_SUCCESS) { err = -1; return nullptr; }
    err = (int)hipMalloc(&s.ws, WS_BYTES);
    if (err) return nullptr;
  }
  return &s;
}

hipDataType dt_of(int code) { return code == kF32 ? HIP_R_32F : HIP_R_16BF; }

#define LT_CHECK(x)                                 \
  do {                                              \
    if ((x) != HIPBLAS_STATUS_SUCCESS) return -2;   \
  } while (0)

// epilogue: 0 none, 1 bias, 2 gelu_aux_bias, 3 dgelu_bgrad, 4 gelu_bias, 5 dgelu, 6 bgradb (bias gradient
// of B reduced over k, written to the bias pointer -- the weight-gradient GEMM's fused bias gradient),
// 7 bgrada.  transA / transB: bit 0 / bit 1 of `trans`.
// aux_dt < 0: leave the aux type unset (hipBLASLt then uses D's type)
int build(Plan& p, hipblasLtHandle_t h, int epi, int trans, int64_t m, int64_t n, int64_t k, int io_dt, int bias_dt,
          int aux_dt = kBF16) {
  const int transA = trans & 1, transB = (trans >> 1) & 1;
  const hipblasOperation_t opA = transA ? HIPBLAS_OP_T : HIPBLAS_OP_N, opB = transB ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)));
  hipblasLtEpilogue_t e = HIPBLASLT_EPILOGUE_DEFAULT;
  if (epi == 1) e = HIPBLASLT_EPILOGUE_BIAS;
  if (epi == 2) e = HIPBLASLT_EPILOGUE_GELU_AUX_BIAS;
  if (epi == 3) e = HIPBLASLT_EPILOGUE_DGELU_BGRAD;
  if (epi == 4) e = HIPBLASLT_EPILOGUE_GELU_BIAS;
  if (epi == 5) e = HIPBLASLT_EPILOGUE_DGELU;
  if (epi == 6) e = HIPBLASLT_EPILOGUE_BGRADB;
  if (epi == 7) e = HIPBLASLT_EPILOGUE_BGRADA;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
  if (epi != 0 && epi != 5) {
    const hipDataType bt = dt_of(bias_dt);
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (epi == 2 || epi == 3 || epi == 5) {
    const int64_t ld = m;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    if (aux_dt >= 0) {
      const hipDataType at = dt_of(aux_dt);
      LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
    }
  }
  const hipDataType t = dt_of(io_dt);
  // A: op(A) is m x k; stored column-major [k, m] (transA) or [m, k]
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.a, t, transA ? k : m, transA ? m : k, transA ? k : m));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.b, t, transB ? n : k, transB ? k : n, transB ? n : k));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.d, t, m, n, m));
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsb = WS_BYTES;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  // plain / bias GEMMs (ops.linear's NT products) time a wider candidate list than the fused-epilogue ones
  const int want = (epi == 0 || epi == 1) ? 16 : 8;
  p.cands.resize(want);
  int got = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.d, p.d, pref, want, p.cands.data(),
                                                              &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || got <= 0) return -3;   // epilogue / type combination not supported
  p.cands.resize(got);
  p.algo = p.cands[0].algo;
  p.ws = p.cands[0].workspaceSize;
  return 0;
}

// C (optional, same layout as D, never D itself): D = op(A) op(B) + C, the accumulate input read in the kernel's
// epilogue (beta = 1) -- a residual stream added where the GEMM writes its output
int run(State& s, Plan& p, const hipblasLtMatmulAlgo_t& algo, size_t ws, const void* A, const void* B, void* D,
        hipStream_t st, const void* C = nullptr) {
  const float alpha = 1.f, beta = C ? 1.f : 0.f;
  return hipblasLtMatmul(s.handle, p.desc, &alpha, A, p.a, B, p.b, &beta, C ? C : D, p.d, D, p.d, &algo, s.ws, ws,
                         st) == HIPBLAS_STATUS_SUCCESS ? 0 : -4;
}

}  // namespace

// D[n_cols=n, rows=m] (column-major) = op(A) B with the given epilogue; see the header comment for the
// row-major mapping.  bias: epilogue 1/2 input [m], epilogue 3 output (bias gradient) [m].  aux: epilogue 2
// output / epilogue 3 input, same layout as D.  Returns 0, a hipError_t, or a negative hipBLASLt code
// (-3: no algorithm for this epilogue/type combination -- the caller falls back to separate kernels).
static int lt_matmul_impl(int epilogue, int trans, int64_t m, int64_t n, int64_t k, const void* A, const void* B,
                          const void* C, void* D, void* bias, int bias_dt, void* aux, int io_dt, int tune,
                          hipStream_t st) {
  std::lock_guard<std::mutex> g(g_mu);
  int err = 0;
  State* s = state_for_device(err);
  if (!s) return err ? err : -1;
  if (C && (C == D || (epilogue != 0 && epilogue != 1))) return (int)hipErrorInvalidValue;
  const auto key = std::make_tuple(epilogue, trans, m, n, k, io_dt, bias_dt, C ? 1 : 0);
  auto it = s->plans.find(key);
  if (it == s->plans.end()) {
    Plan p;
    const int rc = build(p, s->handle, epilogue, trans, m, n, k, io_dt, bias_dt);
    if (rc) return rc;
    it = s->plans.emplace(key, p).first;
  }
  Plan& p = it->second;
  if (epilogue != 0 && epilogue != 5) {
    if (hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
        HIPBLAS_STATUS_SUCCESS) return -2;
  }
  if (epilogue == 2 || epilogue == 3 || epilogue == 5) {
    if (hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)) !=
        HIPBLAS_STATUS_SUCCESS) return -2;
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  hipStreamIsCapturing(st, &cap);
  if (tune && !p.tuned && cap == hipStreamCaptureStatusNone && p.cands.size() > 1) {
    // time every candidate (3 reps after one warm-up) on this stream; the outputs are recomputed below
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (auto& c : p.cands) {
      if (c.workspaceSize > WS_BYTES) continue;
      if (run(*s, p, c.algo, c.workspaceSize, A, B, D, st, C)) continue;
      hipEventRecord(e0, st);
      for (int r = 0; r < 3; ++r) run(*s, p, c.algo, c.workspaceSize, A, B, D, st, C);
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) {
        best = ms;
        p.algo = c.algo;
        p.ws = c.workspaceSize;
      }
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    p.tuned = true;
  }
  const int rc = run(*s, p, p.algo, p.ws, A, B, D, st, C);
  if (rc) return rc;
  return (int)hipGetLastError();
}

PDT_API int pdt_lt_matmul(int epilogue, int trans, int64_t m, int64_t n, int64_t k, const void* A, const void* B,
                          void* D, void* bias, int bias_dt, void* aux, int io_dt, int tune, hipStream_t st) {
  return lt_matmul_impl(epilogue, trans, m, n, k, A, B, nullptr, D, bias, bias_dt, aux, io_dt, tune, st);
}

// The same with an accumulate input: D = op(A) op(B) (+ bias) + C, C a distinct buffer of D's layout (epilogue
// 0 or 1 only) -- e.g. a projection GEMM that adds the residual stream as it writes.
PDT_API int pdt_lt_matmul_c(int epilogue, int trans, int64_t m, int64_t n, int64_t k, const void* A, const void* B,
                            const void* C, void* D, void* bias, int bias_dt, int io_dt, int tune, hipStream_t st) {
  return lt_matmul_impl(epilogue, trans, m, n, k, A, B, C, D, bias, bias_dt, nullptr, io_dt, tune, st);
}

// Diagnostics: number of heuristic algorithms hipBLASLt offers for a combination (<0: descriptor error).
PDT_API int pdt_lt_probe(int epilogue, int trans, int64_t m, int64_t n, int64_t k, int io_dt, int bias_dt, int aux_dt) {
  std::lock_guard<std::mutex> g(g_mu);
  int err = 0;
  State* s = state_for_device(err);
  if (!s) return err ? -100 - err : -100;
  Plan p;
  const int rc = build(p, s->handle, epilogue, trans, m, n, k, io_dt, bias_dt, aux_dt);
  const int n_algos = rc == 0 ? (int)p.cands.size() : rc;
  if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
  if (p.a) hipblasLtMatrixLayoutDestroy(p.a);
  if (p.b) hipblasLtMatrixLayoutDestroy(p.b);
  if (p.d) hipblasLtMatrixLayoutDestroy(p.d);
  return n_algos;
}
