// hipBLASLt GEMMs with an in-process per-shape algorithm search and optional epilogues (gfx950).
//
// Used by ops/linear.py's per-shape library selection (VCX_GEMM_SELECT=1) and by the probes in
// scripts/. Measured on this image's hipBLASLt (scripts/lt_probe3.py): BIAS / GELU / GELU_BIAS /
// DGELU have bf16 algorithms at the GPT-2 MLP shapes, GELU_AUX(_BIAS) / DGELU_BGRAD / BGRADB do
// not, and DGELU does not compute the tanh-GELU derivative the model needs — so the MLP keeps its
// GEMM + HIP bias-GELU kernels, and the selection layer stays opt-in (A/B: no in-step gain).
//
// Row-major API: out[M, N] = alpha * op(A) op(B) (+ beta * out) with A [M, K] ([K, M] if trans_a)
// and B [K, N] ([N, K] if trans_b). hipBLASLt is column-major, so the call is issued as
// out^T = op(B)^T op(A)^T: matA = B, matB = A, m = N, n = M; the "bias" vector has length N.
//
// Algorithm choice: for each (shape, layout, epilogue) key the top heuristic candidates are timed
// on the caller's stream the first time the key is seen outside graph capture (on scratch
// outputs, so an accumulating output is never clobbered) and the fastest is cached; a key first
// seen DURING capture takes the heuristic's first choice.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

#define LT_CHECK(expr)                                                                              \
  do {                                                                                              \
    hipblasStatus_t st_ = (expr);                                                                   \
    TORCH_CHECK(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: ", #expr, " failed (", (int)st_, ")"); \
  } while (0)

#define HIP_CHECK(expr)                                                                 \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    TORCH_CHECK(e_ == hipSuccess, "HIP: ", #expr, " failed: ", hipGetErrorString(e_)); \
  } while (0)

constexpr size_t kWorkspace = 64ull << 20;
constexpr int kMaxDev = 16;

struct Choice {
  hipblasLtMatmulAlgo_t algo;
  bool tuned;
  float ms;
};

struct DevState {
  hipblasLtHandle_t handle = nullptr;
  void* ws = nullptr;
  std::unordered_map<std::string, Choice> cache;
};

std::mutex g_mu;
DevState g_dev[kMaxDev];

DevState& dev_state() {
  int d = 0;
  HIP_CHECK(hipGetDevice(&d));
  TORCH_CHECK(d >= 0 && d < kMaxDev);
  DevState& s = g_dev[d];
  if (!s.handle) {
    LT_CHECK(hipblasLtCreate(&s.handle));
    HIP_CHECK(hipMalloc(&s.ws, kWorkspace));
  }
  return s;
}

// RAII holder for the per-call descriptors
struct Desc {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  ~Desc() {
    if (a) hipblasLtMatrixLayoutDestroy(a);
    if (b) hipblasLtMatrixLayoutDestroy(b);
    if (c) hipblasLtMatrixLayoutDestroy(c);
    if (op) hipblasLtMatmulDescDestroy(op);
  }
  void set_ptr(hipblasLtMatmulDescAttributes_t attr, void* p) {
    LT_CHECK(hipblasLtMatmulDescSetAttribute(op, attr, &p, sizeof(p)));
  }
};

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  HIP_CHECK(hipStreamIsCapturing(s, &st));
  return st != hipStreamCaptureStatusNone;
}

int tune_candidates() {
  const char* e = std::getenv("VCX_LT_TUNE");
  return e ? std::max(1, std::atoi(e)) : 24;  // 1: heuristic first choice only
}

bool is_dgelu(hipblasLtEpilogue_t e) { return e == HIPBLASLT_EPILOGUE_DGELU || e == HIPBLASLT_EPILOGUE_DGELU_BGRAD; }

// out = alpha op(a) op(b) + beta out [+ epilogue]. Returns false (and launches nothing) if
// hipBLASLt has no algorithm for this epilogue/layout, so the caller can take the unfused path.
bool lt_matmul(at::Tensor a, at::Tensor b, at::Tensor out, bool trans_a, bool trans_b, int64_t epilogue,
               c10::optional<at::Tensor> bias, c10::optional<at::Tensor> aux, double alpha, double beta) {
  for (const at::Tensor* t : {&a, &b, &out}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 2 && t->is_contiguous(),
                "lt_matmul: a, b, out must be contiguous 2-D bf16 GPU tensors");
  }
  const int64_t M = trans_a ? a.size(1) : a.size(0);
  const int64_t K = trans_a ? a.size(0) : a.size(1);
  const int64_t Kb = trans_b ? b.size(1) : b.size(0);
  const int64_t N = trans_b ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "lt_matmul: inner dimensions differ (", K, " vs ", Kb, ")");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "lt_matmul: out must be [M, N]");
  const auto epi = (hipblasLtEpilogue_t)epilogue;
  const bool want_bias = epi == HIPBLASLT_EPILOGUE_BIAS || epi == HIPBLASLT_EPILOGUE_GELU_BIAS ||
                         epi == HIPBLASLT_EPILOGUE_GELU_AUX_BIAS || epi == HIPBLASLT_EPILOGUE_RELU_BIAS ||
                         epi == HIPBLASLT_EPILOGUE_DGELU_BGRAD;
  const bool want_aux = epi == HIPBLASLT_EPILOGUE_GELU_AUX || epi == HIPBLASLT_EPILOGUE_GELU_AUX_BIAS || is_dgelu(epi);
  TORCH_CHECK(want_bias == bias.has_value(), "lt_matmul: epilogue ", epilogue, " bias mismatch");
  TORCH_CHECK(want_aux == aux.has_value(), "lt_matmul: epilogue ", epilogue, " aux mismatch");
  hipDataType bias_type = HIP_R_16BF;
  if (bias.has_value()) {
    TORCH_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->numel() == N, "lt_matmul: bias must be [N]");
    TORCH_CHECK(bias->scalar_type() == at::kBFloat16 || bias->scalar_type() == at::kFloat);
    bias_type = bias->scalar_type() == at::kFloat ? HIP_R_32F : HIP_R_16BF;
  }
  if (aux.has_value()) {
    TORCH_CHECK(aux->is_cuda() && aux->is_contiguous() && aux->scalar_type() == at::kBFloat16 && aux->dim() == 2 &&
                    aux->size(0) == M && aux->size(1) == N,
                "lt_matmul: aux must be a contiguous bf16 [M, N] tensor");
  }

  hipStream_t stream = c10::hip::getCurrentHIPStream().stream();
  std::lock_guard<std::mutex> lock(g_mu);
  DevState& st = dev_state();

  Desc d;
  LT_CHECK(hipblasLtMatmulDescCreate(&d.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t opA = trans_b ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // matA = b
  const hipblasOperation_t opB = trans_a ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // matB = a
  LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (bias.has_value()) {
    d.set_ptr(HIPBLASLT_MATMUL_DESC_BIAS_POINTER, bias->data_ptr());
    LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bias_type,
                                             sizeof(bias_type)));
  }
  if (aux.has_value()) {
    const int64_t ld = N;
    d.set_ptr(HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, aux->data_ptr());
    LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
  }
  // stored (pre-op) column-major shapes: a row-major [r, c] tensor is column-major [c, r], ld c
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.a, HIP_R_16BF, b.size(1), b.size(0), b.size(1)));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.b, HIP_R_16BF, a.size(1), a.size(0), a.size(1)));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.c, HIP_R_16BF, N, M, N));

  const float fa = (float)alpha, fb = (float)beta;
  const std::string key = std::to_string(M) + "," + std::to_string(N) + "," + std::to_string(K) + "," +
                          std::to_string((int)trans_a) + std::to_string((int)trans_b) + "," + std::to_string(epilogue) +
                          "," + std::to_string((int)bias_type) + "," + std::to_string((int)(fb != 0.f));
  auto it = st.cache.find(key);
  const bool cap = capturing(stream);
  if (it == st.cache.end() || (!it->second.tuned && !cap)) {
    hipblasLtMatmulPreference_t pref;
    LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
    const uint64_t wsz = kWorkspace;
    LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz,
                                                   sizeof(wsz)));
    const int want = tune_candidates();
    std::vector<hipblasLtMatmulHeuristicResult_t> res(want);
    int got = 0;
    hipblasStatus_t hs =
        hipblasLtMatmulAlgoGetHeuristic(st.handle, d.op, d.a, d.b, d.c, d.c, pref, want, res.data(), &got);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (hs != HIPBLAS_STATUS_SUCCESS || got == 0) return false;
    Choice best{res[0].algo, false, 0.f};
    if (!cap && want > 1) {
      // time every candidate into scratch outputs (aux/bias outputs too; DGELU's aux is an input)
      at::Tensor o2 = at::empty_like(out);
      at::Tensor aux2, bias2;
      if (aux.has_value()) {
        aux2 = is_dgelu(epi) ? *aux : at::empty_like(*aux);
        d.set_ptr(HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, aux2.data_ptr());
      }
      if (bias.has_value()) {
        bias2 = epi == HIPBLASLT_EPILOGUE_DGELU_BGRAD ? at::empty_like(*bias) : *bias;
        d.set_ptr(HIPBLASLT_MATMUL_DESC_BIAS_POINTER, bias2.data_ptr());
      }
      if (fb != 0.f) o2.zero_();
      hipEvent_t e0, e1;
      HIP_CHECK(hipEventCreate(&e0));
      HIP_CHECK(hipEventCreate(&e1));
      float best_ms = 1e30f;
      for (int i = 0; i < got; ++i) {
        if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > kWorkspace) continue;
        auto run = [&]() {
          return hipblasLtMatmul(st.handle, d.op, &fa, b.data_ptr(), d.a, a.data_ptr(), d.b, &fb, o2.data_ptr(), d.c,
                                 o2.data_ptr(), d.c, &res[i].algo, st.ws, kWorkspace, stream);
        };
        if (run() != HIPBLAS_STATUS_SUCCESS) continue;  // warm-up + validity
        const int reps = 3;
        bool ok = true;
        HIP_CHECK(hipEventRecord(e0, stream));
        for (int r = 0; r < reps && ok; ++r) ok = run() == HIPBLAS_STATUS_SUCCESS;
        HIP_CHECK(hipEventRecord(e1, stream));
        HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ok && ms < best_ms) {
          best_ms = ms;
          best = Choice{res[i].algo, true, ms / reps};
        }
      }
      HIP_CHECK(hipEventDestroy(e0));
      HIP_CHECK(hipEventDestroy(e1));
      if (aux.has_value()) d.set_ptr(HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, aux->data_ptr());
      if (bias.has_value()) d.set_ptr(HIPBLASLT_MATMUL_DESC_BIAS_POINTER, bias->data_ptr());
      if (!best.tuned) return false;  // no candidate ran
    }
    it = st.cache.insert_or_assign(key, best).first;
  }
  LT_CHECK(hipblasLtMatmul(st.handle, d.op, &fa, b.data_ptr(), d.a, a.data_ptr(), d.b, &fb, out.data_ptr(), d.c,
                           out.data_ptr(), d.c, &it->second.algo, st.ws, kWorkspace, stream));
  return true;
}

// {key: tuned time in ms (-1: untuned heuristic choice)} of every cached choice on this device
std::unordered_map<std::string, double> lt_tuned() {
  std::lock_guard<std::mutex> lock(g_mu);
  int d = 0;
  HIP_CHECK(hipGetDevice(&d));
  std::unordered_map<std::string, double> r;
  for (auto& kv : g_dev[d].cache) r[kv.first] = kv.second.tuned ? kv.second.ms : -1.0;
  return r;
}

}  // namespace

void vcx_register_lt(pybind11::module& m) {
  m.def("lt_matmul", &lt_matmul, "hipBLASLt GEMM with a fused epilogue (row-major API)", pybind11::arg("a"),
        pybind11::arg("b"), pybind11::arg("out"), pybind11::arg("trans_a"), pybind11::arg("trans_b"),
        pybind11::arg("epilogue"), pybind11::arg("bias") = pybind11::none(), pybind11::arg("aux") = pybind11::none(),
        pybind11::arg("alpha") = 1.0, pybind11::arg("beta") = 0.0);
  m.def("lt_tuned", &lt_tuned);
  m.attr("LT_EPI_DEFAULT") = (int)HIPBLASLT_EPILOGUE_DEFAULT;
  m.attr("LT_EPI_BIAS") = (int)HIPBLASLT_EPILOGUE_BIAS;
  m.attr("LT_EPI_GELU_AUX_BIAS") = (int)HIPBLASLT_EPILOGUE_GELU_AUX_BIAS;
  m.attr("LT_EPI_DGELU") = (int)HIPBLASLT_EPILOGUE_DGELU;
  m.attr("LT_EPI_DGELU_BGRAD") = (int)HIPBLASLT_EPILOGUE_DGELU_BGRAD;
}
