// Torch bindings for the gfx950 kernels. Every entry point validates shapes/dtypes on the
// host (a wrong shape must never reach a hand-written kernel: an out-of-bounds access can
// reset the whole node) and launches on the caller's current HIP stream, so the ops compose
// with torch streams and hipGraph capture.
#include <torch/extension.h>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "kernels/vcx_api.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DT(x, dt) TORCH_CHECK((x).scalar_type() == (dt), #x " has wrong dtype ", (x).scalar_type())
#define CHECK_IN(x, dt) \
  CHECK_CUDA(x);        \
  CHECK_CONTIG(x);      \
  CHECK_DT(x, dt)

const auto kBF = at::kBFloat16;
const auto kF = at::kFloat;

void* opt_ptr(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// ------------------------------------------------------------------ optimizer / local SGD
void grad_sumsq(at::Tensor g, at::Tensor ostate) {
  CHECK_IN(g, kBF);
  CHECK_IN(ostate, kF);
  TORCH_CHECK(g.numel() % 8 == 0, "flat buffer length must be a multiple of 8");
  vcx_grad_sumsq(g.data_ptr(), g.numel(), ostate.data_ptr<float>(), cur_stream());
}

void adam_prologue(at::Tensor ostate, double max_norm) {
  CHECK_IN(ostate, kF);
  TORCH_CHECK(ostate.numel() >= 4);
  vcx_adam_prologue(ostate.data_ptr<float>(), (float)max_norm, cur_stream());
}

void adamw_flat(at::Tensor param, at::Tensor grad, at::Tensor master, at::Tensor m, at::Tensor v, int64_t n_decay,
                at::Tensor ostate, double beta1, double beta2, double eps, double wd) {
  CHECK_IN(param, kBF);
  CHECK_IN(grad, kBF);
  CHECK_IN(master, kF);
  CHECK_IN(m, kF);
  CHECK_IN(v, kF);
  CHECK_IN(ostate, kF);
  const int64_t n = param.numel();
  TORCH_CHECK(n % 8 == 0 && grad.numel() == n && master.numel() == n && m.numel() == n && v.numel() == n,
              "adamw_flat: buffers must share a length that is a multiple of 8");
  TORCH_CHECK(n_decay >= 0 && n_decay <= n && n_decay % 8 == 0);
  vcx_adamw_flat(param.data_ptr(), grad.data_ptr(), master.data_ptr<float>(), m.data_ptr<float>(),
                 v.data_ptr<float>(), n, n_decay, ostate.data_ptr<float>(), (float)beta1, (float)beta2, (float)eps,
                 (float)wd, cur_stream());
}

void lsgd_delta(at::Tensor master, at::Tensor anchor, at::Tensor delta) {
  CHECK_IN(master, kF);
  CHECK_IN(anchor, kF);
  CHECK_IN(delta, kBF);
  const int64_t n = master.numel();
  TORCH_CHECK(n % 8 == 0 && anchor.numel() == n && delta.numel() == n);
  vcx_lsgd_delta(master.data_ptr<float>(), anchor.data_ptr<float>(), delta.data_ptr(), n, cur_stream());
}

void lsgd_apply(at::Tensor avg, at::Tensor anchor, at::Tensor master, at::Tensor param,
                c10::optional<at::Tensor> mom, double outer_lr, double mu, bool nesterov, double avg_scale) {
  CHECK_IN(avg, kBF);
  CHECK_IN(anchor, kF);
  CHECK_IN(master, kF);
  CHECK_IN(param, kBF);
  const int64_t n = avg.numel();
  TORCH_CHECK(n % 8 == 0 && anchor.numel() == n && master.numel() == n && param.numel() == n);
  if (mom.has_value()) {
    CHECK_IN((*mom), kF);
    TORCH_CHECK(mom->numel() == n);
  }
  vcx_lsgd_apply(avg.data_ptr(), anchor.data_ptr<float>(), master.data_ptr<float>(), param.data_ptr(),
                 mom.has_value() ? mom->data_ptr<float>() : nullptr, n, (float)outer_lr, (float)mu, nesterov ? 1 : 0,
                 (float)avg_scale, cur_stream());
}

void f32_to_bf16(at::Tensor src, at::Tensor dst) {
  CHECK_IN(src, kF);
  CHECK_IN(dst, kBF);
  TORCH_CHECK(src.numel() == dst.numel() && src.numel() % 8 == 0);
  vcx_f32_to_bf16(src.data_ptr<float>(), dst.data_ptr(), src.numel(), cur_stream());
}

// ---------------------------------------------------------------- hand-written MFMA GEMM (gemm.hip)
// C[M, N] = A[M, K] . B[N, K]^T with epilogue: 0 store, 1 +bias, 2 +bias -> (C = pre, C2 = gelu(pre)),
// 3 C = acc * gelu'(C2) with fp32 column sums added into `colsum` (must be zeroed by the caller)
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K) { return vcx_gemm_nt_supported((int)M, (int)N, (int)K); }
bool gemm_nt_supported_epi(int64_t M, int64_t N, int64_t K, int64_t epi) {
  return vcx_gemm_nt_supported_epi((int)M, (int)N, (int)K, (int)epi);
}

void gemm_nt(at::Tensor a, at::Tensor b, at::Tensor c, c10::optional<at::Tensor> c2, c10::optional<at::Tensor> bias,
             c10::optional<at::Tensor> colsum, int64_t epi) {
  TORCH_CHECK(a.is_cuda() && a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "gemm_nt: 2-D cuda tensors");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && c.scalar_type() == at::kBFloat16,
              "gemm_nt: bf16 operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1, "gemm_nt: K-contiguous rows");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && c.size(0) == M && c.size(1) == N, "gemm_nt: shape mismatch");
  TORCH_CHECK(vcx_gemm_nt_supported_epi((int)M, (int)N, (int)K, (int)epi),
              "gemm_nt: needs N % 256 == 0, K % 64 == 0, K >= 128, and M % 256 == 0 for epilogues 2/3");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && c.stride(0) % 8 == 0, "gemm_nt: 16-B aligned rows");
  // the kernel moves 16 B per lane: a column-offset view (e.g. c[:, 4:260]) would be misaligned
  for (const at::Tensor* t : {&a, &b, &c})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_nt: 16-B aligned base pointers");
  TORCH_CHECK(epi >= 0 && epi <= 4, "gemm_nt: epilogue 0..4");
  void* c2p = nullptr;
  if (epi == 2 || epi == 3) {
    TORCH_CHECK(c2 && c2->sizes() == c.sizes() && c2->strides() == c.strides() && c2->scalar_type() == at::kBFloat16,
                "gemm_nt: epilogue 2/3 needs c2 like c");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(c2->data_ptr()) % 16 == 0, "gemm_nt: 16-B aligned c2");
    c2p = c2->data_ptr();
  }
  const void* bp = nullptr;
  if (epi == 1 || epi == 2 || epi == 4) {
    TORCH_CHECK(bias && bias->numel() == N && bias->is_contiguous() && bias->scalar_type() == at::kBFloat16,
                "gemm_nt: bias [N] bf16");
    bp = bias->data_ptr();
  }
  float* cs = nullptr;
  if (epi == 3) {
    TORCH_CHECK(colsum && colsum->numel() == N && colsum->scalar_type() == at::kFloat && colsum->is_contiguous(),
                "gemm_nt: colsum [N] fp32");
    cs = colsum->data_ptr<float>();
  }
  vcx_gemm_nt(a.data_ptr(), b.data_ptr(), c.data_ptr(), c2p, bp, cs, (int)M, (int)N, (int)K, (int)a.stride(0),
              (int)b.stride(0), (int)c.stride(0), (int)epi, cur_stream());
}


// Persistent store-overlapped GEMM (gemm_ps.hip): c[M, N] = a[M, K] . b[N, K]^T with epilogue
// 0 store, 1 +bias, 2 +bias -> (c = pre, c2 = gelu(pre)); grid_cap <= 0: one workgroup per CU
bool gemm_ps_supported(int64_t M, int64_t N, int64_t K, int64_t epi) {
  return vcx_gemm_ps_supported((int)M, (int)N, (int)K, (int)epi);
}

void gemm_ps(at::Tensor a, at::Tensor b, at::Tensor c, c10::optional<at::Tensor> c2, c10::optional<at::Tensor> bias,
             c10::optional<at::Tensor> colsum, int64_t epi, int64_t grid_cap) {
  TORCH_CHECK(a.is_cuda() && a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "gemm_ps: 2-D cuda tensors");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && c.scalar_type() == at::kBFloat16,
              "gemm_ps: bf16 operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1, "gemm_ps: K-contiguous rows");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && c.size(0) == M && c.size(1) == N, "gemm_ps: shape mismatch");
  TORCH_CHECK(vcx_gemm_ps_supported((int)M, (int)N, (int)K, (int)epi),
              "gemm_ps: needs M, N % 256 == 0, K % 128 == 0, K >= 256, epilogue 0 (store), 1 (bias), 2 (bias+GELU), "
              "4 (DGELU + bias grad), 5 (bias+GELU, c = gelu'(pre)) or 6 (c = acc * c2 + bias grad), N <= 16384 with "
              "a bias");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && c.stride(0) % 8 == 0, "gemm_ps: 16-B aligned rows");
  for (const at::Tensor* t : {&a, &b, &c})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_ps: 16-B aligned base pointers");
  // buffer resources cover one 256-row panel each: 32-bit byte offsets
  TORCH_CHECK(256 * std::max({a.stride(0), b.stride(0), c.stride(0)}) * 2 < (int64_t(1) << 31), "gemm_ps: rows too long");
  void* c2p = nullptr;
  if (epi == 2 || epi == 4 || epi == 5 || epi == 6) {
    TORCH_CHECK(c2 && c2->sizes() == c.sizes() && c2->strides() == c.strides() && c2->scalar_type() == at::kBFloat16,
                "gemm_ps: epilogues 2/4/5/6 need c2 like c");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(c2->data_ptr()) % 16 == 0, "gemm_ps: 16-B aligned c2");
    c2p = c2->data_ptr();
  }
  const void* bp = nullptr;
  if (epi == 1 || epi == 2 || epi == 5) {
    TORCH_CHECK(bias && bias->numel() == N && bias->is_contiguous() && bias->scalar_type() == at::kBFloat16,
                "gemm_ps: bias [N] bf16");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(bias->data_ptr()) % 16 == 0, "gemm_ps: 16-B aligned bias");
    bp = bias->data_ptr();
  }
  float* cs = nullptr;
  if (epi == 4 || epi == 6) {
    TORCH_CHECK(colsum && colsum->numel() == N && colsum->scalar_type() == at::kFloat && colsum->is_contiguous(),
                "gemm_ps: colsum [N] fp32");
    cs = colsum->data_ptr<float>();
  }
  vcx_gemm_ps(a.data_ptr(), b.data_ptr(), c.data_ptr(), c2p, bp, cs, (int)M, (int)N, (int)K, (int)a.stride(0),
              (int)b.stride(0), (int)c.stride(0), (int)epi, (int)grid_cap, cur_stream());
}

// The zero-at-rest workspace of the BN kernels: fp32 [2C] atomic sums, zeroed once here and zeroed again
// by the finalize kernel of every call. Correct only while every stats -> finalize pair that uses one
// workspace runs back to back on its stream: launches on one stream are ordered, so the layers of a
// model can share it, but two host threads launching BN of the same width on the same stream could
// interleave their pairs (one finalize would read both sums). The cache is therefore keyed by the
// launching host thread as well: one workspace per (device, stream, C, thread). It must exist before a
// hipGraph capture that uses it (one eager step first, as every trainer here does): created inside a
// capture, its zero fill would only be a node of the graph, not done by the time eager calls use it.
static float* bn_workspace(const at::Tensor& x, int64_t C) {
  static std::mutex mu;
  // never destroyed: no device free during static destruction at interpreter exit
  static auto* cache = new std::map<std::tuple<int, uintptr_t, int64_t, size_t>, at::Tensor>();
  const auto key = std::make_tuple((int)x.get_device(), (uintptr_t)cur_stream(), C,
                                   std::hash<std::thread::id>{}(std::this_thread::get_id()));
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache->find(key);
  if (it == cache->end()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    TORCH_CHECK(hipStreamIsCapturing(cur_stream(), &cs) == hipSuccess && cs == hipStreamCaptureStatusNone,
                "bn: first call of this width on this stream/thread inside a graph capture; run one eager step first");
    it = cache->emplace(key, at::zeros({2 * C}, x.options().dtype(at::kFloat))).first;
  }
  return it->second.data_ptr<float>();
}

// Train-mode BatchNorm (+ residual) (+ ReLU) on NHWC bf16 activations (batchnorm.hip). x / res / y:
// contiguous [..., C] (the NHWC view of a channels-last tensor); gamma / beta bf16 [C]; running stats
// bf16 or fp32 [C], updated in place (skipped when undefined); nbt: the layer's num_batches_tracked
// (int64, incremented on the device) or None. Returns y, mean, rstd, scale (fp32 [C]) and, with the ReLU,
// its mask as one bit per element (uint8 [R, C / 8]: bit i of byte e = element 8 e + i is > 0), which
// the backward reads instead of y; undefined without the ReLU.
// layer_ws: the layer's own fp32 [4C] workspace [fwd sums | bwd sums] instead of the shared one; its
// forward half must be zero on entry (the caller's bookkeeping: ops/batchnorm.py) and the backward
// half is zeroed by this call (finalize inside the apply pass, batchnorm.hip apply_kernel FIN)
static float* check_layer_ws(const c10::optional<at::Tensor>& lws, const at::Tensor& x, int64_t C) {
  if (!lws || !lws->defined()) return nullptr;
  TORCH_CHECK(lws->is_cuda() && lws->get_device() == x.get_device() && lws->scalar_type() == at::kFloat &&
                  lws->is_contiguous() && lws->numel() == 4 * C, "bn: layer workspace fp32 [4C] on x's device");
  return lws->data_ptr<float>();
}

std::vector<at::Tensor> bn_fwd_train(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor gamma, at::Tensor beta,
                                     c10::optional<at::Tensor> run_mean, c10::optional<at::Tensor> run_var, double eps,
                                     double momentum, bool relu, c10::optional<at::Tensor> nbt,
                                     c10::optional<at::Tensor> layer_ws) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.scalar_type() == at::kBFloat16, "bn: x bf16 contiguous NHWC");
  const int64_t C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(vcx_bn_supported((int)C) && R > 0, "bn: C must be a power of two in 8..2048");
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && gamma.scalar_type() == at::kBFloat16 &&
                  beta.scalar_type() == at::kBFloat16 && gamma.is_contiguous() && beta.is_contiguous(), "bn: gamma/beta bf16 [C]");
  if (res) TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous() && res->scalar_type() == at::kBFloat16, "bn: residual like x");
  void *rm = nullptr, *rv = nullptr;
  int fp32 = 0;
  if (run_mean && run_mean->defined()) {
    TORCH_CHECK(run_var && run_mean->numel() == C && run_var->numel() == C && run_mean->is_contiguous() &&
                    run_var->is_contiguous() && run_mean->scalar_type() == run_var->scalar_type() &&
                    (run_mean->scalar_type() == at::kBFloat16 || run_mean->scalar_type() == at::kFloat), "bn: running stats [C]");
    rm = run_mean->data_ptr();
    rv = run_var->data_ptr();
    fp32 = run_mean->scalar_type() == at::kFloat;
  }
  int64_t* nb = nullptr;
  if (nbt && nbt->defined()) {
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1 && nbt->get_device() == x.get_device(),
                "bn: num_batches_tracked int64 [1] on x's device");
    nb = nbt->data_ptr<int64_t>();
  }
  auto f = x.options().dtype(at::kFloat);
  at::Tensor st = at::empty({4, C}, f);
  at::Tensor y = at::empty_like(x);
  at::Tensor mask = relu ? at::empty({R, C / 8}, x.options().dtype(at::kByte)) : at::Tensor();
  float* lws = check_layer_ws(layer_ws, x, C);
  vcx_bn_fwd_train(x.data_ptr(), res ? res->data_ptr() : nullptr, y.data_ptr(), relu ? mask.data_ptr() : nullptr, R,
                   (int)C, gamma.data_ptr(), beta.data_ptr(), rm, rv, fp32, (float)eps, (float)momentum,
                   lws ? lws : bn_workspace(x, C), st[0].data_ptr<float>(), st[1].data_ptr<float>(),
                   st[2].data_ptr<float>(), st[3].data_ptr<float>(), nb, relu ? 1 : 0, lws ? 1 : 0, cur_stream());
  return {y, st[0], st[1], st[2], mask};
}

// ResNet stem max-pool 3x3 / stride 2 / pad 1 on the NHWC view [N, H, W, C] (bf16, C % 8 == 0):
// returns y [N, OH, OW, C] and the uint8 window index of each output element
std::vector<at::Tensor> maxpool3s2_fwd(at::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous() && x.scalar_type() == at::kBFloat16 && x.size(3) % 8 == 0 &&
                  x.size(1) >= 1 && x.size(2) >= 1, "maxpool3s2: x bf16 contiguous NHWC, C % 8 == 0");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(N * H * W * C < (1ll << 40) && H < (1 << 20) && W < (1 << 20), "maxpool3s2: size");
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  at::Tensor y = at::empty({N, OH, OW, C}, x.options());
  at::Tensor idx = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  vcx_maxpool3s2_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)OH, (int)OW,
                     cur_stream());
  return {y, idx};
}

at::Tensor maxpool3s2_bwd(at::Tensor dy, at::Tensor idx, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.is_contiguous() && dy.scalar_type() == at::kBFloat16 &&
                  idx.sizes() == dy.sizes() && idx.is_contiguous() && idx.scalar_type() == at::kByte &&
                  idx.get_device() == dy.get_device() && dy.size(3) % 8 == 0, "maxpool3s2_bwd: dy bf16 / idx u8 NHWC alike");
  const int64_t N = dy.size(0), OH = dy.size(1), OW = dy.size(2), C = dy.size(3);
  TORCH_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1, "maxpool3s2_bwd: input size does not match");
  at::Tensor dx = at::empty({N, H, W, C}, dy.options());
  vcx_maxpool3s2_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)OH, (int)OW,
                     cur_stream());
  return dx;
}

static void nhwc_check(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.is_contiguous() && t.scalar_type() == at::kBFloat16 && t.size(3) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && t.numel() < (1ll << 40),
              what, ": bf16 contiguous NHWC [N, H, W, C], C % 8 == 0, 16-B aligned");
}

// x [N, H, W, C] -> x[:, ::s, ::s, :] contiguous
at::Tensor subsample_nhwc(at::Tensor x, int64_t s) {
  nhwc_check(x, "subsample_nhwc");
  TORCH_CHECK(s >= 1 && s <= 8, "subsample_nhwc: stride 1..8");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  at::Tensor y = at::empty({N, (H - 1) / s + 1, (W - 1) / s + 1, C}, x.options());
  if (y.numel()) vcx_subsample_nhwc(x.data_ptr(), y.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)s, cur_stream());
  return y;
}

// full[:, ::s, ::s, :] += g, in place
void subsample_add_nhwc(at::Tensor full, at::Tensor g, int64_t s) {
  nhwc_check(full, "subsample_add_nhwc");
  nhwc_check(g, "subsample_add_nhwc");
  TORCH_CHECK(s >= 1 && s <= 8 && full.get_device() == g.get_device(), "subsample_add_nhwc: stride 1..8, one device");
  const int64_t N = full.size(0), H = full.size(1), W = full.size(2), C = full.size(3);
  TORCH_CHECK(g.size(0) == N && g.size(1) == (H - 1) / s + 1 && g.size(2) == (W - 1) / s + 1 && g.size(3) == C,
              "subsample_add_nhwc: g must be [N, ceil(H / s), ceil(W / s), C]");
  if (g.numel()) vcx_subsample_add_nhwc(full.data_ptr(), g.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)s, cur_stream());
}

// g [N, C] -> out [N, H, W, C] = g[:, None, None, :] * scale
at::Tensor bcast_hw_nhwc(at::Tensor g, int64_t H, int64_t W, double scale) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() && g.scalar_type() == at::kBFloat16 && g.size(1) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0 && H >= 1 && W >= 1,
              "bcast_hw_nhwc: g bf16 contiguous [N, C], C % 8 == 0");
  const int64_t N = g.size(0), C = g.size(1);
  TORCH_CHECK(N * H * W * C < (1ll << 40), "bcast_hw_nhwc: size");
  at::Tensor out = at::empty({N, H, W, C}, g.options());
  if (out.numel()) vcx_bcast_hw_nhwc(g.data_ptr(), out.data_ptr(), (int)N, (int)(H * W), (int)C, (float)scale, cur_stream());
  return out;
}

at::Tensor bn_apply(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor scale, at::Tensor shift, bool relu) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.scalar_type() == at::kBFloat16, "bn: x bf16 contiguous NHWC");
  const int64_t C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(vcx_bn_supported((int)C), "bn: C must be a power of two in 8..2048");
  TORCH_CHECK(scale.numel() == C && shift.numel() == C && scale.scalar_type() == at::kFloat &&
                  shift.scalar_type() == at::kFloat && scale.is_contiguous() && shift.is_contiguous(), "bn: scale/shift fp32 [C]");
  if (res) TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous() && res->scalar_type() == at::kBFloat16, "bn: residual like x");
  at::Tensor y = at::empty_like(x);
  vcx_bn_apply(x.data_ptr(), res ? res->data_ptr() : nullptr, y.data_ptr(), R, (int)C, scale.data_ptr<float>(),
               shift.data_ptr<float>(), relu ? 1 : 0, cur_stream());
  return y;
}

// returns dx, d residual (undefined unless want_dres), dgamma, dbeta (fp32 [C])
// gw / gb: flat bf16 [C] gradient buffers of gamma / beta that dgamma / dbeta are ADDED into (both or
// neither); the returned dgamma / dbeta are then for information only. layer_ws: the forward's layer
// workspace (its backward half zero on entry; its forward half is zeroed by this call)
std::vector<at::Tensor> bn_bwd(at::Tensor dy, c10::optional<at::Tensor> mask, at::Tensor x, at::Tensor mean, at::Tensor rstd,
                               at::Tensor scale, bool relu, bool want_dres, c10::optional<at::Tensor> gw,
                               c10::optional<at::Tensor> gb, c10::optional<at::Tensor> layer_ws) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && x.is_contiguous() && dy.sizes() == x.sizes() &&
                  dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "bn_bwd: dy, x bf16 NHWC alike");
  const int64_t C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(relu == (mask && mask->defined()), "bn_bwd: the ReLU mask with relu (and only then)");
  if (relu)
    TORCH_CHECK(mask->is_cuda() && mask->is_contiguous() && mask->scalar_type() == at::kByte &&
                    mask->numel() * 8 == R * C && mask->get_device() == x.get_device(), "bn_bwd: mask uint8 [R, C / 8]");
  TORCH_CHECK(vcx_bn_supported((int)C), "bn: C must be a power of two in 8..2048");
  for (const at::Tensor* t : {&mean, &rstd, &scale})
    TORCH_CHECK(t->numel() == C && t->scalar_type() == at::kFloat && t->is_contiguous(), "bn_bwd: stats fp32 [C]");
  const bool flat = gw && gw->defined();
  TORCH_CHECK(flat == (gb && gb->defined()), "bn_bwd: gw and gb together");
  if (flat)
    for (const at::Tensor* t : {&*gw, &*gb})
      TORCH_CHECK(t->is_cuda() && t->get_device() == x.get_device() && t->numel() == C && t->is_contiguous() &&
                      t->scalar_type() == at::kBFloat16, "bn_bwd: gradient buffers bf16 [C]");
  at::Tensor sums = at::empty({2 * C}, x.options().dtype(at::kFloat));
  at::Tensor dx = at::empty_like(x);
  at::Tensor dres = want_dres ? at::empty_like(x) : at::Tensor();
  float* lws = check_layer_ws(layer_ws, x, C);
  vcx_bn_bwd(dy.data_ptr(), relu ? mask->data_ptr() : nullptr, x.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
             scale.data_ptr<float>(), R, (int)C, lws ? lws : bn_workspace(x, C), sums.data_ptr<float>(),
             flat ? gw->data_ptr() : nullptr, flat ? gb->data_ptr() : nullptr, dx.data_ptr(),
             want_dres ? dres.data_ptr() : nullptr, relu ? 1 : 0, lws ? 1 : 0, cur_stream());
  return {dx, dres, sums.narrow(0, C, C), sums.narrow(0, 0, C)};
}

// Weight gradient out[M, N] (+)= a[K, M]^T . b[K, N] (token-major operands) on the hand-written
// gemm_wg (csrc/kernels/gemm_wg.hip): split-K over the token axis with fp32 partials summed into out.
// splits <= 0: vcx_gemm_wg_splits; loaders: the waves that stage the LDS ring (8, or 4 with waves 4-7
// compute-only)
bool gemm_wg_supported(int64_t M, int64_t N, int64_t K, int64_t splits) {
  return vcx_gemm_wg_supported((int)M, (int)N, (int)K, (int)(splits > 0 ? splits : vcx_gemm_wg_splits((int)M, (int)N, (int)K)));
}

void gemm_wg(at::Tensor a, at::Tensor b, at::Tensor out, bool accumulate, int64_t splits, int64_t loaders) {
  TORCH_CHECK(a.is_cuda() && a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm_wg: 2-D cuda tensors");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
              "gemm_wg: bf16 operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.is_contiguous(), "gemm_wg: row-major operands, contiguous out");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K && out.size(0) == M && out.size(1) == N, "gemm_wg: shape mismatch");
  if (splits <= 0) splits = vcx_gemm_wg_splits((int)M, (int)N, (int)K);
  TORCH_CHECK(vcx_gemm_wg_supported((int)M, (int)N, (int)K, (int)splits),
              "gemm_wg: needs M % 128 == 0, N % 256 == 0, K % 64 == 0, K / 192 >= splits, split panels under 2 GB");
  TORCH_CHECK(loaders == 4 || loaders == 8, "gemm_wg: loaders 4 or 8");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm_wg: 16-B aligned rows");
  const int64_t tok = ((K / 64 + splits - 1) / splits) * 64;  // the longest split's token rows
  TORCH_CHECK(tok * std::max(a.stride(0), b.stride(0)) * 2 < (int64_t(1) << 31) - (int64_t(1) << 20),
              "gemm_wg: a split's operand panel must stay under 2 GB (more splits)");
  for (const at::Tensor* t : {&a, &b, &out})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_wg: 16-B aligned base pointers");
  at::Tensor ws = at::empty({splits, M, N}, a.options().dtype(at::kFloat));
  vcx_gemm_wg(a.data_ptr(), b.data_ptr(), ws.data_ptr<float>(), out.data_ptr(), (int)M, (int)N, (int)K,
              (int)a.stride(0), (int)b.stride(0), (int)splits, accumulate ? 1 : 0, (int)loaders, cur_stream());
}

// out[M, N] = a[M, K] . b[N, K]^T (+ bias[N]) on gemm_f (csrc/kernels/gemm_f.hip): 256 x 256 tiles, 4 waves of 128 x 128
bool gemm_f_supported(int64_t M, int64_t N, int64_t K) { return vcx_gemm_f_supported((int)M, (int)N, (int)K); }

// splits < 0: vcx_gemm_f_splits (one round of workgroups); the fp32 partials live in a temporary [splits, M, N]
static std::pair<int, at::Tensor> f_splits(int64_t M, int64_t N, int64_t K, int64_t splits, const at::Tensor& like) {
  if (splits < 0) splits = vcx_gemm_f_splits((int)M, (int)N, (int)K);
  if (splits == 0) splits = 1;
  TORCH_CHECK(vcx_gemm_f_split_ok((int)M, (int)N, (int)K, (int)splits),
              "gemm_f: the K slices (K / 32) must split into even counts >= 6");
  at::Tensor ws = splits > 1 ? at::empty({splits, M, N}, like.options().dtype(at::kFloat)) : at::Tensor();
  return {(int)splits, ws};
}

int64_t gemm_f_splits(int64_t M, int64_t N, int64_t K) { return vcx_gemm_f_splits((int)M, (int)N, (int)K); }

void gemm_f(at::Tensor a, at::Tensor b, at::Tensor out, c10::optional<at::Tensor> bias, int64_t waves, int64_t splits) {
  TORCH_CHECK(a.is_cuda() && a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm_f: 2-D cuda tensors");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
              "gemm_f: bf16 operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "gemm_f: row-major operands");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && out.size(0) == M && out.size(1) == N, "gemm_f: shape mismatch");
  TORCH_CHECK(vcx_gemm_f_supported((int)M, (int)N, (int)K), "gemm_f: needs N % 128 == 0 or N == 64, K % 64 == 0, K >= 192");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "gemm_f: 16-B aligned rows");
  for (const at::Tensor* t : {&a, &b, &out})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_f: 16-B aligned base pointers");
  TORCH_CHECK(a.get_device() == b.get_device() && a.get_device() == out.get_device(), "gemm_f: one device");
  const bool hb = bias && bias->defined();
  if (hb)
    TORCH_CHECK(bias->is_cuda() && bias->get_device() == a.get_device() && bias->numel() == N && bias->is_contiguous() &&
                    bias->scalar_type() == at::kBFloat16 && reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0,
                "gemm_f: bias bf16 [N], contiguous, 8-B aligned");
  TORCH_CHECK(256 * std::max(a.stride(0), b.stride(0)) * 2 < (int64_t(1) << 31), "gemm_f: tile panels under 2 GB");
  auto [ns, ws] = f_splits(M, N, K, splits, a);
  TORCH_CHECK(ns == 1 || out.stride(0) % 4 == 0, "gemm_f: split output rows 8-B aligned");
  vcx_gemm_f(a.data_ptr(), b.data_ptr(), out.data_ptr(), hb ? bias->data_ptr() : nullptr, (int)M, (int)N, (int)K, (int)a.stride(0), (int)b.stride(0),
             (int)out.stride(0), (int)waves, ns, ns > 1 ? ws.data_ptr<float>() : nullptr, cur_stream());
}

// 3x3 convolution (pad 1, stride 1|2) forward on gemm_f as an implicit GEMM: y[N, Ho, Wo, Cout] (+ bias) =
// conv(x[N, H, W, Cin], w[Cout][3][3][Cin]) with the patch matrix of x gathered by the LDS-DMA's per-lane offsets
bool gemm_f_conv3x3_supported(int64_t imgs, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int64_t stride) {
  return vcx_gemm_f_conv3x3_supported((int)imgs, (int)H, (int)W, (int)Cin, (int)Cout, (int)stride);
}

void gemm_f_conv3x3(at::Tensor x, at::Tensor w, at::Tensor out, int64_t stride, c10::optional<at::Tensor> bias,
                    int64_t waves, int64_t splits, bool flip_taps) {
  // w: [Cout, 3, 3, Cin], or tap-major [9, Cout, Cin] (the transpose of a channels-last weight matrix)
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && (w.dim() == 4 || w.dim() == 3) && out.dim() == 4,
              "gemm_f_conv3x3: x [N, H, W, Cin], w [Cout, 3, 3, Cin] or [9, Cout, Cin], out [N, Ho, Wo, Cout] on the GPU");
  for (const at::Tensor* t : {&x, &w, &out}) {
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->get_device() == x.get_device(),
                "gemm_f_conv3x3: contiguous bf16 tensors on one device");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_f_conv3x3: 16-B aligned base pointers");
  }
  const bool tap_major = w.dim() == 3;
  const int64_t imgs = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = tap_major ? w.size(1) : w.size(0);
  TORCH_CHECK(tap_major ? (w.size(0) == 9 && w.size(2) == Cin) : (w.size(1) == 3 && w.size(2) == 3 && w.size(3) == Cin),
              "gemm_f_conv3x3: w [Cout, 3, 3, Cin] or tap-major [9, Cout, Cin]");
  TORCH_CHECK(stride == 1 || stride == 2, "gemm_f_conv3x3: stride 1 or 2");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  TORCH_CHECK(out.size(0) == imgs && out.size(1) == Ho && out.size(2) == Wo && out.size(3) == Cout,
              "gemm_f_conv3x3: out [N, Ho, Wo, Cout]");
  TORCH_CHECK(vcx_gemm_f_conv3x3_supported((int)imgs, (int)H, (int)W, (int)Cin, (int)Cout, (int)stride),
              "gemm_f_conv3x3: needs Cin a power of two >= 64, Cout % 128 == 0 or Cout == 64, x under 2 GB");
  const bool hb = bias && bias->defined();
  if (hb)
    TORCH_CHECK(bias->is_cuda() && bias->get_device() == x.get_device() && bias->numel() == Cout &&
                    bias->is_contiguous() && bias->scalar_type() == at::kBFloat16, "gemm_f_conv3x3: bias bf16 [Cout]");
  auto [ns, ws] = f_splits(imgs * Ho * Wo, Cout, 9 * Cin, splits, x);
  vcx_gemm_f_conv3x3(x.data_ptr(), w.data_ptr(), out.data_ptr(), hb ? bias->data_ptr() : nullptr, (int)imgs, (int)H,
                     (int)W, (int)Cin, (int)Cout, (int)stride, (int)waves, ns, ns > 1 ? ws.data_ptr<float>() : nullptr,
                     flip_taps ? 1 : 0, tap_major ? 1 : 0, cur_stream());
}

// 3x3 convolution (pad 1, stride 1|2) weight gradient on gemm_wg with the patch matrix of x gathered while
// staging: out [Cout, 9 Cin] (+)= dY^T P(x) -- the [Cout][ky][kx][Cin] (channels-last) weight layout.
// dy: NHWC [imgs, Ho, Wo, Cout], x: NHWC [imgs, H, W, Cin], both contiguous bf16
bool gemm_wg_conv3x3_supported(int64_t Cout, int64_t Cin, int64_t imgs, int64_t H, int64_t W, int64_t stride) {
  if (stride != 1 && stride != 2) return false;
  const int64_t tokens = imgs * ((H - 1) / stride + 1) * ((W - 1) / stride + 1);
  if (tokens >= (int64_t(1) << 31)) return false;
  const int splits = vcx_gemm_wg_splits((int)Cout, (int)(9 * Cin), (int)tokens);
  return vcx_gemm_wg_conv3x3_supported((int)Cout, (int)Cin, (int)tokens, imgs * H * W * Cin * 2, splits);
}

void gemm_wg_conv3x3(at::Tensor dy, at::Tensor x, at::Tensor out, bool accumulate, int64_t stride, int64_t splits) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && out.is_cuda() && dy.dim() == 4 && x.dim() == 4 && out.dim() == 2,
              "gemm_wg_conv3x3: dy [N, Ho, Wo, Cout], x [N, H, W, Cin], out [Cout, 9 Cin] on the GPU");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
              "gemm_wg_conv3x3: bf16");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && out.is_contiguous(), "gemm_wg_conv3x3: contiguous NHWC");
  const int64_t imgs = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = dy.size(3);
  TORCH_CHECK(stride == 1 || stride == 2, "gemm_wg_conv3x3: stride 1 or 2");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  TORCH_CHECK(dy.size(0) == imgs && dy.size(1) == Ho && dy.size(2) == Wo, "gemm_wg_conv3x3: dy / x shapes");
  TORCH_CHECK(out.size(0) == Cout && out.size(1) == 9 * Cin, "gemm_wg_conv3x3: out [Cout, 9 Cin]");
  const int64_t tokens = imgs * Ho * Wo;
  TORCH_CHECK(tokens < (int64_t(1) << 31), "gemm_wg_conv3x3: size");
  if (splits <= 0) splits = vcx_gemm_wg_splits((int)Cout, (int)(9 * Cin), (int)tokens);
  TORCH_CHECK(vcx_gemm_wg_conv3x3_supported((int)Cout, (int)Cin, (int)tokens, imgs * H * W * Cin * 2, (int)splits),
              "gemm_wg_conv3x3: needs Cout % 128 == 0, Cin % 128 == 0, N Ho Wo % 64 == 0, N Ho Wo / 192 >= splits, "
              "x under 2 GB");
  for (const at::Tensor* t : {&dy, &x, &out})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_wg_conv3x3: 16-B aligned base pointers");
  at::Tensor ws = at::empty({splits, Cout, 9 * Cin}, dy.options().dtype(at::kFloat));
  vcx_gemm_wg_conv3x3(dy.data_ptr(), x.data_ptr(), ws.data_ptr<float>(), out.data_ptr(), (int)Cout, (int)Cin, (int)imgs,
                      (int)H, (int)W, (int)stride, (int)splits, accumulate ? 1 : 0, cur_stream());
}

at::Tensor transpose_bf16(at::Tensor src, c10::optional<at::Tensor> dst) {
  TORCH_CHECK(src.is_cuda() && src.dim() == 2 && src.is_contiguous() && src.scalar_type() == at::kBFloat16,
              "transpose_bf16: contiguous 2-D bf16");
  at::Tensor out = dst ? *dst : at::empty({src.size(1), src.size(0)}, src.options());
  TORCH_CHECK(out.size(0) == src.size(1) && out.size(1) == src.size(0) && out.is_contiguous(), "transpose_bf16: dst");
  vcx_transpose_bf16(src.data_ptr(), out.data_ptr(), (int)src.size(0), (int)src.size(1), cur_stream());
  return out;
}

// out (bf16) (+)= in (fp32); zero_in: in is zeroed after the read (a zero-at-rest accumulation buffer)
void add_f32_into_bf16(at::Tensor in, at::Tensor out, bool accumulate, bool zero_in) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kFloat && out.scalar_type() == at::kBFloat16 &&
                  in.numel() == out.numel() && in.is_contiguous() && out.is_contiguous() &&
                  in.get_device() == out.get_device() && in.numel() < (int64_t(1) << 31),
              "add_f32_into_bf16: fp32 in, bf16 out of equal size on one device");
  vcx_add_f32_into_bf16(in.data_ptr<float>(), out.data_ptr(), (int)in.numel(), accumulate ? 1 : 0, zero_in ? 1 : 0,
                        cur_stream());
}

void reduce_bcast_bf16(at::Tensor in, c10::optional<at::Tensor> out, c10::optional<at::Tensor> mine, int64_t P) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kBFloat16 && in.is_contiguous(), "reduce_bcast: bf16 cuda in");
  const int64_t n = in.numel() / P;
  TORCH_CHECK(P > 0 && n * P == in.numel() && n % 8 == 0, "reduce_bcast: numel must be P * n with n % 8 == 0");
  if (out) TORCH_CHECK(out->numel() == in.numel() && out->is_contiguous() && out->scalar_type() == at::kBFloat16,
                       "reduce_bcast: out must match in");
  if (mine) TORCH_CHECK(mine->numel() == n && mine->is_contiguous() && mine->scalar_type() == at::kBFloat16,
                        "reduce_bcast: mine must hold n bf16");
  vcx_reduce_bcast_bf16(in.data_ptr(), out ? out->data_ptr() : nullptr, mine ? mine->data_ptr() : nullptr, (int)P, n,
                        cur_stream());
}

void axpy_bf16(at::Tensor src, at::Tensor acc, double scale) {
  CHECK_IN(src, kBF);
  CHECK_IN(acc, kBF);
  TORCH_CHECK(src.numel() == acc.numel() && src.numel() % 8 == 0);
  vcx_axpy_bf16(src.data_ptr(), acc.data_ptr(), src.numel(), (float)scale, cur_stream());
}

void splitk_reduce(at::Tensor part, at::Tensor acc, bool accumulate) {
  CHECK_IN(part, kBF);
  CHECK_IN(acc, kBF);
  const int64_t n = acc.numel();
  TORCH_CHECK(n % 8 == 0 && part.numel() % n == 0, "splitk_reduce: part must be [S, acc.numel()], numel % 8 == 0");
  vcx_splitk_reduce(part.data_ptr(), acc.data_ptr(), (int)(part.numel() / n), n, accumulate ? 1 : 0, cur_stream());
}

// ------------------------------------------------------------------ norms / activations
std::vector<at::Tensor> ln_fwd(at::Tensor a, c10::optional<at::Tensor> b, at::Tensor w, c10::optional<at::Tensor> bias,
                               double eps, bool rms, c10::optional<at::Tensor> bb) {
  CHECK_IN(a, kBF);
  CHECK_IN(w, kBF);
  const int C = (int)a.size(-1);
  const int64_t R = a.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 8192, "layernorm: C must be a multiple of 8 and <= 8192");
  TORCH_CHECK(w.numel() == C);
  TORCH_CHECK(R < INT32_MAX);
  if (b.has_value()) {
    CHECK_IN((*b), kBF);
    TORCH_CHECK(b->sizes() == a.sizes());
  }
  if (bias.has_value()) {
    CHECK_IN((*bias), kBF);
    TORCH_CHECK(bias->numel() == C);
  }
  if (bb.has_value()) {
    CHECK_IN((*bb), kBF);
    TORCH_CHECK(bb->numel() == C && b.has_value(), "branch bias needs a branch tensor");
  }
  auto y = at::empty_like(a);
  at::Tensor xout = b.has_value() ? at::empty_like(a) : a;
  auto mean = at::empty({R}, a.options().dtype(kF));
  auto rstd = at::empty({R}, a.options().dtype(kF));
  vcx_ln_fwd(a.data_ptr(), opt_ptr(b), b.has_value() ? xout.data_ptr() : nullptr, y.data_ptr(), w.data_ptr(),
             opt_ptr(bias), mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)R, C, (float)eps, rms ? 1 : 0,
             opt_ptr(bb), cur_stream());
  return {y, xout, mean, rstd};
}

// Grad outputs that the caller may pass in (views of the flat gradient buffer): the column sums
// are then ADDED into them (no separate autograd accumulation pass); otherwise fresh tensors.
at::Tensor grad_out(const c10::optional<at::Tensor>& given, int64_t n, const at::Tensor& like, int* mask, int bit) {
  if (given.has_value()) {
    CHECK_IN((*given), kBF);
    TORCH_CHECK(given->numel() == n, "gradient output has the wrong size");
    *mask |= 1 << bit;
    return *given;
  }
  return at::empty({n}, like.options());
}

// returns {dx, dw, db or None, dbb or None}
std::vector<at::Tensor> ln_bwd(at::Tensor dy, at::Tensor x, at::Tensor w, at::Tensor mean, at::Tensor rstd,
                               c10::optional<at::Tensor> dres, bool has_bias, bool rms, bool has_bb,
                               c10::optional<at::Tensor> dw_out, c10::optional<at::Tensor> db_out,
                               c10::optional<at::Tensor> dbb_out) {
  CHECK_IN(dy, kBF);
  CHECK_IN(x, kBF);
  CHECK_IN(w, kBF);
  CHECK_IN(mean, kF);
  CHECK_IN(rstd, kF);
  const int C = (int)x.size(-1);
  const int64_t R = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && C <= 8192 && dy.sizes() == x.sizes() && w.numel() == C);
  TORCH_CHECK(mean.numel() == R && rstd.numel() == R);
  if (dres.has_value()) {
    CHECK_IN((*dres), kBF);
    TORCH_CHECK(dres->sizes() == x.sizes());
  }
  const int P = vcx_ln_bwd_partials((int)R, C);
  auto dx = at::empty_like(x);
  auto dw_part = at::empty({P, C}, x.options().dtype(kF));
  int mask = 0;
  at::Tensor dw = grad_out(dw_out, C, x, &mask, 0);
  at::Tensor db_part, db;
  if (has_bias) {
    db_part = at::empty({P, C}, x.options().dtype(kF));
    db = grad_out(db_out, C, x, &mask, 1);
  }
  at::Tensor dbb_part, dbb;
  if (has_bb) {
    dbb_part = at::empty({P, C}, x.options().dtype(kF));
    dbb = grad_out(dbb_out, C, x, &mask, 2);
  }
  vcx_ln_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
             opt_ptr(dres), dx.data_ptr(), dw_part.data_ptr<float>(), has_bias ? db_part.data_ptr<float>() : nullptr,
             dw.data_ptr(), has_bias ? db.data_ptr() : nullptr, (int)R, C, rms ? 1 : 0,
             has_bb ? dbb_part.data_ptr<float>() : nullptr, has_bb ? dbb.data_ptr() : nullptr,
             at::empty({3 * VCX_COLSUM_NB * C}, x.options().dtype(kF)).data_ptr<float>(), mask, cur_stream());
  return {dx, dw, db, dbb};
}

// out[F] (+)= column sums of y [.., F] (bias gradient of a token-major GEMM output)
at::Tensor colsum_bf16(at::Tensor y, c10::optional<at::Tensor> out) {
  CHECK_IN(y, kBF);
  const int64_t F = y.size(-1), R = y.numel() / F;
  TORCH_CHECK(F % 8 == 0 && R > 0 && R < INT32_MAX, "colsum_bf16: last dim must be a multiple of 8");
  int mask = 0;
  at::Tensor o = grad_out(out, F, y, &mask, 0);
  auto part = at::empty({vcx_bias_gelu_partials((int)R), F}, y.options().dtype(kF));
  auto stage = at::empty({VCX_COLSUM_NB * F}, y.options().dtype(kF));
  vcx_colsum_bf16(y.data_ptr(), part.data_ptr<float>(), o.data_ptr(), (int)R, (int)F, mask, stage.data_ptr<float>(),
                  cur_stream());
  return o;
}

at::Tensor bias_gelu_fwd(at::Tensor x, at::Tensor b) {
  CHECK_IN(x, kBF);
  CHECK_IN(b, kBF);
  const int64_t F = x.size(-1), R = x.numel() / F;
  TORCH_CHECK(F % 8 == 0 && b.numel() == F && R < INT32_MAX);
  auto y = at::empty_like(x);
  vcx_bias_gelu_fwd(x.data_ptr(), b.data_ptr(), y.data_ptr(), (int)R, (int)F, cur_stream());
  return y;
}

std::vector<at::Tensor> bias_gelu_bwd(at::Tensor x, at::Tensor b, at::Tensor dy, c10::optional<at::Tensor> db_out) {
  CHECK_IN(x, kBF);
  CHECK_IN(b, kBF);
  CHECK_IN(dy, kBF);
  const int64_t F = x.size(-1), R = x.numel() / F;
  TORCH_CHECK(F % 8 == 0 && b.numel() == F && dy.sizes() == x.sizes() && R < INT32_MAX);
  auto dx = at::empty_like(x);
  auto part = at::empty({vcx_bias_gelu_partials((int)R), F}, x.options().dtype(kF));
  int mask = 0;
  auto db = grad_out(db_out, F, x, &mask, 0);
  auto stage = at::empty({VCX_COLSUM_NB * F}, x.options().dtype(kF));
  vcx_bias_gelu_bwd(x.data_ptr(), b.data_ptr(), dy.data_ptr(), dx.data_ptr(), part.data_ptr<float>(), db.data_ptr(),
                    (int)R, (int)F, stage.data_ptr<float>(), mask, cur_stream());
  return {dx, db};
}

at::Tensor gelu_fwd(at::Tensor x) {
  CHECK_IN(x, kBF);
  TORCH_CHECK(x.numel() % 8 == 0);
  auto y = at::empty_like(x);
  vcx_gelu_fwd(x.data_ptr(), y.data_ptr(), x.numel(), cur_stream());
  return y;
}

at::Tensor gelu_bwd(at::Tensor x, at::Tensor dy) {
  CHECK_IN(x, kBF);
  CHECK_IN(dy, kBF);
  TORCH_CHECK(x.numel() % 8 == 0 && dy.numel() == x.numel());
  auto dx = at::empty_like(x);
  vcx_gelu_bwd(x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), cur_stream());
  return dx;
}

at::Tensor swiglu_fwd(at::Tensor gu) {
  CHECK_IN(gu, kBF);
  const int64_t F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "swiglu: feature dim must be a multiple of 16");
  const int64_t R = gu.numel() / F2;
  auto sizes = gu.sizes().vec();
  sizes.back() = F2 / 2;
  auto y = at::empty(sizes, gu.options());
  vcx_swiglu_fwd(gu.data_ptr(), y.data_ptr(), R, (int)(F2 / 2), cur_stream());
  return y;
}

at::Tensor swiglu_bwd(at::Tensor gu, at::Tensor dy) {
  CHECK_IN(gu, kBF);
  CHECK_IN(dy, kBF);
  const int64_t F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0 && dy.numel() * 2 == gu.numel());
  auto dgu = at::empty_like(gu);
  vcx_swiglu_bwd(gu.data_ptr(), dy.data_ptr(), dgu.data_ptr(), gu.numel() / F2, (int)(F2 / 2), cur_stream());
  return dgu;
}

std::vector<at::Tensor> xent_fwd(at::Tensor logits, at::Tensor tgt, int64_t V) {
  CHECK_IN(logits, kBF);
  CHECK_IN(tgt, at::kLong);
  TORCH_CHECK(logits.dim() == 2);
  const int64_t R = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(Vp % 8 == 0 && V <= Vp && V > 0 && tgt.numel() == R);
  auto lse = at::empty({R}, logits.options().dtype(kF));
  auto loss = at::empty({R}, logits.options().dtype(kF));
  vcx_xent_fwd(logits.data_ptr(), tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), loss.data_ptr<float>(), R, (int)V,
               (int)Vp, cur_stream());
  return {loss, lse};
}

void xent_bwd(at::Tensor logits, at::Tensor tgt, at::Tensor lse, at::Tensor gscale, at::Tensor dlogits, int64_t V) {
  CHECK_IN(logits, kBF);
  CHECK_IN(tgt, at::kLong);
  CHECK_IN(lse, kF);
  CHECK_IN(gscale, kF);
  CHECK_IN(dlogits, kBF);
  const int64_t R = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(logits.dim() == 2 && dlogits.sizes() == logits.sizes() && tgt.numel() == R && lse.numel() == R);
  TORCH_CHECK(Vp % 8 == 0 && V <= Vp && gscale.numel() >= 1);
  vcx_xent_bwd(logits.data_ptr(), tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), gscale.data_ptr<float>(),
               dlogits.data_ptr(), R, (int)V, (int)Vp, cur_stream());
}

// fused loss + gradient; returns per-row losses or None if the row does not fit (caller falls back)
c10::optional<at::Tensor> xent_fused(at::Tensor logits, at::Tensor tgt, at::Tensor nvalid, int64_t V) {
  CHECK_IN(logits, kBF);
  CHECK_IN(tgt, at::kLong);
  CHECK_IN(nvalid, kF);
  TORCH_CHECK(logits.dim() == 2);
  const int64_t R = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(Vp % 8 == 0 && V <= Vp && V > 0 && tgt.numel() == R && nvalid.numel() >= 1);
  auto loss = at::empty({R}, logits.options().dtype(kF));
  if (!vcx_xent_fused(logits.data_ptr(), tgt.data_ptr<int64_t>(), nvalid.data_ptr<float>(), loss.data_ptr<float>(), R,
                      (int)V, (int)Vp, cur_stream()))
    return c10::nullopt;
  return loss;
}

void xent_rescale(at::Tensor d, at::Tensor dloss) {
  CHECK_IN(d, kBF);
  CHECK_IN(dloss, kF);
  TORCH_CHECK(d.numel() % 8 == 0 && dloss.numel() >= 1);
  vcx_xent_rescale(d.data_ptr(), dloss.data_ptr<float>(), d.numel(), cur_stream());
}

// ------------------------------------------------------------------ embedding
at::Tensor embed_fwd(at::Tensor idx, at::Tensor wte, c10::optional<at::Tensor> wpe, int64_t T) {
  CHECK_IN(idx, at::kLong);
  CHECK_IN(wte, kBF);
  TORCH_CHECK(wte.dim() == 2 && wte.size(1) % 8 == 0);
  const int64_t R = idx.numel(), V = wte.size(0), C = wte.size(1);
  TORCH_CHECK(T > 0 && R % T == 0);
  if (wpe.has_value()) {
    CHECK_IN((*wpe), kBF);
    TORCH_CHECK(wpe->dim() == 2 && wpe->size(1) == C && wpe->size(0) >= T, "position table too short");
  }
  auto out = at::empty({R, C}, wte.options());
  vcx_embed_fwd(idx.data_ptr<int64_t>(), wte.data_ptr(), opt_ptr(wpe), out.data_ptr(), R, (int)T, (int)C, (int)V,
                cur_stream());
  return out;
}

// returns {dwte, dwpe or None}; with wte_grad / wpe_grad given (flat .grad views) the gradients
// are added into them and those same tensors are returned
std::vector<at::Tensor> embed_bwd(at::Tensor idx, at::Tensor dx, int64_t V, int64_t T, int64_t Tpos,
                                  c10::optional<at::Tensor> wte_grad, c10::optional<at::Tensor> wpe_grad) {
  CHECK_IN(idx, at::kLong);
  CHECK_IN(dx, kBF);
  const int64_t R = idx.numel(), C = dx.size(-1);
  TORCH_CHECK(dx.numel() == R * C && C % 8 == 0 && C <= 8192 && T > 0 && R % T == 0 && Tpos >= 0 && Tpos >= (Tpos ? T : 0));
  auto scratch = at::zeros({V, C}, dx.options().dtype(kF));
  at::Tensor dwte, dwpe;
  int acc_wte = 0, acc_wpe = 0;
  if (wte_grad.has_value()) {
    CHECK_IN((*wte_grad), kBF);
    TORCH_CHECK(wte_grad->numel() == V * C);
    dwte = *wte_grad;
    acc_wte = 1;
  } else {
    dwte = at::empty({V, C}, dx.options());
  }
  if (Tpos > 0) {
    if (wpe_grad.has_value()) {
      CHECK_IN((*wpe_grad), kBF);
      TORCH_CHECK(wpe_grad->numel() == Tpos * C);
      dwpe = *wpe_grad;
      acc_wpe = 1;
    } else {
      dwpe = at::zeros({Tpos, C}, dx.options());  // rows >= T get no gradient
    }
  }
  vcx_embed_bwd(idx.data_ptr<int64_t>(), dx.data_ptr(), scratch.data_ptr<float>(), dwte.data_ptr(), acc_wte,
                Tpos > 0 ? dwpe.data_ptr() : nullptr, acc_wpe, R, (int)T, (int)C, (int)V, cur_stream());
  return {dwte, dwpe};
}

// ------------------------------------------------------------------ rotary embedding (Llama)
std::vector<at::Tensor> rope_qkv_fwd(at::Tensor qkv, at::Tensor cosv, at::Tensor sinv, int64_t Hq, int64_t Hkv) {
  CHECK_IN(qkv, kBF);
  CHECK_IN(cosv, kF);
  CHECK_IN(sinv, kF);
  TORCH_CHECK(qkv.dim() == 3, "rope_qkv: qkv must be [B, T, (Hq + 2 Hkv) * D]");
  const int64_t B = qkv.size(0), T = qkv.size(1), W = qkv.size(2);
  TORCH_CHECK(Hq > 0 && Hkv > 0 && W % (Hq + 2 * Hkv) == 0);
  const int64_t D = W / (Hq + 2 * Hkv);
  TORCH_CHECK(D % 8 == 0, "rope_qkv: head dim must be a multiple of 8");
  TORCH_CHECK(cosv.dim() == 2 && cosv.size(0) >= T && cosv.size(1) == D / 2 && sinv.sizes() == cosv.sizes(),
              "rope_qkv: cos/sin tables must be [>= T, D/2]");
  auto q = at::empty({B, Hq, T, D}, qkv.options());
  auto k = at::empty({B, Hkv, T, D}, qkv.options());
  auto v = at::empty({B, Hkv, T, D}, qkv.options());
  vcx_rope_qkv(qkv.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), cosv.data_ptr<float>(),
               sinv.data_ptr<float>(), (int)B, (int)T, (int)Hq, (int)Hkv, (int)D, 0, cur_stream());
  return {q, k, v};
}

at::Tensor rope_qkv_bwd(at::Tensor dq, at::Tensor dk, at::Tensor dv, at::Tensor cosv, at::Tensor sinv) {
  CHECK_IN(dq, kBF);
  CHECK_IN(dk, kBF);
  CHECK_IN(dv, kBF);
  CHECK_IN(cosv, kF);
  CHECK_IN(sinv, kF);
  TORCH_CHECK(dq.dim() == 4 && dk.dim() == 4 && dk.sizes() == dv.sizes());
  const int64_t B = dq.size(0), Hq = dq.size(1), T = dq.size(2), D = dq.size(3), Hkv = dk.size(1);
  TORCH_CHECK(dk.size(0) == B && dk.size(2) == T && dk.size(3) == D && D % 8 == 0);
  TORCH_CHECK(cosv.size(0) >= T && cosv.size(1) == D / 2 && sinv.sizes() == cosv.sizes());
  auto dqkv = at::empty({B, T, (Hq + 2 * Hkv) * D}, dq.options());
  vcx_rope_qkv(dqkv.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), cosv.data_ptr<float>(),
               sinv.data_ptr<float>(), (int)B, (int)T, (int)Hq, (int)Hkv, (int)D, 1, cur_stream());
  return dqkv;
}

// ------------------------------------------------------------------ attention (head dim 64)
std::vector<at::Tensor> attn_fwd(at::Tensor qkv, double scale) {
  CHECK_IN(qkv, kBF);
  TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.size(4) == 64, "attn_fwd: qkv must be [B, T, 3, H, 64]");
  const int64_t B = qkv.size(0), T = qkv.size(1), H = qkv.size(3);
  TORCH_CHECK(B * H * ((T + 127) / 128) < INT32_MAX && T > 0);
  auto out = at::empty({B, T, H, 64}, qkv.options());
  auto lse = at::empty({B, H, T}, qkv.options().dtype(kF));
  vcx_attn_fwd_d64(qkv.data_ptr(), out.data_ptr(), lse.data_ptr<float>(), (int)B, (int)T, (int)H, (float)scale,
                   cur_stream());
  return {out, lse};
}

at::Tensor attn_bwd(at::Tensor qkv, at::Tensor out, at::Tensor dout, at::Tensor lse, double scale) {
  CHECK_IN(qkv, kBF);
  CHECK_IN(out, kBF);
  CHECK_IN(dout, kBF);
  CHECK_IN(lse, kF);
  TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.size(4) == 64);
  const int64_t B = qkv.size(0), T = qkv.size(1), H = qkv.size(3);
  TORCH_CHECK(out.sizes() == at::IntArrayRef({B, T, H, 64}) && dout.sizes() == out.sizes());
  TORCH_CHECK(lse.numel() == B * H * T);
  auto dqkv = at::empty_like(qkv);
  auto delta = at::empty({B, H, T}, lse.options());
  vcx_attn_bwd_d64(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
                   dqkv.data_ptr(), nullptr, (int)B, (int)T, (int)H, (float)scale, cur_stream());
  return dqkv;
}

// attn_bwd plus the gradient of a bias added to qkv ([3 * H * 64]: the fused QKV projection's
// bias), reduced from per-block column sums the backward kernels emit — no separate pass over
// dqkv. db_out: the preset (flat) gradient buffer to add into; returned otherwise.
std::vector<at::Tensor> attn_bwd_bias(at::Tensor qkv, at::Tensor out, at::Tensor dout, at::Tensor lse, double scale,
                                      c10::optional<at::Tensor> db_out) {
  CHECK_IN(qkv, kBF);
  CHECK_IN(out, kBF);
  CHECK_IN(dout, kBF);
  CHECK_IN(lse, kF);
  TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.size(4) == 64);
  const int64_t B = qkv.size(0), T = qkv.size(1), H = qkv.size(3), F = 3 * H * 64;
  TORCH_CHECK(out.sizes() == at::IntArrayRef({B, T, H, 64}) && dout.sizes() == out.sizes());
  TORCH_CHECK(lse.numel() == B * H * T);
  auto dqkv = at::empty_like(qkv);
  auto delta = at::empty({B, H, T}, lse.options());
  const int P = vcx_attn_bias_partials((int)B, (int)T);
  auto part = at::empty({P, F}, lse.options());
  int mask = 0;
  at::Tensor db = grad_out(db_out, F, qkv, &mask, 0);
  auto stage = at::empty({VCX_COLSUM_NB * F}, lse.options());
  vcx_attn_bwd_d64(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
                   dqkv.data_ptr(), part.data_ptr<float>(), (int)B, (int)T, (int)H, (float)scale, cur_stream());
  vcx_colsum_f32(part.data_ptr<float>(), db.data_ptr(), P, (int)F, mask, stage.data_ptr<float>(), cur_stream());
  return {dqkv, db};
}

// head-major GQA attention (Llama family): q [B, Hq, T, D], k / v [B, Hkv, T, D], D in {64, 128}
static void check_hm(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
  CHECK_IN(q, kBF);
  CHECK_IN(k, kBF);
  CHECK_IN(v, kBF);
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && k.sizes() == v.sizes(), "attn_hm: q [B,Hq,T,D], k/v [B,Hkv,T,D]");
  TORCH_CHECK(q.size(0) == k.size(0) && q.size(2) == k.size(2) && q.size(3) == k.size(3));
  TORCH_CHECK(q.size(3) == 64 || q.size(3) == 128, "attn_hm: head dim must be 64 or 128");
  TORCH_CHECK(q.size(1) % k.size(1) == 0, "attn_hm: Hq must be a multiple of Hkv");
}

std::vector<at::Tensor> attn_hm_fwd(at::Tensor q, at::Tensor k, at::Tensor v, double scale) {
  check_hm(q, k, v);
  const int64_t B = q.size(0), Hq = q.size(1), T = q.size(2), D = q.size(3), Hkv = k.size(1);
  auto out = at::empty({B, T, Hq, D}, q.options());
  auto lse = at::empty({B, Hq, T}, q.options().dtype(kF));
  vcx_attn_hm_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), lse.data_ptr<float>(), (int)B, (int)T,
                  (int)Hq, (int)Hkv, (int)D, (float)scale, cur_stream());
  return {out, lse};
}

std::vector<at::Tensor> attn_hm_bwd(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor out, at::Tensor dout,
                                    at::Tensor lse, double scale) {
  check_hm(q, k, v);
  CHECK_IN(out, kBF);
  CHECK_IN(dout, kBF);
  CHECK_IN(lse, kF);
  const int64_t B = q.size(0), Hq = q.size(1), T = q.size(2), D = q.size(3), Hkv = k.size(1);
  TORCH_CHECK(out.sizes() == at::IntArrayRef({B, T, Hq, D}) && dout.sizes() == out.sizes());
  TORCH_CHECK(lse.numel() == B * Hq * T);
  auto dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
  auto delta = at::empty({B, Hq, T}, lse.options());
  vcx_attn_hm_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                  delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), (int)B, (int)T, (int)Hq,
                  (int)Hkv, (int)D, (float)scale, cur_stream());
  return {dq, dk, dv};
}

}  // namespace

void vcx_register_vision(pybind11::module& m);
void vcx_register_compress(pybind11::module& m);
void vcx_register_lt(pybind11::module& m);
extern "C" const char* vcx_source_digest();  // generated by _build.py (digest of the sources linked here)

PYBIND11_MODULE(_C, m) {
  m.doc() = "gfx950 HIP kernels of distributedvolunteercomputing_amd";
  m.def("source_digest", [] { return std::string(vcx_source_digest()); });
  m.def("grad_sumsq", &grad_sumsq);
  m.def("adam_prologue", &adam_prologue);
  m.def("adamw_flat", &adamw_flat);
  m.def("lsgd_delta", &lsgd_delta);
  m.def("lsgd_apply", &lsgd_apply);
  m.def("f32_to_bf16", &f32_to_bf16);
  m.def("axpy_bf16", &axpy_bf16);
  m.def("reduce_bcast_bf16", &reduce_bcast_bf16);
  m.def("gemm_nt_supported", &gemm_nt_supported);
  m.def("gemm_nt_supported_epi", &gemm_nt_supported_epi);
  m.def("gemm_ps_supported", &gemm_ps_supported);
  m.def("bn_supported", [](int64_t C) { return vcx_bn_supported((int)C); });
  m.def("bn_fwd_train", &bn_fwd_train, py::arg("x"), py::arg("res"), py::arg("gamma"), py::arg("beta"),
        py::arg("run_mean"), py::arg("run_var"), py::arg("eps"), py::arg("momentum"), py::arg("relu"),
        py::arg("nbt") = py::none(), py::arg("layer_ws") = py::none());
  m.def("bn_apply", &bn_apply);
  m.def("maxpool3s2_fwd", &maxpool3s2_fwd);
  m.def("maxpool3s2_bwd", &maxpool3s2_bwd);
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("mask"), py::arg("x"), py::arg("mean"), py::arg("rstd"), py::arg("scale"),
        py::arg("relu"), py::arg("want_dres"), py::arg("gw") = py::none(), py::arg("gb") = py::none(),
        py::arg("layer_ws") = py::none());
  m.def("gemm_ps", &gemm_ps, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("c2") = py::none(),
        py::arg("bias") = py::none(), py::arg("colsum") = py::none(), py::arg("epi") = 0, py::arg("grid_cap") = 0);
  m.def("gemm_f_supported", &gemm_f_supported, py::arg("M"), py::arg("N"), py::arg("K"));
  m.def("gemm_f_conv3x3_supported", &gemm_f_conv3x3_supported, py::arg("imgs"), py::arg("H"), py::arg("W"),
        py::arg("Cin"), py::arg("Cout"), py::arg("stride"));
  m.def("gemm_f_conv3x3", &gemm_f_conv3x3, py::arg("x"), py::arg("w"), py::arg("out"), py::arg("stride"),
        py::arg("bias") = py::none(), py::arg("waves") = 0, py::arg("splits") = -1, py::arg("flip_taps") = false);
  m.def("gemm_f_splits", &gemm_f_splits, py::arg("M"), py::arg("N"), py::arg("K"));
  m.def("gemm_f", &gemm_f, py::arg("a"), py::arg("b"), py::arg("out"), py::arg("bias") = py::none(),
        py::arg("waves") = 0, py::arg("splits") = -1);
  m.def("gemm_wg_supported", &gemm_wg_supported, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("splits") = 0);
  m.def("gemm_wg_conv3x3_supported", &gemm_wg_conv3x3_supported, py::arg("Cout"), py::arg("Cin"), py::arg("imgs"),
        py::arg("H"), py::arg("W"), py::arg("stride"));
  m.def("gemm_wg_conv3x3", &gemm_wg_conv3x3, py::arg("dy"), py::arg("x"), py::arg("out"), py::arg("accumulate") = false,
        py::arg("stride") = 1, py::arg("splits") = 0);
  m.def("gemm_wg", &gemm_wg, py::arg("a"), py::arg("b"), py::arg("out"), py::arg("accumulate") = false,
        py::arg("splits") = 0, py::arg("loaders") = 8);
  m.def("gemm_nt", &gemm_nt, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("c2") = py::none(),
        py::arg("bias") = py::none(), py::arg("colsum") = py::none(), py::arg("epi") = 0);
  m.def("transpose_bf16", &transpose_bf16, py::arg("src"), py::arg("dst") = py::none());
  m.def("subsample_nhwc", &subsample_nhwc, py::arg("x"), py::arg("stride"));
  m.def("subsample_add_nhwc", &subsample_add_nhwc, py::arg("full"), py::arg("g"), py::arg("stride"));
  m.def("bcast_hw_nhwc", &bcast_hw_nhwc, py::arg("g"), py::arg("H"), py::arg("W"), py::arg("scale"));
  m.def("add_f32_into_bf16", &add_f32_into_bf16, py::arg("src"), py::arg("out"), py::arg("accumulate"),
        py::arg("zero_src") = false);
  m.def("splitk_reduce", &splitk_reduce);
  m.def("ln_fwd", &ln_fwd);
  m.def("ln_bwd", &ln_bwd, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("mean"),
        pybind11::arg("rstd"), pybind11::arg("dres"), pybind11::arg("has_bias"), pybind11::arg("rms"),
        pybind11::arg("has_bb"), pybind11::arg("dw_out") = pybind11::none(), pybind11::arg("db_out") = pybind11::none(),
        pybind11::arg("dbb_out") = pybind11::none());
  m.def("colsum_bf16", &colsum_bf16, pybind11::arg("y"), pybind11::arg("out") = pybind11::none());
  m.def("gelu_fwd", &gelu_fwd);
  m.def("bias_gelu_fwd", &bias_gelu_fwd);
  m.def("bias_gelu_bwd", &bias_gelu_bwd, pybind11::arg("x"), pybind11::arg("b"), pybind11::arg("dy"),
        pybind11::arg("db_out") = pybind11::none());
  m.def("gelu_bwd", &gelu_bwd);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("xent_fused", &xent_fused);
  m.def("xent_rescale", &xent_rescale);
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd, pybind11::arg("idx"), pybind11::arg("dx"), pybind11::arg("V"), pybind11::arg("T"),
        pybind11::arg("Tpos"), pybind11::arg("wte_grad") = pybind11::none(), pybind11::arg("wpe_grad") = pybind11::none());
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_set_variant", &vcx_attn_set_variant, pybind11::arg("fwd_wpe"), pybind11::arg("fwd_dma"),
        pybind11::arg("bwd_dma"), pybind11::arg("stage_epi") = -1);
  m.def("rope_qkv_fwd", &rope_qkv_fwd);
  m.def("rope_qkv_bwd", &rope_qkv_bwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("attn_hm_fwd", &attn_hm_fwd);
  m.def("attn_hm_bwd", &attn_hm_bwd);
  m.def("attn_hm_set_variant", &vcx_attn_hm_set_variant);
  m.def("attn_bwd_bias", &attn_bwd_bias, pybind11::arg("qkv"), pybind11::arg("out"), pybind11::arg("dout"),
        pybind11::arg("lse"), pybind11::arg("scale"), pybind11::arg("db_out") = pybind11::none());
  vcx_register_vision(m);
  vcx_register_compress(m);
  vcx_register_lt(m);
}
