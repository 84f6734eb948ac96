// Torch bindings for the MobileNet-SSD inference kernels (kernels/vision.hip).
// Host-side shape checks guard every launch (no hand-written kernel sees a shape it was not
// written for).
#include <cstdlib>
#include <map>
#include <mutex>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/vcx_api_vision.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHK(x, dt)                                                      \
  TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor");               \
  TORCH_CHECK((x).is_contiguous(), #x " must be contiguous");           \
  TORCH_CHECK((x).scalar_type() == (dt), #x " has dtype ", (x).scalar_type())

at::Tensor resize_area_u8(at::Tensor src, int64_t h, int64_t w) {
  CHK(src, at::kByte);
  TORCH_CHECK(src.dim() == 4 && src.size(3) == 3, "expect [N,H,W,3] uint8");
  TORCH_CHECK(h > 0 && w > 0 && w <= src.size(2) && h <= src.size(1), "area resize is a downscale");
  auto dst = at::empty({src.size(0), h, w, 3}, src.options());
  vcx_resize_area_u8(src.data_ptr<uint8_t>(), dst.data_ptr<uint8_t>(), (int)src.size(0), (int)src.size(1),
                     (int)src.size(2), (int)h, (int)w, cur_stream());
  return dst;
}

at::Tensor resize_bilinear_u8(at::Tensor src, int64_t h, int64_t w) {
  CHK(src, at::kByte);
  TORCH_CHECK(src.dim() == 4 && src.size(3) == 3 && h > 0 && w > 0);
  auto dst = at::empty({src.size(0), h, w, 3}, src.options());
  vcx_resize_bilinear_u8(src.data_ptr<uint8_t>(), dst.data_ptr<uint8_t>(), (int)src.size(0), (int)src.size(1),
                         (int)src.size(2), (int)h, (int)w, cur_stream());
  return dst;
}

at::Tensor blob_bilinear(at::Tensor src, int64_t S, double scale, double mean) {
  CHK(src, at::kByte);
  TORCH_CHECK(src.dim() == 4 && src.size(3) == 3 && S > 0);
  TORCH_CHECK(src.size(0) <= 65535 && S <= 65535, "blob_bilinear: grid limits");
  auto dst = at::empty({src.size(0), S, S, 4}, src.options().dtype(at::kBFloat16));
  vcx_blob_bilinear(src.data_ptr<uint8_t>(), dst.data_ptr(), (int)src.size(0), (int)src.size(1), (int)src.size(2),
                    (int)S, (float)scale, (float)mean, cur_stream());
  return dst;
}

at::Tensor im2col_nhwc(at::Tensor x, int64_t C, int64_t k, int64_t stride, int64_t pad, int64_t Kp) {
  CHK(x, at::kBFloat16);
  TORCH_CHECK(x.dim() == 4 && C <= x.size(3) && Kp % 32 == 0 && Kp >= k * k * C);
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  const int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0);
  auto out = at::empty({N * Ho * Wo, Kp}, x.options());
  vcx_im2col_nhwc(x.data_ptr(), out.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)x.size(3), (int)Ho, (int)Wo,
                  (int)k, (int)k, (int)stride, (int)pad, (int)Kp, cur_stream());
  return out;
}

// Split-K ticket counters for the in-kernel reduction: one zeroed int array per stream (kernels
// on one stream never overlap; the last block of every tile re-arms its counter to zero). Created
// on first use outside graph capture (the executor's warm-up passes run before its capture).
// Measured: the last block's serial reduction of a 128 x 128 tile (S partials per element)
// runs 50-120 us per layer against 5-8 us for the separate splitk_bias_act launch, so the
// in-kernel path is opt-in (VCX_SPLITK_INKERNEL=1).
static int* splitk_counters(const at::Tensor& like) {
  static const bool on = [] {
    const char* e = std::getenv("VCX_SPLITK_INKERNEL");
    return e && e[0] == '1';
  }();
  if (!on) return nullptr;
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, at::Tensor> bufs;
  const hipStream_t st = cur_stream();
  std::lock_guard<std::mutex> g(mu);
  auto key = std::make_pair((int)like.get_device(), st);
  auto it = bufs.find(key);
  if (it == bufs.end()) it = bufs.emplace(key, at::zeros({4096}, like.options().dtype(at::kInt))).first;
  return it->second.data_ptr<int>();
}

at::Tensor dwconv3x3(at::Tensor x, at::Tensor w, at::Tensor b, int64_t stride, bool relu) {
  CHK(x, at::kBFloat16);
  CHK(w, at::kBFloat16);
  CHK(b, at::kFloat);
  TORCH_CHECK(x.dim() == 4);
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && w.numel() == 10 * C && b.numel() == C && (stride == 1 || stride == 2),
              "dwconv3x3: paired weights [5, C, 2] (ops/vision.py dw_pair_weights)");
  TORCH_CHECK(((uintptr_t)x.data_ptr() & 15) == 0 && ((uintptr_t)w.data_ptr() & 15) == 0 &&
              ((uintptr_t)b.data_ptr() & 15) == 0, "dwconv3x3: 16-B aligned operands");
  const int64_t Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  TORCH_CHECK(Wo * (C / 8) < INT32_MAX && N * ((Ho + 1) / 2) <= 65535 && N * H * W * C < ((int64_t)1 << 40),
              "dwconv3x3: grid limits");
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  vcx_dwconv3x3(x.data_ptr(), w.data_ptr(), b.data_ptr<float>(), y.data_ptr(), (int)N, (int)H, (int)W, (int)C,
                (int)Ho, (int)Wo, (int)stride, relu ? 1 : 0, cur_stream());
  return y;
}

at::Tensor gemm_bias_act(at::Tensor X, at::Tensor Wt, c10::optional<at::Tensor> bias, bool relu) {
  CHK(X, at::kBFloat16);
  CHK(Wt, at::kBFloat16);
  TORCH_CHECK(X.dim() == 2 && Wt.dim() == 2 && X.size(1) == Wt.size(1), "X [M,K] . Wt[N,K]^T");
  const int64_t M = X.size(0), K = X.size(1), N = Wt.size(0);
  TORCH_CHECK(K % 32 == 0, "K must be a multiple of 32");
  TORCH_CHECK(M < INT32_MAX && M * K < (int64_t)1 << 40);
  const float* bp = nullptr;
  if (bias.has_value()) {
    CHK((*bias), at::kFloat);
    TORCH_CHECK(bias->numel() == N);
    bp = bias->data_ptr<float>();
  }
  auto Y = at::empty({M, N}, X.options());
  const int S = vcx_vision_ksplit((int)M, (int)N, (int)K);
  at::Tensor ws = S > 1 ? at::empty({S, M, N}, X.options().dtype(at::kFloat)) : at::Tensor();
  vcx_gemm_bias_act(X.data_ptr(), Wt.data_ptr(), bp, Y.data_ptr(), (int)M, (int)N, (int)K, (int)N, relu ? 1 : 0,
                    S > 1 ? ws.data_ptr<float>() : nullptr, S, S > 1 ? splitk_counters(X) : nullptr, cur_stream());
  return Y;
}

// MobileNet block in one kernel: depthwise 3x3 (pad 1, stride 1|2) + bias (+ReLU), then the
// pointwise GEMM + bias (+ReLU); the depthwise activation stays on chip.
at::Tensor dw_pw(at::Tensor x, at::Tensor dw_w, at::Tensor dw_b, bool dw_relu, int64_t stride, at::Tensor Wt,
                 at::Tensor bias, bool relu) {
  CHK(x, at::kBFloat16);
  CHK(dw_w, at::kBFloat16);
  CHK(dw_b, at::kFloat);
  CHK(Wt, at::kBFloat16);
  CHK(bias, at::kFloat);
  TORCH_CHECK(x.dim() == 4 && Wt.dim() == 2, "x NHWC, Wt [N, K]");
  const int64_t imgs = x.size(0), H = x.size(1), W = x.size(2), K = x.size(3), N = Wt.size(0);
  TORCH_CHECK(K % 32 == 0 && K <= 1024 && Wt.size(1) == K && dw_w.numel() == 10 * K && dw_b.numel() == K &&
                  bias.numel() == N,
              "dw_pw: K % 32 == 0, K <= 1024, paired dw_w [5, K, 2], dw_b [K], Wt [N, K], bias [N]");
  TORCH_CHECK(stride == 1 || stride == 2);
  TORCH_CHECK(((uintptr_t)x.data_ptr() & 15) == 0 && ((uintptr_t)dw_w.data_ptr() & 15) == 0 &&
              ((uintptr_t)dw_b.data_ptr() & 15) == 0 && ((uintptr_t)Wt.data_ptr() & 15) == 0,
              "dw_pw: 16-B aligned operands");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  TORCH_CHECK(imgs * Ho * Wo < INT32_MAX && imgs * H * W * K < ((int64_t)1 << 40));
  auto Y = at::empty({imgs, Ho, Wo, N}, x.options());
  vcx_dw_pw(x.data_ptr(), dw_w.data_ptr(), dw_b.data_ptr<float>(), dw_relu ? 1 : 0, Wt.data_ptr(),
            bias.data_ptr<float>(), Y.data_ptr(), (int)imgs, (int)H, (int)W, (int)K, (int)stride, (int)N,
            relu ? 1 : 0, cur_stream());
  return Y;
}

// SSD head of one source: loc||conf as ONE GEMM whose epilogue writes columns [0, split) into
// `loc_all` and [split, N) into `conf_all` (both [images, total]) at the source's offsets, rows
// grouped `rpi` per image — the Permute + Flatten + Concat of the prototxt as address arithmetic.
void gemm_bias_heads(at::Tensor X, at::Tensor Wt, at::Tensor bias, at::Tensor loc_all, int64_t loc_off,
                     at::Tensor conf_all, int64_t conf_off, int64_t split, int64_t rpi) {
  CHK(X, at::kBFloat16);
  CHK(Wt, at::kBFloat16);
  CHK(bias, at::kFloat);
  CHK(loc_all, at::kBFloat16);
  CHK(conf_all, at::kBFloat16);
  TORCH_CHECK(X.dim() == 2 && Wt.dim() == 2 && X.size(1) == Wt.size(1), "X [M,K] . Wt[N,K]^T");
  const int64_t M = X.size(0), K = X.size(1), N = Wt.size(0);
  TORCH_CHECK(K % 32 == 0 && bias.numel() == N && split > 0 && split < N && rpi > 0 && M % rpi == 0);
  const int64_t imgs = M / rpi;
  TORCH_CHECK(loc_all.dim() == 2 && conf_all.dim() == 2 && loc_all.size(0) == imgs && conf_all.size(0) == imgs);
  TORCH_CHECK(loc_off + rpi * split <= loc_all.size(1) && conf_off + rpi * (N - split) <= conf_all.size(1),
              "head output out of the concat buffer");
  const int S = vcx_vision_ksplit((int)M, (int)N, (int)K);
  at::Tensor ws = S > 1 ? at::empty({S, M, N}, X.options().dtype(at::kFloat)) : at::Tensor();
  vcx_gemm_bias_act_mapped(X.data_ptr(), Wt.data_ptr(), bias.data_ptr<float>(),
                           (uint16_t*)loc_all.data_ptr() + loc_off, (int)M, (int)N, (int)K, (int)split, 0,
                           (uint16_t*)conf_all.data_ptr() + conf_off, (int)split, (int)(N - split), (int)rpi,
                           loc_all.size(1), conf_all.size(1), S > 1 ? ws.data_ptr<float>() : nullptr, S,
                           S > 1 ? splitk_counters(X) : nullptr, cur_stream());
}

// Two MobileNet blocks in one kernel (conv1: dw s1 + pw K1 -> N1, conv2: dw s2 + pw N1 -> N2; the first
// block's output never leaves LDS). Returns an undefined tensor when no instance covers the shapes.
at::Tensor dw_pw2(at::Tensor x, at::Tensor dw1_w, at::Tensor dw1_b, bool dw1_relu, at::Tensor W1, at::Tensor b1,
                  bool relu1, at::Tensor dw2_w, at::Tensor dw2_b, bool dw2_relu, at::Tensor W2, at::Tensor b2, bool relu2) {
  CHK(x, at::kBFloat16);
  CHK(dw1_w, at::kBFloat16);
  CHK(W1, at::kBFloat16);
  CHK(dw2_w, at::kBFloat16);
  CHK(W2, at::kBFloat16);
  CHK(dw1_b, at::kFloat);
  CHK(b1, at::kFloat);
  CHK(dw2_b, at::kFloat);
  CHK(b2, at::kFloat);
  TORCH_CHECK(x.dim() == 4 && W1.dim() == 2 && W2.dim() == 2, "x NHWC, W1 [N1, K1], W2 [N2, N1]");
  const int64_t imgs = x.size(0), H = x.size(1), W = x.size(2), K1 = x.size(3), N1 = W1.size(0), N2 = W2.size(0);
  TORCH_CHECK(W1.size(1) == K1 && W2.size(1) == N1 && dw1_w.numel() == 10 * K1 && dw1_b.numel() == K1 &&
                  dw2_w.numel() == 10 * N1 && dw2_b.numel() == N1 && b1.numel() == N1 && b2.numel() == N2,
              "dw_pw2: paired dw weights [5, C, 2], biases [C], W1 [N1, K1], W2 [N2, N1]");
  for (const at::Tensor* t : {&x, &dw1_w, &dw1_b, &W1, &dw2_w, &dw2_b, &W2})
    TORCH_CHECK(((uintptr_t)t->data_ptr() & 15) == 0, "dw_pw2: 16-B aligned operands");
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  TORCH_CHECK(imgs * Ho * Wo < INT32_MAX && imgs * H * W * K1 < ((int64_t)1 << 40));
  auto Y = at::empty({imgs, Ho, Wo, N2}, x.options());
  if (!vcx_dw_pw2(x.data_ptr(), dw1_w.data_ptr(), dw1_b.data_ptr<float>(), dw1_relu ? 1 : 0, W1.data_ptr(),
                  b1.data_ptr<float>(), relu1 ? 1 : 0, dw2_w.data_ptr(), dw2_b.data_ptr<float>(), dw2_relu ? 1 : 0,
                  W2.data_ptr(), b2.data_ptr<float>(), relu2 ? 1 : 0, Y.data_ptr(), (int)imgs, (int)H, (int)W,
                  (int)K1, (int)N1, (int)N2, cur_stream()))
    return at::Tensor();
  return Y;
}

// k BGR frames [k, h, w, 3] uint8 -> their Y4M 4:4:4 records (FRAME header + planes), uint8 [k * (6 + 3 h w)]
at::Tensor bgr_to_y4m(at::Tensor frames) {
  CHK(frames, at::kByte);
  TORCH_CHECK(frames.dim() == 4 && frames.size(3) == 3 && frames.numel() < ((int64_t)1 << 40), "frames [k, h, w, 3] uint8");
  const int64_t k = frames.size(0), h = frames.size(1), w = frames.size(2);
  auto out = at::empty({k * (6 + 3 * h * w)}, frames.options());
  if (k > 0) vcx_bgr_to_y4m(frames.data_ptr<uint8_t>(), out.data_ptr<uint8_t>(), (int)k, (int)w, (int)h, cur_stream());
  return out;
}

// KxK convolution as an implicit GEMM (no im2col matrix): x NHWC bf16 [imgs, H, W, Cs] using
// its first C channels (C % 8 == 0, or C == 4 == Cs), Wt [N, Kp] columns (ky, kx, c)
at::Tensor conv_implicit(at::Tensor x, at::Tensor Wt, at::Tensor bias, int64_t C, int64_t KH, int64_t KW,
                         int64_t stride, int64_t pad, bool relu) {
  CHK(x, at::kBFloat16);
  CHK(Wt, at::kBFloat16);
  CHK(bias, at::kFloat);
  TORCH_CHECK(x.dim() == 4 && Wt.dim() == 2, "x NHWC, Wt [N, Kp]");
  const int64_t imgs = x.size(0), H = x.size(1), W = x.size(2), Cs = x.size(3), N = Wt.size(0), Kp = Wt.size(1);
  TORCH_CHECK(Kp % 32 == 0 && Kp >= KH * KW * C && bias.numel() == N && C <= Cs);
  TORCH_CHECK((C % 8 == 0 && Cs % 8 == 0) || (C == 4 && Cs == 4), "implicit conv: C % 8 == 0, or C == Cs == 4");
  const int64_t Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  auto Y = at::empty({imgs, Ho, Wo, N}, x.options());
  const int S = vcx_vision_ksplit((int)(imgs * Ho * Wo), (int)N, (int)Kp);
  at::Tensor ws = S > 1 ? at::empty({S, imgs * Ho * Wo, N}, x.options().dtype(at::kFloat)) : at::Tensor();
  vcx_conv_implicit(x.data_ptr(), Wt.data_ptr(), bias.data_ptr<float>(), Y.data_ptr(), (int)imgs, (int)H, (int)W,
                    (int)C, (int)Cs, (int)KH, (int)KW, (int)stride, (int)pad, (int)N, (int)Kp, relu ? 1 : 0,
                    S > 1 ? ws.data_ptr<float>() : nullptr, S, S > 1 ? splitk_counters(x) : nullptr, cur_stream());
  return Y;
}

std::vector<at::Tensor> ssd_detect(at::Tensor conf, at::Tensor loc, at::Tensor pri, at::Tensor var, int64_t C,
                                   int64_t bg, double thresh, double nms_thresh, int64_t topk, int64_t keep) {
  CHK(conf, at::kBFloat16);
  CHK(loc, at::kBFloat16);
  CHK(pri, at::kFloat);
  CHK(var, at::kFloat);
  const int64_t N = conf.size(0);
  const int64_t P = pri.numel() / 4;
  TORCH_CHECK(conf.numel() == N * P * C && loc.numel() == N * P * 4 && var.numel() == P * 4);
  TORCH_CHECK(P <= 2048, "ssd_detect: at most 2048 priors per image");
  TORCH_CHECK(topk > 0 && topk <= 256 && keep > 0 && keep <= 4096 && C >= 2 && C <= 63 && bg >= 0 && bg < C);
  TORCH_CHECK((C - 1) * topk <= 4096, "ssd_detect: (C-1)*topk must fit the merge sort");
  auto fo = conf.options().dtype(at::kFloat);
  auto io = conf.options().dtype(at::kInt);
  TORCH_CHECK(C <= 32, "ssd_detect: at most 32 classes");
  auto prob = at::empty({N, C, P}, fo);
  auto cls_out = at::empty({N, C, topk, 5}, fo);
  // every entry is written by the kernels (the background class's count is never read; the merge
  // zero-pads each image's rows past its count): no fill kernels in front of them
  auto cls_cnt = at::empty({N, C}, io);
  auto out = at::empty({N, keep, 7}, fo);
  auto cnt = at::empty({N}, io);
  vcx_ssd_detect(conf.data_ptr(), loc.data_ptr(), pri.data_ptr<float>(), var.data_ptr<float>(), prob.data_ptr<float>(),
                 cls_out.data_ptr<float>(), cls_cnt.data_ptr<int>(), out.data_ptr<float>(), cnt.data_ptr<int>(),
                 (int)N, (int)P, (int)C, (int)bg, (float)thresh, (float)nms_thresh, (int)topk, (int)keep,
                 cur_stream());
  return {out, cnt};
}

at::Tensor annotate(at::Tensor frames, at::Tensor dets, at::Tensor det_cnt, int64_t label, double thresh,
                    int64_t box_bgr, at::Tensor name_mask, int64_t nm_x, int64_t nm_y, int64_t name_bgr,
                    at::Tensor lab_masks, int64_t lm_x, int64_t lm_y, int64_t lab_bgr) {
  CHK(frames, at::kByte);
  CHK(dets, at::kFloat);
  CHK(det_cnt, at::kInt);
  CHK(name_mask, at::kByte);
  CHK(lab_masks, at::kByte);
  TORCH_CHECK(frames.dim() == 4 && frames.size(3) == 3 && dets.dim() == 3 && dets.size(2) == 7);
  TORCH_CHECK(dets.size(0) == frames.size(0) && det_cnt.numel() == frames.size(0));
  TORCH_CHECK(name_mask.dim() == 2 && lab_masks.dim() == 3);
  auto counts = at::zeros({frames.size(0)}, det_cnt.options());
  vcx_annotate(frames.data_ptr<uint8_t>(), (int)frames.size(0), (int)frames.size(1), (int)frames.size(2),
               dets.data_ptr<float>(), det_cnt.data_ptr<int>(), (int)dets.size(1), (int)label, (float)thresh,
               (uint32_t)box_bgr, name_mask.data_ptr<uint8_t>(), (int)name_mask.size(0), (int)name_mask.size(1),
               (int)nm_x, (int)nm_y, (uint32_t)name_bgr, lab_masks.data_ptr<uint8_t>(), (int)lab_masks.size(0),
               (int)lab_masks.size(1), (int)lab_masks.size(2), (int)lm_x, (int)lm_y, (uint32_t)lab_bgr,
               counts.data_ptr<int>(), cur_stream());
  return counts;
}

}  // namespace

void vcx_register_vision(pybind11::module& m) {
  m.def("resize_area_u8", &resize_area_u8);
  m.def("resize_bilinear_u8", &resize_bilinear_u8);
  m.def("blob_bilinear", &blob_bilinear);
  m.def("im2col_nhwc", &im2col_nhwc);
  m.def("dwconv3x3", &dwconv3x3);
  m.def("gemm_bias_act", &gemm_bias_act);
  m.def("gemm_bias_heads", &gemm_bias_heads);
  m.def("dw_pw", &dw_pw);
  m.def("dw_pw2", &dw_pw2);
  m.def("bgr_to_y4m", &bgr_to_y4m);
  m.def("conv_implicit", &conv_implicit);
  m.def("ssd_detect", &ssd_detect);
  m.def("annotate", &annotate);
}
