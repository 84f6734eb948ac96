// Torch bindings for the gradient-compression kernels (kernels/compress.hip).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/vcx_api_compress.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHK(x)                                                  \
  TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor");       \
  TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")

// state: int32[8] on device, prepared by the caller: {0, k, 0, ...}; hist: int32[topk_hist_words()]
// zeros (left zeroed); idx_out / val_out zeroed by the caller (unfilled slots must read 0)
void topk_ef(at::Tensor g, at::Tensor e, int64_t k, at::Tensor state, at::Tensor hist, at::Tensor idx_out,
             at::Tensor val_out) {
  CHK(g);
  CHK(e);
  CHK(state);
  CHK(hist);
  CHK(idx_out);
  CHK(val_out);
  TORCH_CHECK(e.scalar_type() == at::kFloat && g.numel() == e.numel());
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat);
  TORCH_CHECK(state.scalar_type() == at::kInt && state.numel() >= 8 && hist.scalar_type() == at::kInt &&
              hist.numel() >= vcx_topk_hist_words());
  TORCH_CHECK((reinterpret_cast<uintptr_t>(state.data_ptr()) & 7) == 0, "state must be 8-byte aligned");
  TORCH_CHECK(idx_out.scalar_type() == at::kInt && idx_out.numel() >= k && val_out.numel() >= k);
  TORCH_CHECK(val_out.scalar_type() == at::kBFloat16 || val_out.scalar_type() == at::kFloat);
  TORCH_CHECK(k > 0 && k <= g.numel() && g.numel() < INT32_MAX);
  vcx_topk_ef(g.data_ptr(), g.scalar_type() == at::kBFloat16, e.data_ptr<float>(), g.numel(), (int)k,
              state.data_ptr<int>(), (uint32_t*)hist.data_ptr<int>(), idx_out.data_ptr<int32_t>(), val_out.data_ptr(),
              val_out.scalar_type() == at::kBFloat16, cur_stream());
}

// indices come from other peers: out-of-range ones are dropped inside the kernel (no host sync)
void scatter_add(at::Tensor idx, at::Tensor val, double scale, at::Tensor dense) {
  CHK(idx);
  CHK(val);
  CHK(dense);
  TORCH_CHECK(idx.scalar_type() == at::kInt && dense.scalar_type() == at::kFloat && idx.numel() == val.numel());
  TORCH_CHECK(val.scalar_type() == at::kBFloat16 || val.scalar_type() == at::kFloat);
  TORCH_CHECK(dense.numel() < INT32_MAX);
  vcx_scatter_add(idx.data_ptr<int32_t>(), val.data_ptr(), val.scalar_type() == at::kBFloat16, idx.numel(),
                  (float)scale, dense.data_ptr<float>(), dense.numel(), cur_stream());
}

// wire: int32 [P, L]; per peer k indices then k values of `val_dtype` (bf16 or fp32) packed after them
void scatter_add_packed(at::Tensor wire, int64_t k, bool val_bf16, double scale, at::Tensor dense) {
  CHK(wire);
  CHK(dense);
  TORCH_CHECK(wire.scalar_type() == at::kInt && wire.dim() == 2 && dense.scalar_type() == at::kFloat);
  const int64_t L = wire.size(1), vw = val_bf16 ? (k + 1) / 2 : k;
  TORCH_CHECK(k > 0 && L >= k + vw, "scatter_add_packed: wire rows too short for k pairs");
  TORCH_CHECK(dense.numel() < INT32_MAX && wire.size(0) * k < INT32_MAX);
  vcx_scatter_add_packed(wire.data_ptr<int32_t>(), (int)wire.size(0), (int)k, L, val_bf16, (float)scale,
                         dense.data_ptr<float>(), dense.numel(), cur_stream());
}

int64_t topk_hist_words() { return vcx_topk_hist_words(); }

void check_desc(const at::Tensor& d, int64_t nmat) {
  CHK(d);
  TORCH_CHECK(d.scalar_type() == at::kByte && d.numel() == nmat * vcx_psgd_desc_size(), "bad descriptor table");
}

// M += G (error feedback, skipped when G is None) fused with P = M Q over every matrix; lazy: the
// previous reconstruct ran with update_m=false, so M -= P_prev Q^T is applied first
void psgd_mq(at::Tensor desc, int64_t nmat, int64_t nblocks, at::Tensor M, at::Tensor Q, at::Tensor P, int64_t rank,
             std::optional<at::Tensor> G, bool lazy) {
  check_desc(desc, nmat);
  CHK(M);
  CHK(Q);
  CHK(P);
  const void* g = nullptr;
  if (G.has_value()) {
    CHK((*G));
    TORCH_CHECK(G->scalar_type() == at::kBFloat16 && G->numel() == M.numel(), "psgd_mq: G must be bf16 like M");
    g = G->data_ptr();
  }
  vcx_psgd_mq(desc.data_ptr(), (int)nmat, (int)nblocks, M.data_ptr<float>(), g, Q.data_ptr<float>(),
              P.data_ptr<float>(), (int)rank, lazy ? 1 : 0, cur_stream());
}

void psgd_mtp(at::Tensor desc, int64_t nmat, int64_t nblocks, at::Tensor M, at::Tensor P, at::Tensor Q, int64_t rank) {
  check_desc(desc, nmat);
  CHK(M);
  CHK(Q);
  CHK(P);
  vcx_psgd_mtp(desc.data_ptr(), (int)nmat, (int)nblocks, M.data_ptr<float>(), P.data_ptr<float>(),
               Q.data_ptr<float>(), (int)rank, cur_stream());
}

void psgd_orth(at::Tensor desc, int64_t nmat, int64_t nblocks, at::Tensor P, at::Tensor G, int64_t rank) {
  check_desc(desc, nmat);
  CHK(P);
  CHK(G);
  TORCH_CHECK(P.scalar_type() == at::kFloat && G.scalar_type() == at::kFloat && G.numel() >= 2 * nmat * rank * rank,
              "psgd_orth: G must hold 2 * nmat * rank^2 floats");
  vcx_psgd_orth(desc.data_ptr(), (int)nmat, (int)nblocks, P.data_ptr<float>(), G.data_ptr<float>(), (int)rank,
                cur_stream());
}

void psgd_reconstruct(at::Tensor desc, int64_t nmat, int64_t nblocks, at::Tensor M, at::Tensor P, at::Tensor Q,
                      at::Tensor out, int64_t rank, bool update_m) {
  check_desc(desc, nmat);
  CHK(M);
  CHK(P);
  CHK(Q);
  CHK(out);
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.numel() == M.numel());
  vcx_psgd_reconstruct(desc.data_ptr(), (int)nmat, (int)nblocks, M.data_ptr<float>(), P.data_ptr<float>(),
                       Q.data_ptr<float>(), out.data_ptr(), (int)rank, update_m ? 1 : 0, cur_stream());
}

void ef_accum(at::Tensor g, at::Tensor e) {
  CHK(g);
  CHK(e);
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 && e.scalar_type() == at::kFloat && g.numel() == e.numel() &&
              g.numel() % 8 == 0);
  vcx_ef_accum(g.data_ptr(), e.data_ptr<float>(), g.numel(), cur_stream());
}

}  // namespace

void vcx_register_compress(pybind11::module& m) {
  m.def("topk_ef", &topk_ef);
  m.def("scatter_add", &scatter_add);
  m.def("scatter_add_packed", &scatter_add_packed);
  m.def("topk_hist_words", &topk_hist_words);
  m.def("psgd_mq", &psgd_mq, pybind11::arg("desc"), pybind11::arg("nmat"), pybind11::arg("nblocks"),
        pybind11::arg("M"), pybind11::arg("Q"), pybind11::arg("P"), pybind11::arg("rank"),
        pybind11::arg("G") = pybind11::none(), pybind11::arg("lazy") = false);
  m.def("psgd_mtp", &psgd_mtp);
  m.def("psgd_orth", &psgd_orth);
  m.def("psgd_orth_rows", &vcx_psgd_orth_rows);
  m.def("psgd_reconstruct", &psgd_reconstruct, pybind11::arg("desc"), pybind11::arg("nmat"), pybind11::arg("nblocks"),
        pybind11::arg("M"), pybind11::arg("P"), pybind11::arg("Q"), pybind11::arg("out"), pybind11::arg("rank"),
        pybind11::arg("update_m") = true);
  m.def("ef_accum", &ef_accum);
  m.def("psgd_desc_size", &vcx_psgd_desc_size);
  m.def("psgd_rows_per_block", &vcx_psgd_rows_per_block);
  m.def("psgd_mtp_rows", &vcx_psgd_mtp_rows);
  m.def("psgd_mtp_cols", &vcx_psgd_mtp_cols);
}
