// Launchers of kernels/compress.hip (top-k + error feedback, PowerSGD).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

void vcx_topk_ef(const void* g, int g_is_bf16, float* e, int64_t n, int k, int* st, uint32_t* hist,
                 int32_t* idx_out, void* val_out, int val_is_bf16, hipStream_t s);
int vcx_topk_hist_words();  // size of the histogram scratch topk_ef needs (uint32 words)
// dense[idx] += scale * val over m pairs; indices outside [0, n) are dropped
void vcx_scatter_add(const int32_t* idx, const void* val, int val_is_bf16, int64_t m, float scale, float* dense,
                     int64_t n, hipStream_t s);
// same over P all-gathered wire blocks of L int32 words each: k indices then k packed values
void vcx_scatter_add_packed(const int32_t* wire, int P, int k, int64_t L, int val_is_bf16, float scale, float* dense,
                            int64_t n, hipStream_t s);
// M += G (bf16, G may be null) fused with P = M Q; lazy: first M -= P_prev Q^T (P_prev = P on entry)
void vcx_psgd_mq(const void* desc, int nmat, int nblocks, float* M, const void* G, const float* Q, float* P, int rank,
                 int lazy, hipStream_t s);
void vcx_psgd_mtp(const void* desc, int nmat, int nblocks, const float* M, const float* P, float* Q, int rank,
                  hipStream_t s);
// CholeskyQR2 of every matrix's P (blocks of psgd_orth_rows() rows); G: 2 * nmat * rank^2 floats scratch
void vcx_psgd_orth(const void* desc, int nmat, int nblocks, float* P, float* G, int rank, hipStream_t s);
int vcx_psgd_orth_rows();
void vcx_psgd_reconstruct(const void* desc, int nmat, int nblocks, float* M, const float* P, const float* Q,
                          void* out, int rank, int update_m, hipStream_t s);
void vcx_ef_accum(const void* g, float* e, int64_t n, hipStream_t s);
int vcx_psgd_desc_size();
// block tables: psgd_mq / psgd_reconstruct take rows_per_block rows per block; psgd_mtp blocks are
// (row slab of mtp_rows) x (column chunk of mtp_cols)
int vcx_psgd_rows_per_block();
int vcx_psgd_mtp_rows();
int vcx_psgd_mtp_cols();
