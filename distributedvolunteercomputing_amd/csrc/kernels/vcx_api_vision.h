// Launchers of kernels/vision.hip (MobileNet-SSD inference path).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

void vcx_resize_area_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int h, int w, hipStream_t s);
void vcx_resize_bilinear_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int h, int w, hipStream_t s);
void vcx_blob_bilinear(const uint8_t* src, void* dst, int N, int H, int W, int S, float scale, float mean,
                       hipStream_t s);
void vcx_im2col_nhwc(const void* x, void* out, int N, int H, int W, int C, int Cs, int Ho, int Wo, int KH, int KW,
                     int stride, int pad, int Kp, hipStream_t s);
void vcx_dwconv3x3(const void* x, const void* w, const float* b, void* y, int N, int H, int W, int C, int Ho, int Wo,
                   int stride, int relu, hipStream_t s);
int vcx_vision_ksplit(int M, int N, int K);
void vcx_gemm_bias_act_mapped(const void* X, const void* Wt, const float* bias, void* Y, int M, int N, int K, int ldy,
                              int relu, void* Y2, int split, int ldy2, int rpi, int64_t img_stride,
                              int64_t img_stride2, float* ws, int S, int* cnt, hipStream_t s);
void vcx_conv_implicit(const void* x, const void* Wt, const float* bias, void* Y, int imgs, int H, int W, int C,
                       int Cs, int KH, int KW, int stride, int pad, int N, int Kp, int relu, float* ws, int S,
                       int* cnt, hipStream_t s);
void vcx_dw_pw(const void* x, const void* dw_w, const float* dw_b, int dw_relu, const void* Wt, const float* bias,
               void* Y, int imgs, int H, int W, int K, int stride, int N, int relu, hipStream_t s);
bool vcx_dw_pw2(const void* x, const void* dw1_w, const float* dw1_b, int dw1_relu, const void* W1, const float* b1,
                int relu1, const void* dw2_w, const float* dw2_b, int dw2_relu, const void* W2, const float* b2,
                int relu2, void* Y, int imgs, int H, int W, int K1, int N1, int N2, hipStream_t s);
void vcx_gemm_bias_act(const void* X, const void* Wt, const float* bias, void* Y, int M, int N, int K, int ldy,
                       int relu, float* ws, int S, int* cnt, hipStream_t s);
void vcx_ssd_detect(const void* conf, const void* loc, const float* pri, const float* var, float* prob,
                    float* cls_out, int* cls_cnt, float* out, int* out_cnt, int N, int P, int C, int bg, float thresh,
                    float nms_thresh, int topk, int keep, hipStream_t s);
void vcx_bgr_to_y4m(const uint8_t* bgr, uint8_t* out, int k, int w, int h, hipStream_t s);
void vcx_annotate(uint8_t* frames, int N, int h, int w, const float* dets, const int* det_cnt, int keep, int label,
                  float thresh, uint32_t box_bgr, const uint8_t* name_mask, int nm_h, int nm_w, int nm_x, int nm_y,
                  uint32_t name_bgr, const uint8_t* lab_masks, int lm_n, int lm_h, int lm_w, int lm_x, int lm_y,
                  uint32_t lab_bgr, int* counts_out, hipStream_t s);
