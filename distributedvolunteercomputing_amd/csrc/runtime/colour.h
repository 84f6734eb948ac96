// Host colour conversion for the video I/O path (Y4M sources and sinks): BGR <-> planar YUV
// (BT.601 full range, the formulas of io/video.py, evaluated in float32 in the same order so the
// result is bit-identical to the numpy reference). The reference does this inside OpenCV's C++
// VideoCapture / VideoWriter (/root/reference/worker.py:86,110,131); numpy needed 13-20 ms per
// 720p frame; these loops run over up to 8 row bands with the GIL released.
#pragma once
#include <cstdint>

namespace vcxrt {

// bgr [h][w][3] -> yuv planes [3][h][w]
void bgr_to_yuv444(const uint8_t* bgr, uint8_t* yuv, int64_t w, int64_t h);
// k frames [k, h, w, 3] -> [k, 3, h, w] planar (one Y4M 4:4:4 frame body each), frames across threads
void bgr_to_yuv444_frames(const uint8_t* bgr, uint8_t* yuv, int64_t k, int64_t w, int64_t h);
// planes y [h][w], u/v [ch][cw] with cw = w (4:4:4) or (w + 1) / 2 (4:2:0, 2x2 replication) -> bgr [h][w][3]
void yuv_to_bgr(const uint8_t* y, const uint8_t* u, const uint8_t* v, uint8_t* bgr, int64_t w, int64_t h, int64_t cw);

// k BGR frames written at byte `off` of fd (raw, or as Y4M 4:4:4 records): a regular file is grown and the
// range mapped and filled on several threads, anything else gets one positional write;
// returns the bytes written (throws std::runtime_error on a write error)
int64_t write_frames(int fd, int64_t off, const uint8_t* bgr, int64_t k, int64_t w, int64_t h, bool y4m);
// n bytes at `off` of fd (a regular file through a shared mapping filled on several threads); returns n
int64_t write_bytes(int fd, int64_t off, const uint8_t* src, int64_t n);

}  // namespace vcxrt
