#include "colour.h"

#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace vcxrt {

// rows [0, h) in up to 8 contiguous bands on their own threads (a 720p frame is ~1 M pixels;
// below 64k pixels it stays on the calling thread)
template <class F>
static void parallel_rows(int64_t h, int64_t w, F&& fn) {
  const int64_t hw = (int64_t)std::max(1u, std::thread::hardware_concurrency());
  const int64_t nt = std::min<int64_t>({8, hw, std::max<int64_t>(1, h * w / 65536), h});
  if (nt <= 1) {
    fn(0, h);
    return;
  }
  std::vector<std::thread> th;
  const int64_t band = (h + nt - 1) / nt;
  for (int64_t t = 1; t < nt; ++t) {
    const int64_t r0 = t * band, r1 = std::min(h, r0 + band);
    if (r0 < r1) th.emplace_back([&fn, r0, r1] { fn(r0, r1); });
  }
  fn(0, std::min(h, band));
  for (auto& x : th) x.join();
}

static inline uint8_t sat(float x) {
  x += 0.5f;
  x = x < 0.f ? 0.f : (x > 255.f ? 255.f : x);
  return (uint8_t)x;  // truncation, as numpy's astype(uint8) after clip
}

void bgr_to_yuv444(const uint8_t* bgr, uint8_t* yuv, int64_t w, int64_t h) {
  const int64_t n = w * h;
  uint8_t* Y = yuv;
  uint8_t* U = yuv + n;
  uint8_t* V = yuv + 2 * n;
  parallel_rows(h, w, [&](int64_t r0, int64_t r1) {
    for (int64_t i = r0 * w; i < r1 * w; ++i) {
      const float b = bgr[3 * i], g = bgr[3 * i + 1], r = bgr[3 * i + 2];
      const float y = 0.299f * r + 0.587f * g + 0.114f * b;
      Y[i] = sat(y);
      U[i] = sat((b - y) * 0.564f + 128.0f);
      V[i] = sat((r - y) * 0.713f + 128.0f);
    }
  });
}

void bgr_to_yuv444_frames(const uint8_t* bgr, uint8_t* yuv, int64_t k, int64_t w, int64_t h) {
  // frames [k, h, w, 3] -> [k, 3, h, w]: whole frames per thread (a 400 x 225 output frame is below
  // the per-frame banding threshold, so one call per frame ran on one core)
  const int64_t n = w * h;
  const int64_t hw = (int64_t)std::max(1u, std::thread::hardware_concurrency());
  const int64_t nt = std::min<int64_t>({8, hw, std::max<int64_t>(1, k * n / 65536), k});
  auto run = [&](int64_t f0, int64_t f1) {
    for (int64_t f = f0; f < f1; ++f) {
      const uint8_t* src = bgr + f * 3 * n;
      uint8_t* Y = yuv + f * 3 * n;
      uint8_t* U = Y + n;
      uint8_t* V = Y + 2 * n;
      for (int64_t i = 0; i < n; ++i) {
        const float b = src[3 * i], g = src[3 * i + 1], r = src[3 * i + 2];
        const float y = 0.299f * r + 0.587f * g + 0.114f * b;
        Y[i] = sat(y);
        U[i] = sat((b - y) * 0.564f + 128.0f);
        V[i] = sat((r - y) * 0.713f + 128.0f);
      }
    }
  };
  if (nt <= 1) {
    run(0, k);
    return;
  }
  std::vector<std::thread> th;
  const int64_t per = (k + nt - 1) / nt;
  for (int64_t t = 1; t < nt; ++t) {
    const int64_t f0 = t * per, f1 = std::min(k, f0 + per);
    if (f0 < f1) th.emplace_back([&run, f0, f1] { run(f0, f1); });
  }
  run(0, std::min(k, per));
  for (auto& x : th) x.join();
}

void yuv_to_bgr(const uint8_t* y, const uint8_t* u, const uint8_t* v, uint8_t* bgr, int64_t w, int64_t h,
                int64_t cw) {
  const bool sub = cw != w;  // 4:2:0
  parallel_rows(h, w, [&](int64_t r0, int64_t r1) {
  for (int64_t r = r0; r < r1; ++r) {
    const uint8_t* yr = y + r * w;
    const int64_t cr = sub ? r / 2 : r;
    const uint8_t* ur = u + cr * cw;
    const uint8_t* vr = v + cr * cw;
    uint8_t* o = bgr + r * w * 3;
    for (int64_t c = 0; c < w; ++c) {
      const int64_t cc = sub ? c / 2 : c;
      const float Y = yr[c], Uc = (float)ur[cc] - 128.0f, Vc = (float)vr[cc] - 128.0f;
      o[3 * c] = sat(Y + 1.773f * Uc);
      o[3 * c + 1] = sat(Y - 0.344f * Uc - 0.714f * Vc);
      o[3 * c + 2] = sat(Y + 1.403f * Vc);
    }
  }
  });
}

// the whole buffer at `off` (pwrite may write less than asked); errno on failure, 0 on success
static int pwrite_all(int fd, const uint8_t* p, int64_t n, int64_t off) {
  while (n > 0) {
    const ssize_t r = ::pwrite(fd, p, (size_t)std::min<int64_t>(n, 1 << 30), (off_t)off);
    if (r < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    p += r;
    n -= r;
    off += r;
  }
  return 0;
}

// f(f0, f1) over frame ranges of [0, k) on up to 8 threads (the calling thread takes the first)
template <class F>
static void parallel_frames(int64_t k, F&& fn) {
  const int64_t hw = (int64_t)std::max(1u, std::thread::hardware_concurrency());
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({8, hw, k}));
  if (nt <= 1) {
    fn(0, k);
    return;
  }
  std::vector<std::thread> th;
  const int64_t per = (k + nt - 1) / nt;
  for (int64_t t = 1; t < nt; ++t) {
    const int64_t f0 = t * per, f1 = std::min(k, f0 + per);
    if (f0 < f1) th.emplace_back([&fn, f0, f1] { fn(f0, f1); });
  }
  fn(0, std::min(k, per));
  for (auto& x : th) x.join();
}

static void y4m_record(const uint8_t* src, uint8_t* r, int64_t n) {
  std::memcpy(r, "FRAME\n", 6);
  uint8_t *Y = r + 6, *U = Y + n, *V = Y + 2 * n;
  for (int64_t i = 0; i < n; ++i) {
    const float b = src[3 * i], g = src[3 * i + 1], rr = src[3 * i + 2];
    const float y = 0.299f * rr + 0.587f * g + 0.114f * b;
    Y[i] = sat(y);
    U[i] = sat((b - y) * 0.564f + 128.0f);
    V[i] = sat((rr - y) * 0.713f + 128.0f);
  }
}

// The mapped write path grows the file with ftruncate (a sparse range) and fills it through a shared
// mapping: if the filesystem cannot back those pages (full disk / tmpfs), the page fault raises SIGBUS
// and kills the process, where a write() would have failed with ENOSPC. So the mapping is
// used only while the filesystem has the bytes the range still needs, with a 64 MB margin for other
// writers; otherwise the positional write path runs and reports the error as an exception.
static bool room_for(int fd, const struct stat& st, int64_t end) {
  const int64_t need = end - std::min<int64_t>(end, (int64_t)st.st_blocks * 512);
  if (need <= 0) return true;
  struct statvfs vs{};
  if (::fstatvfs(fd, &vs) != 0) return false;
  return (int64_t)vs.f_bavail * (int64_t)vs.f_frsize > need + (int64_t(64) << 20);
}

// `n` bytes at `off` of fd: a regular file grown and the range mapped and filled on up to 8 threads
// (the Y4M records converted on the GPU arrive as bytes), else one positional write
int64_t write_bytes(int fd, int64_t off, const uint8_t* src, int64_t n) {
  if (n <= 0) return 0;
  struct stat st{};
  if (::fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && room_for(fd, st, off + n)) {
    if (st.st_size < off + n && ::ftruncate(fd, (off_t)(off + n)) != 0)
      throw std::runtime_error(std::string("write_bytes: ftruncate: ") + std::strerror(errno));
    const int64_t pg = ::sysconf(_SC_PAGESIZE), base = off - off % pg, len = off + n - base;
    void* m = ::mmap(nullptr, (size_t)len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, (off_t)base);
    if (m != MAP_FAILED) {
      uint8_t* dst = (uint8_t*)m + (off - base);
      const int64_t parts = std::max<int64_t>(1, std::min<int64_t>(8, n >> 20));  // >= 1 MB per thread
      const int64_t per = (n + parts - 1) / parts;
      parallel_frames(parts, [&](int64_t p0, int64_t p1) {
        const int64_t a = p0 * per, b = std::min(n, p1 * per);
        if (a < b) std::memcpy(dst + a, src + a, (size_t)(b - a));
      });
      ::munmap(m, (size_t)len);
      return n;
    }
  }
  const int e = pwrite_all(fd, src, n, off);
  if (e) throw std::runtime_error(std::string("write_bytes: ") + std::strerror(e));
  return n;
}

int64_t write_frames(int fd, int64_t off, const uint8_t* bgr, int64_t k, int64_t w, int64_t h, bool y4m) {
  // k BGR frames [k, h, w, 3] at byte offset `off` of fd, as raw frames (npy body) or as Y4M 4:4:4
  // records ("FRAME\n" + Y, U, V planes). A regular file is grown to cover the range and the range is
  // MAPPED: frame ranges are copied / converted straight into the page cache on up to 8 threads (page
  // faults of a shared mapping run in parallel; write()/pwrite() of one file serialise on its inode
  // lock, and one thread moved only ~3 GB/s into tmpfs: 9-12 ms per 27 MB chunk, the video job's sink
  // bound, profiles/r5_video_job.txt). Anything else (a pipe) gets one positional write.
  const int64_t n = w * h, fb = 3 * n, rec = y4m ? fb + 6 : fb, total = k * rec;
  if (k <= 0) return 0;
  struct stat st{};
  if (::fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && room_for(fd, st, off + total)) {
    if (st.st_size < off + total && ::ftruncate(fd, (off_t)(off + total)) != 0)
      throw std::runtime_error(std::string("write_frames: ftruncate: ") + std::strerror(errno));
    const int64_t pg = ::sysconf(_SC_PAGESIZE), base = off - off % pg, len = off + total - base;
    void* m = ::mmap(nullptr, (size_t)len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, (off_t)base);
    if (m != MAP_FAILED) {
      uint8_t* dst = (uint8_t*)m + (off - base);
      parallel_frames(k, [&](int64_t f0, int64_t f1) {
        if (!y4m) {
          std::memcpy(dst + f0 * fb, bgr + f0 * fb, (size_t)((f1 - f0) * fb));
          return;
        }
        for (int64_t f = f0; f < f1; ++f) y4m_record(bgr + f * fb, dst + f * rec, n);
      });
      ::munmap(m, (size_t)len);
      return total;
    }
  }
  std::vector<uint8_t> buf;
  const uint8_t* out = bgr;
  if (y4m) {
    buf.resize((size_t)total);
    parallel_frames(k, [&](int64_t f0, int64_t f1) {
      for (int64_t f = f0; f < f1; ++f) y4m_record(bgr + f * fb, buf.data() + f * rec, n);
    });
    out = buf.data();
  }
  const int e = pwrite_all(fd, out, total, off);
  if (e) throw std::runtime_error(std::string("write_frames: ") + std::strerror(e));
  return total;
}

}  // namespace vcxrt
