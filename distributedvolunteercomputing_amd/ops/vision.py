"""Vision ops for the MobileNet-SSD video job: resize/blob preprocessing, depthwise conv,
GEMM with bias/ReLU epilogue, SSD detection output, annotation (reference SURVEY.md §2.5 K1-K14).

GPU tensors run the gfx950 kernels of ``vision.hip``; CPU tensors run reference
implementations with the same arithmetic (used by CPU volunteers and as test oracles).
"""
from __future__ import annotations

import functools
import os

import numpy as np

import torch
import torch.nn.functional as F

from ._lib import native, use_native

# BGR colours used by the reference annotation (worker.py:268-276)
BLUE, RED, GREEN = (255, 0, 0), (0, 0, 255), (0, 255, 0)


def _pack_bgr(c):
    return int(c[0]) | (int(c[1]) << 8) | (int(c[2]) << 16)


# ----------------------------------------------------------------------------- resize
def _area_weights(src: int, dst: int) -> torch.Tensor:
    """[dst, src] matrix of INTER_AREA box-filter weights (rows sum to 1)."""
    s = src / dst
    w = torch.zeros(dst, src, dtype=torch.float64)
    for d in range(dst):
        f0, f1 = d * s, min((d + 1) * s, src)
        for x in range(int(f0), min(int(np.ceil(f1)), src)):
            ov = min(f1, x + 1) - max(f0, x)
            if ov > 0:
                w[d, x] = ov
    return (w / w.sum(1, keepdim=True)).float()


def _bilinear_weights(src: int, dst: int) -> torch.Tensor:
    s = src / dst
    w = torch.zeros(dst, src, dtype=torch.float32)
    for d in range(dst):
        f = max((d + 0.5) * s - 0.5, 0.0)
        x0 = min(int(f), src - 1)
        x1 = min(x0 + 1, src - 1)
        a = f - x0
        w[d, x0] += 1 - a
        w[d, x1] += a
    return w


def _separable(frames_u8: torch.Tensor, wy: torch.Tensor, wx: torch.Tensor) -> torch.Tensor:
    f = frames_u8.float()
    wy, wx = wy.to(f.device), wx.to(f.device)
    y = torch.einsum("yh,nhwc->nywc", wy, f)
    y = torch.einsum("xw,nywc->nyxc", wx, y)
    return y


def resize_area_u8(frames: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """[N,H,W,3] uint8 -> [N,h,w,3] uint8 with cv2.INTER_AREA semantics (downscale)."""
    if use_native(frames):
        return native().resize_area_u8(frames.contiguous(), h, w)
    y = _separable(frames, _area_weights(frames.shape[1], h), _area_weights(frames.shape[2], w))
    return y.round().clamp(0, 255).to(torch.uint8)


def resize_bilinear_u8(frames: torch.Tensor, h: int, w: int) -> torch.Tensor:
    if use_native(frames):
        return native().resize_bilinear_u8(frames.contiguous(), h, w)
    y = _separable(frames, _bilinear_weights(frames.shape[1], h), _bilinear_weights(frames.shape[2], w))
    return y.round().clamp(0, 255).to(torch.uint8)


def resize_width(frames: torch.Tensor, width: int = 400) -> torch.Tensor:
    """imutils.resize(frame, width=400): keep aspect, INTER_AREA (bilinear when upscaling)."""
    H, W = frames.shape[1], frames.shape[2]
    h = int(H * width / W)
    if W == width and H == h:
        return frames
    if width <= W and h <= H:
        return resize_area_u8(frames, h, width)
    return resize_bilinear_u8(frames, h, width)


def blob_from_frames(frames: torch.Tensor, size: int = 300, scale: float = 0.007843, mean: float = 127.5):
    """cv2.dnn.blobFromImage(cv2.resize(f, (S,S)), scale, (S,S), mean) for a batch, as
    NHWC bf16 [N, S, S, 4] (channel 3 is zero padding)."""
    if use_native(frames):
        return native().blob_bilinear(frames.contiguous(), size, scale, mean)
    r = resize_bilinear_u8(frames, size, size).float()
    out = torch.zeros(frames.shape[0], size, size, 4, device=frames.device)
    out[..., :3] = (r - mean) * scale
    return out.to(torch.bfloat16)


# ----------------------------------------------------------------------------- conv / gemm
def dw_pair_weights(w9c):
    """[9, C] tap-major depthwise weights -> the paired layout of the dot2 kernels, [5, C, 2] bf16:
    row p < 4 holds (w[2p], w[2p+1]) per channel, row 4 holds (w[8], 0) for even channels and
    (0, w[8]) for odd ones (csrc/kernels/vision.hip dw9_accum)."""
    C = w9c.shape[1]
    w = w9c.to(torch.bfloat16)
    wp = torch.zeros(5, C, 2, dtype=torch.bfloat16, device=w9c.device)
    wp[:4, :, 0] = w[0:8:2]
    wp[:4, :, 1] = w[1:8:2]
    wp[4, 0::2, 0] = w[8, 0::2]
    wp[4, 1::2, 1] = w[8, 1::2]
    return wp


def _dw_unpair(wp):
    w = torch.empty(9, wp.shape[1], dtype=wp.dtype, device=wp.device)
    w[0:8:2], w[1:8:2] = wp[:4, :, 0], wp[:4, :, 1]
    w[8] = wp[4, :, 0] + wp[4, :, 1]
    return w


def dwconv3x3(x, w, b, stride, relu=True):
    """NHWC depthwise 3x3, pad 1. w: [9, C] bf16 tap-major or the paired [5, C, 2] layout of
    dw_pair_weights; b: [C] fp32."""
    if use_native(x):
        return native().dwconv3x3(x, w if w.dim() == 3 else dw_pair_weights(w), b, stride, relu)
    w9c = _dw_unpair(w) if w.dim() == 3 else w
    C = x.shape[3]
    wt = w9c.float().t().reshape(C, 1, 3, 3)
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), wt, b.float(), stride=stride, padding=1, groups=C)
    if relu:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1).contiguous().to(x.dtype)


# (K, N, stride) of the MobileNet blocks whose 2-D-tile fused depthwise->pointwise kernel
# (csrc/kernels/vision.hip) beats the two kernels. The persistent form (dwpw_persist_kernel: weights
# in LDS once per workgroup, next tile's halo loaded during this tile's GEMM and stores; default)
# wins for conv1..conv3: 325 us for the three vs 405 as conv1 fused + two kernels each for conv2 and
# conv3, detector chunk 1.22 vs 1.33 ms (profiles/r3_dwpw_persist_ab.txt). The one-tile form
# (VCX_DWPW_PERSIST=0) only wins for conv1 (its conv2/conv3 instances run 199 / 179 us vs 136 / 145
# unfused: one tile's load -> depthwise -> GEMM -> store phases do not overlap), so that setting
# fuses conv1 alone; VCX_DWPW=tile1 / tile3 choose explicitly.
DWPW_TILE_ALL = {(32, 64, 1), (64, 128, 2), (128, 128, 1)}
DWPW_TILE = DWPW_TILE_ALL if os.environ.get("VCX_DWPW_PERSIST", "1") != "0" else {(32, 64, 1)}


def dw_pw(x, wp, db, dw_relu, stride, Wt, bias, relu=True):
    """A MobileNet block as one kernel: depthwise 3x3 (pad 1) + bias (+ReLU) on NHWC x [N, H, W, K],
    then the pointwise GEMM with Wt [Cout, K] + bias (+ReLU) -> [N, Ho, Wo, Cout]. wp: paired
    depthwise weights (dw_pair_weights). The depthwise activation is rounded to bf16 as the
    two-kernel path rounds it, and never goes through memory."""
    if use_native(x):
        return native().dw_pw(x, wp, db, dw_relu, stride, Wt, bias, relu)
    d = dwconv3x3(x, wp, db, stride, dw_relu)
    N, Ho, Wo, K = d.shape
    return gemm_bias_act(d.reshape(-1, K), Wt, bias, relu).view(N, Ho, Wo, -1)


def dw_pw2(x, b1, b2):
    """Two MobileNet blocks (conv1: depthwise s1 + pointwise, conv2: depthwise s2 + pointwise) as ONE
    kernel where an instance exists (csrc/kernels/vision.hip dwpw2_persist_kernel: the first block's
    output stays in LDS), else the two fused-block kernels. b1 / b2: dicts with the depthwise paired
    weights / bias / relu ("dw_w", "dw_b", "dw_relu") and the pointwise "w", "b", "relu" of each block."""
    if use_native(x):
        y = native().dw_pw2(x, b1["dw_w"], b1["dw_b"], b1["dw_relu"], b1["w"], b1["b"], b1["relu"],
                            b2["dw_w"], b2["dw_b"], b2["dw_relu"], b2["w"], b2["b"], b2["relu"])
        if y is not None and y.numel() > 0:
            return y
    h = dw_pw(x, b1["dw_w"], b1["dw_b"], b1["dw_relu"], 1, b1["w"], b1["b"], b1["relu"])
    return dw_pw(h, b2["dw_w"], b2["dw_b"], b2["dw_relu"], 2, b2["w"], b2["b"], b2["relu"])


def gemm_bias_act(X, Wt, bias=None, relu=False):
    """Y = act(X . Wt^T + bias): X [M,K], Wt [N,K] bf16, bias [N] fp32 -> [M,N] bf16."""
    if use_native(X):
        return native().gemm_bias_act(X, Wt, bias, relu)
    y = X.float() @ Wt.float().t()
    if bias is not None:
        y = y + bias.float()
    if relu:
        y = F.relu(y)
    return y.to(X.dtype)


def im2col_nhwc(x, C, k, stride, pad, Kp):
    if use_native(x):
        return native().im2col_nhwc(x, C, k, stride, pad, Kp)
    xc = x[..., :C].permute(0, 3, 1, 2).float()
    N, _, H, W = xc.shape
    cols = F.unfold(xc, k, padding=pad, stride=stride)  # [N, C*k*k, L] with (c, ky, kx) order
    L = cols.shape[-1]
    cols = cols.view(N, C, k * k, L).permute(0, 3, 2, 1).reshape(N * L, k * k * C)  # (ky,kx,c)
    out = torch.zeros(N * L, Kp, device=x.device)
    out[:, : k * k * C] = cols
    return out.to(x.dtype)


# ----------------------------------------------------------------------------- detection
def ssd_detect(conf_logits, loc, priors, variances, *, num_classes=21, background=0, conf_thresh=0.25,
               nms_thresh=0.45, top_k=100, keep_top_k=100):
    """conf_logits [N, P*C] raw (softmax fused), loc [N, P*4] -> (dets [N, keep, 7], counts [N])."""
    if use_native(conf_logits):
        return native().ssd_detect(conf_logits.contiguous(), loc.contiguous(), priors.float().contiguous(),
                                   variances.float().contiguous(), num_classes, background, conf_thresh,
                                   nms_thresh, top_k, keep_top_k)
    from ..models.caffe import detection_output

    N = conf_logits.shape[0]
    P = priors.numel() // 4
    prob = torch.softmax(conf_logits.float().view(N, P, num_classes), -1).view(N, -1)
    lists = detection_output(loc.float(), prob, priors.float(), variances.float(), num_classes=num_classes,
                             background=background, conf_thresh=conf_thresh, nms_thresh=nms_thresh, top_k=top_k,
                             keep_top_k=keep_top_k)
    out = torch.zeros(N, keep_top_k, 7)
    cnt = torch.zeros(N, dtype=torch.int32)
    for n, d in enumerate(lists):
        k = min(len(d), keep_top_k)
        out[n, :k] = d[:k]
        cnt[n] = k
    return out, cnt


# ----------------------------------------------------------------------------- annotation
@functools.lru_cache(maxsize=256)
def text_mask(text: str) -> np.ndarray:
    """Rasterise `text` with Pillow's built-in bitmap font -> uint8 mask [h, w] (cv2.putText
    with Hershey fonts is unavailable here; glyph shapes differ, placement follows cv2)."""
    from PIL import Image, ImageDraw, ImageFont

    font = ImageFont.load_default()
    x0, y0, x1, y1 = font.getbbox(text) if text else (0, 0, 1, 1)
    w, h = max(1, x1), max(1, y1)
    im = Image.new("L", (w, h), 0)
    ImageDraw.Draw(im).text((0, 0), text, fill=255, font=font)
    m = (np.asarray(im) > 127).astype(np.uint8)
    # thickness 2 in the reference: dilate by one pixel to the right/bottom
    m2 = m.copy()
    m2[:, 1:] |= m[:, :-1]
    m2[1:, :] |= m[:-1, :]
    return m2


@functools.lru_cache(maxsize=8)
def label_masks(cls_name: str = "person", max_count: int = 100) -> np.ndarray:
    """Stack of "<cls>: k" masks for k = 0..max_count, padded to a common size."""
    ms = [text_mask(f"{cls_name}: {k}") for k in range(max_count + 1)]
    h = max(m.shape[0] for m in ms)
    w = max(m.shape[1] for m in ms)
    out = np.zeros((len(ms), h, w), np.uint8)
    for i, m in enumerate(ms):
        out[i, : m.shape[0], : m.shape[1]] = m
    return out


def _draw_np(frame, dets, nd, label, thresh, name_mask, name_xy, lab_masks, lab_xy):
    h, w = frame.shape[:2]
    count = 0

    def put(x, y, c):
        if 0 <= x < w and 0 <= y < h:
            frame[y, x] = c

    for d in dets[:nd]:
        if int(d[1]) != label or d[2] <= thresh:
            continue
        count += 1
        x0, y0, x1, y1 = int(d[3] * w), int(d[4] * h), int(d[5] * w), int(d[6] * h)
        bw, bh = x1 - x0 + 1, y1 - y0 + 1
        if bw <= 0 or bh <= 0 or bw > 4 * w or bh > 4 * h:
            continue
        for x in range(x0, x1 + 1):
            for y, dy in ((y0, -1), (y1, 1)):
                put(x, y, BLUE)
                put(x, y + dy, BLUE)
        for y in range(y0, y1 + 1):
            for x, dx in ((x0, -1), (x1, 1)):
                put(x, y, BLUE)
                put(x + dx, y, BLUE)
    ys, xs = np.nonzero(name_mask)
    for y, x in zip(ys, xs):
        put(name_xy[0] + x, name_xy[1] + y, RED)
    k = min(count, len(lab_masks) - 1)
    ys, xs = np.nonzero(lab_masks[k])
    for y, x in zip(ys, xs):
        put(lab_xy[0] + x, lab_xy[1] + y, GREEN)
    return count


_MASKS: dict = {}


def annotate(frames, dets, counts, requester: str, *, label=15, cls_name="person", thresh=0.2):
    """In-place: boxes for `label` detections with conf > thresh, requester name at (10,25),
    "<cls>: k" at (10, h-20) (cv2.putText origins are text baselines). Returns per-frame counts."""
    h = frames.shape[1]
    dev = frames.device
    key = (requester, cls_name, str(dev))
    masks = _MASKS.get(key)
    if masks is None:  # rasterised (and uploaded) once per (requester, class, device), not per chunk
        nm, lm = text_mask(requester), label_masks(cls_name)
        masks = _MASKS[key] = (nm, lm, torch.from_numpy(nm).to(dev), torch.from_numpy(lm).to(dev))
    nm, lm, nm_d, lm_d = masks
    name_xy = (10, 25 - nm.shape[0] + 2)
    lab_xy = (10, h - 20 - lm.shape[1] + 2)
    if use_native(frames):
        return native().annotate(frames, dets.contiguous(), counts.to(torch.int32).contiguous(), label, thresh,
                                 _pack_bgr(BLUE), nm_d, name_xy[0], name_xy[1],
                                 _pack_bgr(RED), lm_d, lab_xy[0], lab_xy[1], _pack_bgr(GREEN))
    fr = frames.numpy()
    dn = dets.numpy()
    cn = counts.numpy()
    out = [_draw_np(fr[i], dn[i], int(cn[i]), label, thresh, nm, name_xy, lm, lab_xy) for i in range(fr.shape[0])]
    return torch.tensor(out, dtype=torch.int32)
