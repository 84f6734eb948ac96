"""Caffe model format: prototxt parser, caffemodel (protobuf wire) reader/writer, and a
plain-PyTorch graph interpreter used as the numerics oracle.

The reference loads its detector with ``cv2.dnn.readNetFromCaffe(prototxt, caffemodel)``
(/root/reference/worker.py:186-194). The weights file is absent from the reference
(``.MISSING_LARGE_BLOBS``), so ``load_caffemodel`` is exercised on files we serialise
ourselves (``save_caffemodel``) and missing blobs fall back to Caffe-style random init
(msra weights, constant-0 biases — the fillers the prototxt itself names).

No compiled ``caffe.proto`` is needed: the wire decoder below understands just the fields
of ``NetParameter``/``LayerParameter``/``BlobProto`` that carry weights
(layer=100 [V1: layers=2], name=1, blobs=7, BlobProto.shape=7{dim=1}, data=5, legacy
num/channels/height/width=1..4).
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

# ============================================================================ prototxt
_TOK = re.compile(r'\s*(?:(#[^\n]*)|([A-Za-z_][\w]*)\s*(:)?|(\{)|(\})|("(?:[^"\\]|\\.)*")|([^\s{}#"]+))')


def _scalar(tok: str):
    if tok.startswith('"'):
        return tok[1:-1]
    if tok in ("true", "false"):
        return tok == "true"
    try:
        return int(tok)
    except ValueError:
        pass
    try:
        return float(tok)
    except ValueError:
        return tok  # enum identifier (e.g. CAFFE, CENTER_SIZE, TEST)


def parse_prototxt(text: str) -> dict:
    """Protobuf text format -> nested dict; every field maps to a LIST of values."""
    toks = []
    pos = 0
    while pos < len(text):
        m = _TOK.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ValueError(f"prototxt: cannot tokenize near {text[pos:pos + 40]!r}")
        pos = m.end()
        comment, ident, colon, lb, rb, string, other = m.groups()
        if comment:
            continue
        if ident is not None:
            toks.append(("id", ident, bool(colon)))
        elif lb:
            toks.append(("{",))
        elif rb:
            toks.append(("}",))
        elif string is not None:
            toks.append(("val", string))
        elif other is not None:
            toks.append(("val", other))

    def parse_block(i):
        d: dict = {}
        while i < len(toks):
            t = toks[i]
            if t[0] == "}":
                return d, i + 1
            if t[0] != "id":
                raise ValueError(f"prototxt: unexpected token {t}")
            key = t[1]
            nxt = toks[i + 1] if i + 1 < len(toks) else None
            if nxt is not None and nxt[0] == "{":
                sub, i = parse_block(i + 2)
                d.setdefault(key, []).append(sub)
            elif nxt is not None and nxt[0] in ("val", "id") and t[2]:
                d.setdefault(key, []).append(_scalar(nxt[1]))
                i += 2
            else:
                raise ValueError(f"prototxt: field {key!r} without value")
        return d, i

    d, _ = parse_block(0)
    return d


def first(d: dict, key, default=None):
    v = d.get(key)
    return v[0] if v else default


@dataclass
class Layer:
    name: str
    type: str
    bottoms: list
    tops: list
    params: dict = field(default_factory=dict)

    def p(self, section, key, default=None):
        sec = first(self.params, section, {})
        return first(sec, key, default)

    def sub(self, section, subsection, key, default=None):
        sec = first(first(self.params, section, {}), subsection, {})
        return first(sec, key, default)

    def plist(self, section, key):
        sec = first(self.params, section, {})
        return list(sec.get(key, []))


@dataclass
class NetDef:
    name: str
    inputs: list
    input_shapes: list
    layers: list

    def layer(self, name) -> Layer:
        for l in self.layers:
            if l.name == name:
                return l
        raise KeyError(name)


def load_prototxt(path_or_text: str) -> NetDef:
    text = path_or_text
    if "\n" not in path_or_text and len(path_or_text) < 4096:
        with open(path_or_text) as f:
            text = f.read()
    d = parse_prototxt(text)
    shapes = [list(s.get("dim", [])) for s in d.get("input_shape", [])]
    if not shapes and "input_dim" in d:
        shapes = [list(d["input_dim"])]
    layers = []
    for ld in d.get("layer", []) + d.get("layers", []):
        params = {k: v for k, v in ld.items() if k not in ("name", "type", "bottom", "top")}
        layers.append(Layer(first(ld, "name"), first(ld, "type"), list(ld.get("bottom", [])),
                            list(ld.get("top", [])), params))
    return NetDef(first(d, "name", ""), list(d.get("input", [])), shapes, layers)


# ============================================================================ caffemodel wire format
def _varint(buf, i):
    r = s = 0
    while True:
        b = buf[i]
        i += 1
        r |= (b & 0x7F) << s
        if b < 0x80:
            return r, i
        s += 7


def _fields(buf):
    i = 0
    n = len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v = buf[i : i + 8]
            i += 8
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i : i + ln]
            i += ln
        elif wt == 5:
            v = buf[i : i + 4]
            i += 4
        else:
            raise ValueError(f"caffemodel: unsupported wire type {wt}")
        yield fno, wt, v


def _blob(buf) -> np.ndarray:
    shape, legacy, data = None, {}, []
    for fno, wt, v in _fields(buf):
        if fno == 7 and wt == 2:  # BlobShape
            dims = []
            for f2, w2, v2 in _fields(v):
                if f2 == 1:
                    if w2 == 2:
                        j = 0
                        while j < len(v2):
                            d, j = _varint(v2, j)
                            dims.append(d)
                    else:
                        dims.append(v2)
            shape = dims
        elif fno in (1, 2, 3, 4) and wt == 0:
            legacy[fno] = v
        elif fno == 5:
            if wt == 2:
                data.append(np.frombuffer(bytes(v), dtype="<f4"))
            elif wt == 5:
                data.append(np.frombuffer(bytes(v), dtype="<f4"))
    arr = np.concatenate(data) if data else np.zeros(0, np.float32)
    if shape is None and legacy:
        shape = [legacy.get(k, 1) for k in (1, 2, 3, 4)]
    if shape:
        arr = arr.reshape(shape)
    return arr.astype(np.float32)


def load_caffemodel(path) -> dict:
    """-> {layer_name: [blob0 (weights), blob1 (bias), ...]} as float32 ndarrays."""
    with open(path, "rb") as f:
        buf = memoryview(f.read())
    out = {}
    for fno, wt, v in _fields(buf):
        if fno in (100, 2) and wt == 2:  # layer (V2) / layers (V1)
            name, blobs = None, []
            name_field, blob_field = (1, 7) if fno == 100 else (4, 6)
            for f2, w2, v2 in _fields(v):
                if f2 == name_field and w2 == 2:
                    name = bytes(v2).decode()
                elif f2 == blob_field and w2 == 2:
                    blobs.append(_blob(v2))
            if name is not None and blobs:
                out[name] = blobs
    return out


def _enc_varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _enc_ld(fno, payload: bytes):
    return _enc_varint((fno << 3) | 2) + _enc_varint(len(payload)) + payload


def save_caffemodel(path, blobs: dict):
    """Write {layer_name: [ndarray, ...]} as a (V2) caffemodel NetParameter."""
    out = bytearray()
    for name, arrs in blobs.items():
        lp = bytearray(_enc_ld(1, name.encode()))
        for a in arrs:
            a = np.asarray(a, np.float32)
            shape = b"".join(_enc_varint((1 << 3) | 0) + _enc_varint(d) for d in a.shape)
            bp = _enc_ld(7, shape) + _enc_ld(5, a.astype("<f4").tobytes())
            lp += _enc_ld(7, bp)
        out += _enc_ld(100, bytes(lp))
    with open(path, "wb") as f:
        f.write(bytes(out))


# ============================================================================ SSD helpers
def prior_boxes(layer: Layer, fh: int, fw: int, img_h: int, img_w: int) -> np.ndarray:
    """Caffe-SSD PriorBox: returns [2, fh*fw*P*4] (boxes, variances), normalised coords."""
    min_sizes = [float(x) for x in layer.plist("prior_box_param", "min_size")]
    max_sizes = [float(x) for x in layer.plist("prior_box_param", "max_size")]
    ars = [1.0]
    flip = bool(layer.p("prior_box_param", "flip", True))
    for ar in layer.plist("prior_box_param", "aspect_ratio"):
        ar = float(ar)
        if any(abs(ar - a) < 1e-6 for a in ars):
            continue
        ars.append(ar)
        if flip:
            ars.append(1.0 / ar)
    clip = bool(layer.p("prior_box_param", "clip", False))
    var = [float(v) for v in layer.plist("prior_box_param", "variance")] or [0.1]
    if len(var) == 1:
        var = var * 4
    offset = float(layer.p("prior_box_param", "offset", 0.5))
    step_w = float(layer.p("prior_box_param", "step_w", layer.p("prior_box_param", "step", 0)) or img_w / fw)
    step_h = float(layer.p("prior_box_param", "step_h", layer.p("prior_box_param", "step", 0)) or img_h / fh)
    boxes = []
    for h in range(fh):
        for w in range(fw):
            cx, cy = (w + offset) * step_w, (h + offset) * step_h
            for si, s in enumerate(min_sizes):
                cand = [(s, s)]
                if max_sizes:
                    m = math.sqrt(s * max_sizes[si])
                    cand.append((m, m))
                for ar in ars:
                    if abs(ar - 1.0) < 1e-6:
                        continue
                    cand.append((s * math.sqrt(ar), s / math.sqrt(ar)))
                for bw, bh in cand:
                    boxes.append([(cx - bw / 2) / img_w, (cy - bh / 2) / img_h, (cx + bw / 2) / img_w,
                                  (cy + bh / 2) / img_h])
    b = np.asarray(boxes, np.float32).reshape(-1)
    if clip:
        b = np.clip(b, 0.0, 1.0)
    v = np.tile(np.asarray(var, np.float32), len(boxes))
    return np.stack([b, v])


def decode_boxes(loc: torch.Tensor, priors: torch.Tensor, var: torch.Tensor) -> torch.Tensor:
    """CENTER_SIZE decode. loc [..., P, 4], priors/var [P, 4] -> boxes [..., P, 4] (xmin,ymin,xmax,ymax)."""
    pw = priors[:, 2] - priors[:, 0]
    ph = priors[:, 3] - priors[:, 1]
    pcx = (priors[:, 0] + priors[:, 2]) * 0.5
    pcy = (priors[:, 1] + priors[:, 3]) * 0.5
    cx = var[:, 0] * loc[..., 0] * pw + pcx
    cy = var[:, 1] * loc[..., 1] * ph + pcy
    w = torch.exp(var[:, 2] * loc[..., 2]) * pw
    h = torch.exp(var[:, 3] * loc[..., 3]) * ph
    return torch.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], -1)


def jaccard(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """IoU of normalised boxes, a [N,4] x b [M,4] -> [N,M] (Caffe JaccardOverlap, no +1)."""
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp_min(0)
    inter = wh[..., 0] * wh[..., 1]
    area_a = ((a[:, 2] - a[:, 0]).clamp_min(0) * (a[:, 3] - a[:, 1]).clamp_min(0))[:, None]
    area_b = ((b[:, 2] - b[:, 0]).clamp_min(0) * (b[:, 3] - b[:, 1]).clamp_min(0))[None, :]
    union = area_a + area_b - inter
    return torch.where(union > 0, inter / union, torch.zeros_like(inter))


def nms_indices(boxes: torch.Tensor, scores: torch.Tensor, thresh: float, top_k: int) -> list:
    """Caffe ApplyNMSFast (eta=1): candidates sorted by score, greedy keep."""
    order = torch.argsort(scores, descending=True, stable=True)[:top_k]
    iou = jaccard(boxes[order], boxes[order]).cpu()
    keep = []
    for i in range(len(order)):
        if all(iou[i, j] <= thresh for j in keep):
            keep.append(i)
    return [int(order[i]) for i in keep]


def detection_output(loc, conf, priors, var, *, num_classes=21, background=0, conf_thresh=0.25,
                     nms_thresh=0.45, top_k=100, keep_top_k=100):
    """Reference DetectionOutput for a batch. loc [N, P*4], conf [N, P*C] (softmaxed),
    priors/var [P*4]. Returns list of [K, 7] float tensors (img, label, score, x0, y0, x1, y1)."""
    N = loc.shape[0]
    P = priors.numel() // 4
    pr = priors.view(P, 4).float()
    vr = var.view(P, 4).float()
    boxes = decode_boxes(loc.view(N, P, 4).float(), pr, vr)
    conf = conf.view(N, P, num_classes).float()
    out = []
    for n in range(N):
        dets = []
        for c in range(num_classes):
            if c == background:
                continue
            s = conf[n, :, c]
            idx = torch.nonzero(s > conf_thresh).flatten()
            if idx.numel() == 0:
                continue
            kept = nms_indices(boxes[n, idx], s[idx], nms_thresh, top_k)
            for k in kept:
                i = int(idx[k])
                dets.append([n, c, float(s[i])] + [float(v) for v in boxes[n, i]])
        if keep_top_k > 0 and len(dets) > keep_top_k:
            dets.sort(key=lambda d: -d[2])
            dets = dets[:keep_top_k]
        out.append(torch.tensor(dets, dtype=torch.float32).view(-1, 7))
    return out


# ============================================================================ reference interpreter
def msra_init(shape, fan_in, gen):
    std = math.sqrt(2.0 / max(1, fan_in))
    return torch.randn(shape, generator=gen) * std


class CaffeNet(torch.nn.Module):
    """Executes a NetDef with plain torch ops (fp32, NCHW). This is the ORACLE for the
    MI355X executor in ``mobilenet_ssd.py``; it is not the product inference path."""

    def __init__(self, net: NetDef, weights: dict | None = None, seed: int = 0):
        super().__init__()
        self.net = net
        self.blobs = torch.nn.ParameterDict()
        gen = torch.Generator().manual_seed(seed)
        shapes = {net.inputs[0]: list(net.input_shapes[0])} if net.inputs else {}
        for l in net.layers:
            if l.type == "Convolution":
                cin = shapes[l.bottoms[0]][1]
                cout = int(l.p("convolution_param", "num_output"))
                k = int(l.p("convolution_param", "kernel_size", 1))
                g = int(l.p("convolution_param", "group", 1))
                bias = bool(l.p("convolution_param", "bias_term", True))
                wshape = (cout, cin // g, k, k)
                key = l.name.replace("/", "__")
                if weights and l.name in weights:
                    w = torch.from_numpy(np.asarray(weights[l.name][0]).reshape(wshape).copy())
                    b = torch.from_numpy(np.asarray(weights[l.name][1]).reshape(cout).copy()) if bias else None
                else:
                    w = msra_init(wshape, (cin // g) * k * k, gen)
                    b = torch.zeros(cout) if bias else None
                self.blobs[key + "__w"] = torch.nn.Parameter(w, requires_grad=False)
                if b is not None:
                    self.blobs[key + "__b"] = torch.nn.Parameter(b, requires_grad=False)
            shapes.update(self._infer(l, shapes))

    def _infer(self, l: Layer, shapes):
        s = shapes[l.bottoms[0]] if l.bottoms else None
        if l.type == "Convolution":
            cout = int(l.p("convolution_param", "num_output"))
            k = int(l.p("convolution_param", "kernel_size", 1))
            st = int(l.p("convolution_param", "stride", 1))
            pd = int(l.p("convolution_param", "pad", 0))
            h = (s[2] + 2 * pd - k) // st + 1
            w = (s[3] + 2 * pd - k) // st + 1
            return {l.tops[0]: [s[0], cout, h, w]}
        return {l.tops[0]: s} if l.tops and s is not None else {}

    def conv_weights(self, name):
        key = name.replace("/", "__")
        return self.blobs[key + "__w"], self.blobs.get(key + "__b")

    def forward(self, data: torch.Tensor, stop_at: str | None = None) -> dict:
        t = {self.net.inputs[0]: data}
        img_h, img_w = data.shape[2], data.shape[3]
        for l in self.net.layers:
            x = t.get(l.bottoms[0]) if l.bottoms else None
            if l.type == "Convolution":
                w, b = self.conv_weights(l.name)
                y = F.conv2d(x, w, b, stride=int(l.p("convolution_param", "stride", 1)),
                             padding=int(l.p("convolution_param", "pad", 0)),
                             groups=int(l.p("convolution_param", "group", 1)))
            elif l.type == "ReLU":
                y = F.relu(x)
            elif l.type == "Permute":
                y = x.permute(*[int(o) for o in l.plist("permute_param", "order")])
            elif l.type == "Flatten":
                ax = int(l.p("flatten_param", "axis", 1))
                y = x.flatten(ax)
            elif l.type == "PriorBox":
                fh, fw = x.shape[2], x.shape[3]
                y = torch.from_numpy(prior_boxes(l, fh, fw, img_h, img_w)).unsqueeze(0)
            elif l.type == "Concat":
                ax = int(l.p("concat_param", "axis", 1))
                y = torch.cat([t[b] for b in l.bottoms], ax)
            elif l.type == "Reshape":
                dims = [int(d) for d in first(first(l.params, "reshape_param", {}), "shape", {}).get("dim", [])]
                dims = [x.shape[i] if d == 0 else d for i, d in enumerate(dims)]
                y = x.reshape(dims)
            elif l.type == "Softmax":
                y = torch.softmax(x, int(l.p("softmax_param", "axis", 1)))
            elif l.type == "DetectionOutput":
                loc, conf, pri = (t[b] for b in l.bottoms)
                y = detection_output(
                    loc, conf, pri[0, 0], pri[0, 1], num_classes=int(l.p("detection_output_param", "num_classes")),
                    background=int(l.p("detection_output_param", "background_label_id", 0)),
                    conf_thresh=float(l.p("detection_output_param", "confidence_threshold", 0.01)),
                    nms_thresh=float(l.sub("detection_output_param", "nms_param", "nms_threshold", 0.45)),
                    top_k=int(l.sub("detection_output_param", "nms_param", "top_k", -1)),
                    keep_top_k=int(l.p("detection_output_param", "keep_top_k", -1)))
            else:
                raise NotImplementedError(f"Caffe layer type {l.type!r}")
            for top in l.tops:
                t[top] = y
            if stop_at is not None and l.name == stop_at:
                break
        return t
