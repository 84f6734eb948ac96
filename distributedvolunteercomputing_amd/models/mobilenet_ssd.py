"""MobileNet-SSD person detector — the reference's only model (MobileNetSSD_deploy.prototxt,
run by OpenCV DNN on CPU at /root/reference/worker.py:194,245-249).

``SSDExecutor`` compiles the Caffe ``NetDef`` into a plan of MI355X kernels over NHWC bf16
activations for a whole chunk of frames at once:

  Convolution group=C (depthwise 3x3)  -> fused into the following pointwise GEMM (dw_pw: the
                                          depthwise tile is computed while staging the A operand),
                                          or the dwconv3x3 kernel (+bias +ReLU) for wide blocks
  Convolution 1x1                      -> MFMA GEMM  [N*H*W, Cin] x [Cout, Cin]^T (+bias +ReLU)
  Convolution kxk (stem, SSD extras)   -> the same MFMA GEMM as an implicit GEMM (the A tile is
                                          gathered from the NHWC input while staging: no im2col)
  ReLU after a convolution             -> fused into the producer's epilogue
  multibox heads (loc, conf 1x1 convs)
  + Permute(0,2,3,1) + Flatten + Concat -> ONE GEMM per source (loc||conf weights) whose epilogue
                                          writes both straight into the mbox_loc / mbox_conf
                                          concat buffers at the source's offsets
  PriorBox                             -> computed once on the host, cached on the device
  Reshape + Softmax + DetectionOutput  -> one fused softmax/decode/top-k/NMS kernel pair

On CPU the same object runs the plain-PyTorch ``CaffeNet`` interpreter (the oracle).
"""
from __future__ import annotations

import contextlib
import os

import torch

from .. import ops
from ..ops import vision as V
from .caffe import CaffeNet, Layer, NetDef, load_caffemodel, load_prototxt, prior_boxes

CLASSES = ["background", "aeroplane", "bicycle", "bird", "boat", "bottle", "bus", "car", "cat", "chair", "cow",
           "diningtable", "dog", "horse", "motorbike", "person", "pottedplant", "sheep", "sofa", "train",
           "tvmonitor"]

def _conv(name, bottom, cout, k=1, stride=1, pad=0, group=1):
    cp = {"num_output": [cout], "kernel_size": [k]}
    if pad:
        cp["pad"] = [pad]
    if stride != 1:
        cp["stride"] = [stride]
    if group != 1:
        cp["group"] = [group]
    return Layer(name, "Convolution", [bottom], [name], {"convolution_param": [cp]})


def mobilenet_ssd_netdef(num_classes: int = 21, size: int = 300) -> NetDef:
    """The MobileNet-SSD graph of MobileNetSSD_deploy.prototxt (119 layers), built in code:
    MobileNet-v1 backbone (conv0 + 13 dw/pw pairs), 4 SSD extra stages, 6 multibox heads."""
    L = []

    def relu(top):
        L.append(Layer(top + "/relu", "ReLU", [top], [top]))

    L.append(_conv("conv0", "data", 32, 3, 2, 1))
    relu("conv0")
    chans = [(32, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2), (256, 256, 1), (256, 512, 2)] + \
        [(512, 512, 1)] * 5 + [(512, 1024, 2), (1024, 1024, 1)]
    prev = "conv0"
    for i, (cin, cout, s) in enumerate(chans, start=1):
        L.append(_conv(f"conv{i}/dw", prev, cin, 3, s, 1, group=cin))
        relu(f"conv{i}/dw")
        L.append(_conv(f"conv{i}", f"conv{i}/dw", cout))
        relu(f"conv{i}")
        prev = f"conv{i}"
    for i, (mid, out) in zip(range(14, 18), [(256, 512), (128, 256), (128, 256), (64, 128)]):
        L.append(_conv(f"conv{i}_1", prev, mid))
        relu(f"conv{i}_1")
        L.append(_conv(f"conv{i}_2", f"conv{i}_1", out, 3, 2, 1))
        relu(f"conv{i}_2")
        prev = f"conv{i}_2"
    sources = ["conv11", "conv13", "conv14_2", "conv15_2", "conv16_2", "conv17_2"]
    mins = [60.0, 105.0, 150.0, 195.0, 240.0, 285.0]
    maxs = [None, 150.0, 195.0, 240.0, 285.0, 300.0]
    for src, mn, mx in zip(sources, mins, maxs):
        npri = 3 if mx is None else 6
        for kind, c in (("loc", 4 * npri), ("conf", num_classes * npri)):
            nm = f"{src}_mbox_{kind}"
            L.append(_conv(nm, src, c))
            L.append(Layer(nm + "_perm", "Permute", [nm], [nm + "_perm"], {"permute_param": [{"order": [0, 2, 3, 1]}]}))
            L.append(Layer(nm + "_flat", "Flatten", [nm + "_perm"], [nm + "_flat"], {"flatten_param": [{"axis": [1]}]}))
        pp = {"min_size": [mn], "aspect_ratio": [2.0] if mx is None else [2.0, 3.0], "flip": [True], "clip": [False],
              "variance": [0.1, 0.1, 0.2, 0.2], "offset": [0.5]}
        if mx is not None:
            pp["max_size"] = [mx]
        L.append(Layer(f"{src}_mbox_priorbox", "PriorBox", [src, "data"], [f"{src}_mbox_priorbox"],
                       {"prior_box_param": [pp]}))
    for kind, ax in (("loc", 1), ("conf", 1), ("priorbox", 2)):
        sfx = "_flat" if kind != "priorbox" else ""
        L.append(Layer(f"mbox_{kind}", "Concat", [f"{s}_mbox_{kind}{sfx}" for s in sources], [f"mbox_{kind}"],
                       {"concat_param": [{"axis": [ax]}]}))
    L.append(Layer("mbox_conf_reshape", "Reshape", ["mbox_conf"], ["mbox_conf_reshape"],
                   {"reshape_param": [{"shape": [{"dim": [0, -1, num_classes]}]}]}))
    L.append(Layer("mbox_conf_softmax", "Softmax", ["mbox_conf_reshape"], ["mbox_conf_softmax"],
                   {"softmax_param": [{"axis": [2]}]}))
    L.append(Layer("mbox_conf_flatten", "Flatten", ["mbox_conf_softmax"], ["mbox_conf_flatten"],
                   {"flatten_param": [{"axis": [1]}]}))
    L.append(Layer("detection_out", "DetectionOutput", ["mbox_loc", "mbox_conf_flatten", "mbox_priorbox"],
                   ["detection_out"], {"detection_output_param": [{
                       "num_classes": [num_classes], "share_location": [True], "background_label_id": [0],
                       "nms_param": [{"nms_threshold": [0.45], "top_k": [100]}], "code_type": ["CENTER_SIZE"],
                       "keep_top_k": [100], "confidence_threshold": [0.25]}]}))
    return NetDef("MobileNet-SSD", ["data"], [[1, 3, size, size]], L)


_GRAPH_GRAVEYARD = []


def _nullctx():
    return contextlib.nullcontext()


def _round_up(n, a):
    return (n + a - 1) // a * a


class SSDExecutor:
    def __init__(self, net: NetDef | str | None = None, caffemodel: str | None = None, device="cpu", seed: int = 0):
        if net is None:
            net = mobilenet_ssd_netdef()
        elif isinstance(net, (str, os.PathLike)):
            net = load_prototxt(str(net))
        self.net = net
        weights = load_caffemodel(caffemodel) if caffemodel and os.path.exists(caffemodel) else None
        self.ref = CaffeNet(net, weights, seed=seed)
        self.device = torch.device(device)
        self.input_size = int(net.input_shapes[0][2]) if net.input_shapes else 300
        self._prior_cache = {}
        self.step_events = None
        # one HIP graph per chunk shape is opt-in: measured no faster than eager launching (1.39 vs
        # 1.31-1.33 ms per 100-frame chunk: the GPU, not the host, is the bound), and a capture
        # inside the multi-threaded volunteer job was invalidated by the other threads' GPU calls
        self.use_graph = os.environ.get("VCX_VISION_GRAPH", "0") == "1"
        # nt: gemm_nt (256 x 256 tiles) where it applies | vision: the 128 x 128-tile vision GEMM (1.197 vs
        # 1.171 ms per chunk; gemm_nt only where its last tile wave is short: 1.177, profiles/r4_detector_chunk.txt)
        self.pw_gemm = os.environ.get("VCX_VISION_PW", "nt")
        self._graphs = {}
        self._sides = {}
        self.graph_error = None
        self._plan = self._compile() if self.device.type == "cuda" else None

    # ------------------------------------------------------------------ compile
    def _find_heads(self):
        """Multibox heads: 1x1 convolutions whose output goes only through Permute(0,2,3,1) ->
        Flatten into the mbox_loc / mbox_conf Concat (prototxt 1147-1858). Returns
        {conv index: (concat layer index, position in the concat)} and the layer indices the
        fused head GEMMs make redundant (the Permute and Flatten layers)."""
        layers = self.net.layers
        producer = {}
        for i, l in enumerate(layers):
            for t in l.tops:
                producer[t] = i
        heads, skip = {}, set()
        for ci, l in enumerate(layers):
            if l.type != "Concat" or int(l.p("concat_param", "axis", 1)) != 1:
                continue
            chain = []
            for pos, b in enumerate(l.bottoms):
                fi = producer.get(b)
                if fi is None or layers[fi].type != "Flatten":
                    break
                pi = producer.get(layers[fi].bottoms[0])
                if pi is None or layers[pi].type != "Permute":
                    break
                cv = producer.get(layers[pi].bottoms[0])
                if cv is None or layers[cv].type != "Convolution":
                    break
                chain.append((cv, pos, fi, pi))
            else:
                for cv, pos, fi, pi in chain:
                    heads[cv] = (ci, pos)
                    skip.update((fi, pi))
        return heads, skip

    def _compile(self):
        dev = self.device
        plan = []
        layers = self.net.layers
        heads, consumed = self._find_heads()
        consumed = set(consumed)
        shapes = {self.net.inputs[0]: 3}  # channels per blob
        hw = {self.net.inputs[0]: (self.input_size, self.input_size)}  # static spatial sizes
        head_steps = {}  # source blob -> merged head step
        concat_cols = {}  # concat index -> [(position, rows per image, cols)]
        for i, l in enumerate(layers):
            if l.type == "Convolution" and l.bottoms[0] in hw:
                k = int(l.p("convolution_param", "kernel_size", 1))
                st = int(l.p("convolution_param", "stride", 1))
                pd = int(l.p("convolution_param", "pad", 0))
                H, W = hw[l.bottoms[0]]
                hw[l.tops[0]] = ((H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1)
            elif l.bottoms and l.bottoms[0] in hw and l.tops and l.tops[0] not in hw:
                hw[l.tops[0]] = hw[l.bottoms[0]]
        for i, l in enumerate(layers):
            if i in consumed:
                continue
            if l.type == "Convolution" and i in heads:
                # loc || conf of one source: ONE GEMM writing both concat buffers in place
                w, b = self.ref.conv_weights(l.name)
                ci, pos = heads[i]
                src = l.bottoms[0]
                H, W = hw[src]
                cout = w.shape[0]
                concat_cols.setdefault(ci, []).append((pos, H * W, cout))
                hs = head_steps.get(src)
                bias = (b.detach().float() if b is not None else torch.zeros(cout))
                wt = w.detach().float().reshape(cout, -1)
                if hs is None:
                    hs = head_steps[src] = dict(parts=[], src=src)
                    plan.append(("head", l, hs))
                hs["parts"].append(dict(concat=ci, pos=pos, w=wt, b=bias, cout=cout, rows=H * W))
                continue
            if l.type == "Convolution":
                w, b = self.ref.conv_weights(l.name)
                cout, cin_g, k, _ = w.shape
                group = int(l.p("convolution_param", "group", 1))
                stride = int(l.p("convolution_param", "stride", 1))
                pad = int(l.p("convolution_param", "pad", 0))
                relu = False
                if i + 1 < len(layers) and layers[i + 1].type == "ReLU" and layers[i + 1].bottoms[0] == l.tops[0]:
                    relu = True
                    consumed.add(i + 1)
                bias = (b.detach().float() if b is not None else torch.zeros(cout)).to(dev)
                cin = cin_g * group
                if group > 1:
                    if not (group == cin == cout and k == 3 and pad == 1):
                        raise NotImplementedError(f"{l.name}: only depthwise 3x3 pad 1 grouped conv is supported")
                    w9 = w.detach().float().permute(2, 3, 0, 1).reshape(9, cout).contiguous()
                    plan.append(("dw", l, dict(w=V.dw_pair_weights(w9.to(dev, torch.bfloat16)), b=bias,
                                               stride=stride, relu=relu)))
                elif k == 1 and stride == 1 and pad == 0 and cin % 32 == 0:
                    wt = w.detach().float().reshape(cout, cin).to(dev, torch.bfloat16).contiguous()
                    plan.append(("pw", l, dict(w=wt, b=bias, b16=bias.to(torch.bfloat16), relu=relu)))
                else:
                    # implicit GEMM: columns (ky, kx, c); the 3-channel stem reads the 4-channel
                    # padded blob (c = 3 has zero weights) as two taps per 16-B load
                    C = 4 if cin == 3 else cin
                    K = k * k * C
                    Kp = _round_up(K, 32)
                    wk = torch.zeros(cout, k, k, C)
                    wk[..., :cin] = w.detach().float().permute(0, 2, 3, 1)
                    wt = torch.zeros(cout, Kp)
                    wt[:, :K] = wk.reshape(cout, K)
                    plan.append(("conv", l, dict(w=wt.to(dev, torch.bfloat16).contiguous(), b=bias, k=k,
                                                 stride=stride, pad=pad, cin=cin, C=C, Kp=Kp, relu=relu)))
                shapes[l.tops[0]] = cout
            elif l.type == "ReLU":
                plan.append(("relu", l, {}))
            elif l.type == "Permute":
                order = [int(o) for o in l.plist("permute_param", "order")]
                if order != [0, 2, 3, 1]:
                    raise NotImplementedError(f"{l.name}: permute {order}")
                plan.append(("nhwc", l, {}))
            elif l.type == "Concat" and i in concat_cols:
                plan.append(("concat_buf", l, {"index": i}))
            elif l.type == "DetectionOutput":
                # parameters parsed once here, not on every chunk between the last head and the detect launch
                dp = lambda k, d: l.p("detection_output_param", k, d)  # noqa: E731
                nms = lambda k, d: l.sub("detection_output_param", "nms_param", k, d)  # noqa: E731
                plan.append(("detectionoutput", l, dict(
                    nc=int(dp("num_classes", 21)), bg=int(dp("background_label_id", 0)),
                    conf=float(dp("confidence_threshold", 0.01)), nms=float(nms("nms_threshold", 0.45)),
                    top_k=int(nms("top_k", 100)), keep=int(dp("keep_top_k", 100)))))
            elif l.type in ("Flatten", "Concat", "PriorBox", "Reshape", "Softmax"):
                plan.append((l.type.lower(), l, {}))
            else:
                raise NotImplementedError(f"Caffe layer type {l.type!r} ({l.name})")
        # concat offsets (per image, in elements) and merged loc||conf weights per source
        self._concat_total, offs = {}, {}
        for ci, cols in concat_cols.items():
            o = 0
            for pos, rows, cout in sorted(cols):
                offs[(ci, pos)] = o
                o += rows * cout
            self._concat_total[ci] = o
        for hs in head_steps.values():
            parts = hs["parts"]
            if len(parts) != 2:
                raise NotImplementedError(f"{hs['src']}: expected one loc and one conf head")
            a, c = parts
            K = a["w"].shape[1]
            if K % 32:
                raise NotImplementedError(f"{hs['src']}: head GEMM needs K % 32 == 0")
            hs["w"] = torch.cat([a["w"], c["w"]]).to(dev, torch.bfloat16).contiguous()
            hs["b"] = torch.cat([a["b"], c["b"]]).to(dev)
            hs["split"] = a["cout"]
            hs["concats"] = (a["concat"], c["concat"])
            hs["offs"] = (offs[(a["concat"], a["pos"])], offs[(c["concat"], c["pos"])])
            hs["rows"] = a["rows"]
        return self._heads_after_sources(self._fuse_dw_pw(plan))

    @staticmethod
    def _heads_after_sources(plan):
        """Move each multibox head step right behind the step that produces its source (the
        prototxt lists every head after the last extra layer): the head then forks onto the side
        stream as soon as its input exists and overlaps the rest of the backbone / extras,
        instead of waiting behind all of them."""
        heads = [st for st in plan if st[0] == "head"]
        rest = [st for st in plan if st[0] != "head"]
        out = []
        for st in rest:
            out.append(st)
            top = st[1].tops[0] if st[1].tops else None
            for h in heads:
                if h[2]["src"] == top:
                    out.append(h)
        placed = sum(1 for st in out if st[0] == "head")
        if placed != len(heads):  # a source produced outside the plan's steps: keep the original order
            return plan
        return out

    def _fuse_dw_pw(self, plan):
        """Depthwise -> pointwise pairs (every MobileNet block, prototxt 42-106 and after) become one
        `dwpw` step when the depthwise output feeds only that pointwise conv and the block shape
        has a 2-D-tile fused kernel (ops.vision.DWPW_TILE: conv1..conv3, the 150^2 / 75^2 blocks
        where the depthwise round trip through HBM costs most; tile1 = conv1 only). VCX_DWPW=off keeps every block two
        kernels; VCX_DWPW=all also fuses the others through the GEMM's A-staging path (slower)."""
        mode = os.environ.get("VCX_DWPW", "tile")
        if mode == "off":
            return plan
        uses = {}
        for l in self.net.layers:
            if l.tops == l.bottoms:
                continue  # in-place (the ReLUs folded into their producer)
            for b in l.bottoms:
                uses[b] = uses.get(b, 0) + 1
        out, i = [], 0
        while i < len(plan):
            kind, l, p = plan[i]
            if kind == "dw" and i + 1 < len(plan):
                k2, l2, p2 = plan[i + 1]
                K, Co = p["w"].shape[1], (p2["w"].shape[0] if k2 == "pw" else 0)
                tiles = (V.DWPW_TILE_ALL if mode in ("tile3", "all") else {(32, 64, 1)} if mode == "tile1"
                         else V.DWPW_TILE)
                shape_ok = (K, Co, p["stride"]) in tiles or (mode == "all" and K <= 1024 and K % 32 == 0)
                if k2 == "pw" and l2.bottoms[0] == l.tops[0] and uses.get(l.tops[0], 0) == 1 and shape_ok:
                    out.append(("dwpw", l2, dict(dw=p, pw=p2, src=l.bottoms[0])))
                    i += 2
                    continue
            out.append(plan[i])
            i += 1
        return self._fuse_block_pairs(out, uses) if mode != "tile1" and os.environ.get("VCX_DWPW2", "1") != "0" else out

    @staticmethod
    def _fuse_block_pairs(plan, uses):
        """conv1 -> conv2 (a stride-1 block 32 -> 64 followed by a stride-2 block 64 -> 128, the 150^2 ->
        75^2 step of MobileNet, prototxt 42-106) as ONE `dwpw2` step whose kernel keeps conv1's output
        in LDS (ops.vision.dw_pw2); VCX_DWPW2=0 keeps two steps."""
        out, i = [], 0
        while i < len(plan):
            st = plan[i]
            if st[0] == "dwpw" and i + 1 < len(plan) and plan[i + 1][0] == "dwpw":
                a, b = st[2], plan[i + 1][2]
                shapes = (a["dw"]["w"].shape[1], a["pw"]["w"].shape[0], a["dw"]["stride"],
                          b["dw"]["w"].shape[1], b["pw"]["w"].shape[0], b["dw"]["stride"])
                if (shapes == (32, 64, 1, 64, 128, 2) and b["src"] == st[1].tops[0]
                        and uses.get(st[1].tops[0], 0) == 1):
                    out.append(("dwpw2", plan[i + 1][1], dict(b1=a, b2=b, src=a["src"])))
                    i += 2
                    continue
            out.append(st)
            i += 1
        return out

    # ------------------------------------------------------------------ helpers
    def _priors(self, layer, fh, fw):
        key = (layer.name, fh, fw)
        if key not in self._prior_cache:
            pb = prior_boxes(layer, fh, fw, self.input_size, self.input_size)
            self._prior_cache[key] = torch.from_numpy(pb).unsqueeze(0).to(self.device)  # [1, 2, P*4]
        return self._prior_cache[key]

    # ------------------------------------------------------------------ run
    @torch.no_grad()
    def forward_blob(self, blob: torch.Tensor) -> dict:
        """blob: NHWC bf16 [N, S, S, 4] (from ops.vision.blob_from_frames). Returns named tensors;
        'detection_out' -> (dets [N, keep, 7], counts [N])."""
        if self._plan is None:
            x = blob[..., :3].permute(0, 3, 1, 2).float()
            t = self.ref(x)
            d = t["detection_out"]
            keep = 100
            out = torch.zeros(len(d), keep, 7)
            cnt = torch.zeros(len(d), dtype=torch.int32)
            for n, dd in enumerate(d):
                kk = min(len(dd), keep)
                out[n, :kk] = dd[:kk]
                cnt[n] = kk
            t["detection_out"] = (out, cnt)
            return t
        N = blob.shape[0]
        t = {self.net.inputs[0]: blob}
        layout = {self.net.inputs[0]: "nhwc"}
        hw = {self.net.inputs[0]: (blob.shape[1], blob.shape[2])}
        chans = {self.net.inputs[0]: 3}
        assert blob.shape[1] == self.input_size, "the plan's head offsets are for the prototxt input size"
        concat_bufs = {ci: torch.empty(N, tot, device=blob.device, dtype=torch.bfloat16)
                       for ci, tot in self._concat_total.items()}
        marks = self.step_events  # optional per-step timing: list of (layer name, kind, event)
        # the multibox heads (small GEMMs, split-K) run on a side stream, concurrently with the
        # backbone / extras layers after their source; joined before DetectionOutput. Inside the
        # chunk's HIP graph this becomes parallel branches. (Per-step timing keeps one stream.)
        main = torch.cuda.current_stream(blob.device)
        side = self._side_stream(blob.device) if marks is None else None
        side_refs, forked = [], False
        for kind, l, p in self._plan:
            if marks is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                marks.append((l.name, kind, ev))
            src = l.bottoms[0] if l.bottoms else None
            x = t.get(src)
            top = l.tops[0] if l.tops else None
            if kind == "dw":
                y = V.dwconv3x3(x, p["w"], p["b"], p["stride"], p["relu"])
                t[top], layout[top], hw[top], chans[top] = y, "nhwc", (y.shape[1], y.shape[2]), y.shape[3]
            elif kind == "dwpw":
                d, q = p["dw"], p["pw"]
                y = V.dw_pw(t[p["src"]], d["w"], d["b"], d["relu"], d["stride"], q["w"], q["b"], q["relu"])
                t[top], layout[top], hw[top], chans[top] = y, "nhwc", (y.shape[1], y.shape[2]), y.shape[3]
            elif kind == "dwpw2":
                blk = [dict(dw_w=p[k]["dw"]["w"], dw_b=p[k]["dw"]["b"], dw_relu=p[k]["dw"]["relu"], w=p[k]["pw"]["w"],
                            b=p[k]["pw"]["b"], relu=p[k]["pw"]["relu"]) for k in ("b1", "b2")]
                y = V.dw_pw2(t[p["src"]], blk[0], blk[1])
                t[top], layout[top], hw[top], chans[top] = y, "nhwc", (y.shape[1], y.shape[2]), y.shape[3]
            elif kind == "pw":
                H, W = hw[src]
                M = N * H * W
                K, Co = x.shape[-1], p["w"].shape[0]
                epi = 4 if p["relu"] else 1
                if self.pw_gemm == "nt" and ops.native().gemm_nt_supported_epi(M, Co, K, epi):
                    # the wide pointwise layers (K, Cout >= 256) on the training GEMM: 256 x 256
                    # tiles, LDS-DMA ring, bias(+ReLU) epilogue, ragged M
                    y = torch.empty(M, Co, device=x.device, dtype=torch.bfloat16)
                    ops.native().gemm_nt(x.reshape(M, K), p["w"], y, None, p["b16"], None, epi)
                else:
                    y = V.gemm_bias_act(x.reshape(M, K), p["w"], p["b"], p["relu"])
                t[top], layout[top], hw[top], chans[top] = y.view(N, H, W, -1), "nhwc", (H, W), y.shape[1]
            elif kind == "head":
                x = t[p["src"]]
                H, W = hw[p["src"]]
                la, ca = (concat_bufs[c] for c in p["concats"])
                if side is not None:
                    side.wait_stream(main)  # the source activation is ready
                    side_refs.append(x)  # kept alive (not reused by the allocator) until the join
                    forked = True
                with torch.cuda.stream(side) if side is not None else _nullctx():
                    ops.native().gemm_bias_heads(x.reshape(N * H * W, x.shape[-1]), p["w"], p["b"], la,
                                                 p["offs"][0], ca, p["offs"][1], p["split"], H * W)
            elif kind == "concat_buf":
                t[top], layout[top] = concat_bufs[p["index"]], "plain"
            elif kind == "conv":
                k, s, pd = p["k"], p["stride"], p["pad"]
                y = ops.native().conv_implicit(x.contiguous(), p["w"], p["b"], p["C"], k, k, s, pd, p["relu"])
                t[top], layout[top], hw[top], chans[top] = y, "nhwc", (y.shape[1], y.shape[2]), y.shape[3]
            elif kind == "relu":
                t[top] = torch.relu(x)
                layout[top], hw[top], chans[top] = layout[src], hw.get(src), chans.get(src)
            elif kind == "nhwc":  # Permute(0,2,3,1) of a logical NCHW tensor stored NHWC: free
                t[top], layout[top] = x, "plain"
            elif kind == "flatten":
                t[top], layout[top] = x.reshape(N, -1) if x.dim() > 2 or layout[src] != "priors" else x, (
                    "priors" if layout.get(src) == "priors" else "plain")
            elif kind == "priorbox":
                fh, fw = hw[src]
                t[top], layout[top] = self._priors(l, fh, fw), "priors"
            elif kind == "concat":
                ax = int(l.p("concat_param", "axis", 1))
                parts = [t[b] for b in l.bottoms]
                if layout[l.bottoms[0]] == "priors":  # constant for a given input size: concatenated once
                    key = ("cat", l.name, blob.device.index)
                    if key not in self._prior_cache:
                        cat = torch.cat(parts, ax)
                        self._prior_cache[key] = (cat, cat[0, 0].float().contiguous(), cat[0, 1].float().contiguous())
                    t[top], layout[top] = self._prior_cache[key][0], "priors"
                else:
                    t[top], layout[top] = torch.cat([q.reshape(N, -1) for q in parts], ax), "plain"
            elif kind in ("reshape", "softmax"):
                # folded into DetectionOutput: the detect kernel takes raw logits
                t[top], layout[top] = x, "logits"
            elif kind == "detectionoutput":
                if forked:
                    main.wait_stream(side)  # every head has written the concat buffers
                    forked = False
                loc, conf, pri = (t[b] for b in l.bottoms)
                P = pri.shape[-1] // 4
                nc = p["nc"]
                cached = next((v for k, v in self._prior_cache.items() if k[0] == "cat" and v[0] is pri), None)
                boxes, var = (cached[1], cached[2]) if cached is not None else (pri[0, 0], pri[0, 1])
                dets, cnt = V.ssd_detect(conf.reshape(N, P * nc), loc.reshape(N, P * 4), boxes, var,
                                         num_classes=nc, background=p["bg"], conf_thresh=p["conf"],
                                         nms_thresh=p["nms"], top_k=p["top_k"], keep_top_k=p["keep"])
                t[top] = (dets, cnt)
        if forked:
            main.wait_stream(side)
        side_refs.clear()
        if marks is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            marks.append(("<end>", "", ev))
        return t

    def _side_stream(self, dev):
        if os.environ.get("VCX_VISION_STREAMS", "2") == "1":
            return None
        s = self._sides.get(dev)
        if s is None:
            s = self._sides[dev] = torch.cuda.Stream(dev)
        return s

    def step_times(self, blob: torch.Tensor, iters: int = 10) -> list:
        """Per plan step GPU time (ms, mean over `iters` passes): [(layer, kind, ms)]. Steps that
        launch nothing (relu folded, concat views, priors cached) show ~0."""
        self.forward_blob(blob)
        acc = None
        for _ in range(iters):
            self.step_events = []
            self.forward_blob(blob)
            torch.cuda.synchronize()
            ev = self.step_events
            ms = [(a[0], a[1], a[2].elapsed_time(b[2])) for a, b in zip(ev, ev[1:])]
            acc = ms if acc is None else [(n, k, s + m[2]) for (n, k, s), m in zip(acc, ms)]
        self.step_events = None
        return [(n, k, s / iters) for n, k, s in acc]

    def detect(self, frames_u8: torch.Tensor):
        """frames [N, H, W, 3] uint8 BGR (already at the annotation size) -> (dets, counts).
        With VCX_VISION_GRAPH=1 the whole chunk (blob + the plan's kernels + detection) replays
        as one HIP graph per input shape (measured no faster than eager: the GPU is the bound).
        """
        if self._plan is not None and self.use_graph and frames_u8.is_cuda:
            return self._detect_graphed(frames_u8)
        blob = V.blob_from_frames(frames_u8, self.input_size)
        return self.forward_blob(blob)["detection_out"]

    def _detect_eager(self, frames_u8):
        return self.forward_blob(V.blob_from_frames(frames_u8, self.input_size))["detection_out"]

    def _detect_graphed(self, frames_u8):
        key = (tuple(frames_u8.shape), frames_u8.device.index)
        g = self._graphs.get(key)
        if g is None:
            static_in = frames_u8.clone()
            side = torch.cuda.Stream(frames_u8.device)
            side.wait_stream(torch.cuda.current_stream(frames_u8.device))
            with torch.cuda.stream(side):  # warm-up: priors cached, allocator primed
                for _ in range(2):
                    self._detect_eager(static_in)
            torch.cuda.current_stream(frames_u8.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            try:
                # thread_local: volunteers' other threads (pre-resize, transfers) keep using the
                # GPU while a worker captures; only this thread's calls belong to the capture
                with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                    static_out = self._detect_eager(static_in)
            except RuntimeError as e:  # capture invalidated: run this executor eagerly from now on
                _GRAPH_GRAVEYARD.append(graph)  # a failed capture's destructor throws: never run it
                self.use_graph = False
                self.graph_error = f"{type(e).__name__}: {str(e)[:200]}"
                return self._detect_eager(frames_u8)
            g = self._graphs[key] = (graph, static_in, static_out)
        graph, static_in, (dets, cnt) = g
        static_in.copy_(frames_u8)
        graph.replay()
        # the next replay overwrites the graph's buffers: hand out copies (280 KB per 100 frames)
        return dets.clone(), cnt.clone()


def smoke_detect(dev):
    """Tiny end-to-end detection on the GPU (used by __graft_entry__.smoke)."""
    ex = SSDExecutor(device=dev)
    frames = torch.randint(0, 255, (2, 225, 400, 3), dtype=torch.uint8, device=dev)
    dets, cnt = ex.detect(frames)
    V.annotate(frames, dets, cnt, "127.0.0.1:5554")
    torch.cuda.synchronize()
    print(f"[smoke] mobilenet-ssd detect ok, dets/frame={cnt.tolist()}")
