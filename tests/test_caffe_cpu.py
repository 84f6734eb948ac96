"""Caffe prototxt/caffemodel handling and the MobileNet-SSD graph, on CPU."""
import os

import numpy as np
import pytest
import torch

from distributedvolunteercomputing_amd.models import caffe
from distributedvolunteercomputing_amd.models.mobilenet_ssd import SSDExecutor, mobilenet_ssd_netdef

REF_PROTOTXT = "/root/reference/MobileNetSSD_deploy.prototxt.txt"


def test_builtin_graph_census():
    net = mobilenet_ssd_netdef()
    from collections import Counter

    c = Counter(l.type for l in net.layers)
    assert len(net.layers) == 119
    assert c == {"Convolution": 47, "ReLU": 35, "Permute": 12, "Flatten": 13, "PriorBox": 6, "Concat": 3,
                 "Reshape": 1, "Softmax": 1, "DetectionOutput": 1}
    m = caffe.CaffeNet(net)
    assert sum(p.numel() for p in m.parameters()) == 5_783_417


@pytest.mark.skipif(not os.path.exists(REF_PROTOTXT), reason="reference prototxt not mounted")
def test_builtin_graph_equals_reference_prototxt():
    a = caffe.load_prototxt(REF_PROTOTXT)
    b = mobilenet_ssd_netdef()
    assert [(l.name, l.type, l.bottoms, l.tops) for l in a.layers] == [(l.name, l.type, l.bottoms, l.tops)
                                                                       for l in b.layers]
    for la, lb in zip(a.layers, b.layers):
        for sec, vals in lb.params.items():
            for k, v in vals[0].items():
                if not isinstance(v[0], dict):
                    assert la.params[sec][0][k] == v, (la.name, sec, k)


def test_prototxt_parser_features():
    d = caffe.parse_prototxt('name: "x" # comment\nlayer { name: "a" type: "Conv" p { v: 1.5 v: -2 e: CAFFE b: true } }')
    assert d["name"] == ["x"]
    p = d["layer"][0]["p"][0]
    assert p["v"] == [1.5, -2] and p["e"] == ["CAFFE"] and p["b"] == [True]


def test_priors_count_and_values():
    net = mobilenet_ssd_netdef()
    total = 0
    for l, fm in zip([l for l in net.layers if l.type == "PriorBox"], [19, 10, 5, 3, 2, 1]):
        pb = caffe.prior_boxes(l, fm, fm, 300, 300)
        total += pb.shape[1] // 4
    assert total == 1917
    l0 = net.layer("conv11_mbox_priorbox")
    pb = caffe.prior_boxes(l0, 19, 19, 300, 300)
    step = 300 / 19
    c = 0.5 * step / 300
    s = 60 / 300 / 2
    assert np.allclose(pb[0, :4], [c - s, c - s, c + s, c + s], atol=1e-6)
    assert np.allclose(pb[1, :4], [0.1, 0.1, 0.2, 0.2])


def test_caffemodel_roundtrip(tmp_path):
    net = mobilenet_ssd_netdef()
    m = caffe.CaffeNet(net, seed=7)
    blobs = {}
    for l in net.layers:
        if l.type == "Convolution":
            w, b = m.conv_weights(l.name)
            blobs[l.name] = [w.detach().numpy(), b.detach().numpy()]
    path = tmp_path / "m.caffemodel"
    caffe.save_caffemodel(path, blobs)
    back = caffe.load_caffemodel(path)
    assert set(back) == set(blobs)
    for k in blobs:
        assert np.array_equal(back[k][0], blobs[k][0]) and np.array_equal(back[k][1], blobs[k][1])
    m2 = caffe.CaffeNet(net, back, seed=99)
    w1, _ = m.conv_weights("conv5")
    w2, _ = m2.conv_weights("conv5")
    assert torch.equal(w1, w2)


def test_nms_reference_semantics():
    boxes = torch.tensor([[0, 0, 1, 1], [0, 0, 1, 0.9], [2, 2, 3, 3.0]])
    scores = torch.tensor([0.9, 0.8, 0.7])
    assert caffe.nms_indices(boxes, scores, 0.45, 100) == [0, 2]
    assert caffe.nms_indices(boxes, scores, 0.95, 100) == [0, 1, 2]


def test_executor_cpu_path_shapes():
    ex = SSDExecutor()
    from distributedvolunteercomputing_amd.ops import vision as V

    frames = torch.randint(0, 255, (2, 100, 160, 3), dtype=torch.uint8)
    small = V.resize_width(frames, 400)
    assert small.shape == (2, 250, 400, 3)
    dets, cnt = ex.detect(small)
    assert dets.shape == (2, 100, 7) and cnt.shape == (2,)
