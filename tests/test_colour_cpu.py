"""C++ colour conversion of the video I/O path (csrc/runtime/colour.cpp) against the numpy
formulas it replaces: bit-identical for BGR -> YUV 4:4:4, YUV 4:4:4 -> BGR and YUV 4:2:0 -> BGR
(2x2 chroma replication, odd sizes included), and a 4:2:0 Y4M file read through Y4MSource."""
import numpy as np
import pytest

from distributedvolunteercomputing_amd.io import video as V


@pytest.mark.parametrize("h,w", [(720, 1280), (225, 400), (7, 9), (721, 1281), (1, 1)])
def test_bgr_yuv444_roundtrip_bit_exact(h, w):
    f = np.random.default_rng(h * w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    y = V.bgr_to_yuv444(f)
    assert np.array_equal(y, V._bgr_to_yuv444_np(f))
    assert np.array_equal(V.yuv444_to_bgr(y), V._yuv444_to_bgr_np(y))


def _write_y4m_420(path, planes, w, h):
    with open(path, "wb") as fh:
        fh.write(f"YUV4MPEG2 W{w} H{h} F30:1 Ip A1:1 C420jpeg\n".encode())
        for y, u, v in planes:
            fh.write(b"FRAME\n" + y.tobytes() + u.tobytes() + v.tobytes())


@pytest.mark.parametrize("h,w", [(72, 128), (9, 13)])
def test_y4m_420_source_matches_numpy(tmp_path, h, w):
    rng = np.random.default_rng(w)
    cw, ch = (w + 1) // 2, (h + 1) // 2
    planes = [(rng.integers(0, 256, (h, w), dtype=np.uint8), rng.integers(0, 256, (ch, cw), dtype=np.uint8),
               rng.integers(0, 256, (ch, cw), dtype=np.uint8)) for _ in range(3)]
    p = tmp_path / "a.y4m"
    _write_y4m_420(p, planes, w, h)
    src = V.Y4MSource(str(p))
    for y, u, v in planes:
        ok, f = src.read()
        assert ok
        ref = V._yuv444_to_bgr_np(np.stack([y, u.repeat(2, 0).repeat(2, 1)[:h, :w], v.repeat(2, 0).repeat(2, 1)[:h, :w]]))
        assert np.array_equal(f, ref)
    assert src.read()[0] is False
    src.release()


def test_native_colour_rejects_strided_buffers():
    from distributedvolunteercomputing_amd._native_loader import native

    f = np.zeros((8, 16, 3), np.uint8)
    out = np.zeros((3, 8, 32), np.uint8)[:, :, ::2]  # a strided view: must not be written linearly
    with pytest.raises(ValueError):
        native().bgr_to_yuv444(f, out, 16, 8)


@pytest.mark.parametrize("k,h,w", [(100, 225, 400), (3, 7, 9), (1, 1, 1)])
def test_y4m_write_many_matches_per_frame(tmp_path, k, h, w):
    """The sink's batched path (one multi-threaded native conversion per received chunk, frames
    written from the planar buffer) produces the same file as writing frame by frame, whether the
    frames are consecutive views of one chunk buffer or scattered arrays."""
    frames = np.random.default_rng(k + h).integers(0, 256, (k, h, w, 3), dtype=np.uint8)
    a, b, c = (V.Y4MWriter(str(tmp_path / f"{n}.y4m"), w, h, 30) for n in "abc")
    for f in frames:
        a.write(f)
    b.write_many([frames[i] for i in range(k)])  # views of one contiguous block
    c.write_many([frames[i].copy() for i in range(k)][::-1][::-1])  # separate arrays: stacked copy
    for x in (a, b, c):
        x.release()
    ra, rb, rc = ((tmp_path / f"{n}.y4m").read_bytes() for n in "abc")
    assert ra == rb == rc
    assert len(ra) > k * 3 * h * w


@pytest.mark.parametrize("chunks", [[5], [3, 1, 7], [1, 1, 1, 1]])
def test_npy_sink_streams_and_finalises_header(tmp_path, chunks):
    """The npy sink writes each chunk at its offset as it arrives (threaded positional writes into the
    page cache) and rewrites the header with the final frame count on release: np.load reads it back."""
    rng = np.random.default_rng(len(chunks))
    n = sum(chunks)
    frames = rng.integers(0, 256, (n, 19, 23, 3), dtype=np.uint8)
    w = V.NpyWriter(tmp_path / "o.npy", 23, 19)
    i = 0
    for c in chunks:
        if c == 1:
            w.write(frames[i])
        else:
            w.write_many(list(frames[i:i + c]))
        i += c
    w.release()
    out = np.load(tmp_path / "o.npy")
    assert out.shape == frames.shape and np.array_equal(out, frames)
    assert (tmp_path / "o.npy").stat().st_size == V.NpyWriter.HEADER + frames.nbytes


def test_native_write_bytes_positional(tmp_path):
    """write_bytes: a regular file grows to cover the range and keeps the bytes before it."""
    from distributedvolunteercomputing_amd._native_loader import native

    rt = native()
    p = tmp_path / "b.bin"
    data = np.random.default_rng(1).integers(0, 256, 3 << 20, dtype=np.uint8)
    with open(p, "wb") as f:
        f.write(b"head")
        assert rt.write_bytes(f.fileno(), 100, data) == data.nbytes
        assert rt.write_bytes(f.fileno(), 100 + data.nbytes, data[:7]) == 7
    b = p.read_bytes()
    assert b[:4] == b"head" and b[4:100] == bytes(96)
    assert b[100:100 + data.nbytes] == data.tobytes() and b[100 + data.nbytes:] == data[:7].tobytes()
