"""Host-side rules of the hand-written forward GEMM / implicit-GEMM convolution (csrc/kernels/gemm_f.hip), which run
on the CPU: which shapes it takes, the tile it picks and the automatic K split (one round of <= 256 workgroups,
each split an even number >= 6 of 32-deep slices)."""
import pytest

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def C():
    from distributedvolunteercomputing_amd.ops._lib import native

    try:
        return native()
    except RuntimeError as e:  # the extension is built by __graft_entry__.build() / _build; CPU-only rules
        pytest.skip(str(e))


def test_supported_shapes(C):
    assert C.gemm_f_supported(65536, 2304, 768)
    assert C.gemm_f_supported(300, 128, 192) and C.gemm_f_supported(1000, 64, 576)  # narrow tiles
    assert not C.gemm_f_supported(512, 96, 768)    # N neither 64 nor a multiple of 128
    assert not C.gemm_f_supported(512, 256, 160)   # K < 192
    assert not C.gemm_f_supported(512, 256, 800)   # K % 64
    # every ResNet-50 3x3 convolution at B = 128 (stride 1 and the stride-2 first blocks)
    for hw, c, s in [(56, 64, 1), (28, 128, 1), (14, 256, 1), (7, 512, 1), (56, 128, 2), (28, 256, 2), (14, 512, 2)]:
        assert C.gemm_f_conv3x3_supported(128, hw, hw, c, c, s)
    assert not C.gemm_f_conv3x3_supported(128, 224, 224, 3, 64, 2)   # the 7x7 stem's 3 channels
    assert not C.gemm_f_conv3x3_supported(2, 8, 8, 96, 128, 1)       # Cin not a power of two


def test_automatic_split(C):
    # few tiles, deep K: split until one round of 256 workgroups, even slice counts >= 6 per split
    assert C.gemm_f_splits(128 * 14 * 14, 256, 9 * 256) == 2   # 98 tiles, 72 slices
    assert C.gemm_f_splits(128 * 7 * 7, 512, 9 * 512) == 4     # 50 tiles, 144 slices
    assert C.gemm_f_splits(65536, 2304, 768) == 1              # 2304 tiles: no split
    assert C.gemm_f_splits(128 * 28 * 28, 128, 9 * 128) == 1   # 392 tiles of 256 x 128
    for M, N, K in [(700, 640, 1536), (196, 512, 4608), (2500, 512, 2304)]:
        s = C.gemm_f_splits(M, N, K)
        nk = K // 32
        assert nk % s == 0 and (nk // s) % 2 == 0 and nk // s >= 6
