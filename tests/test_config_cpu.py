"""The runtime config (config.py): env parsing, validation, live updates seen by the ops."""
import pytest

from distributedvolunteercomputing_amd import config


def test_from_env_parses_and_validates():
    c = config.from_env({"VCX_GEMM": "vcx", "VCX_ASYNC_WGRAD": "1", "VCX_WGRAD_BIG_SPLIT_MIN_M": "4096",
                         "VCX_GLOO_HOST": "10.0.0.2", "VCX_STORE_PORT": "30000"})
    assert c.gemm == "vcx" and c.async_wgrad is True and c.wgrad_big_split_min_m == 4096
    assert c.gloo_host == "10.0.0.2" and c.store_port_train == c.store_port_video == 30000
    assert config.from_env({}) == config.RuntimeConfig()
    with pytest.raises(ValueError):
        config.from_env({"VCX_GEMM": "cublas"})
    with pytest.raises(ValueError):
        config.from_env({"VCX_WGRAD_BIG_SPLIT_MIN_M": "many"})


def test_update_override_and_consumers():
    import importlib

    from distributedvolunteercomputing_amd.ops import _lib

    linear = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")

    assert config.get().force_reference_ops is False
    with _lib.reference_ops():
        assert config.get().force_reference_ops is True
        assert not _lib.use_native(object())
    assert config.get().force_reference_ops is False
    with config.override(gemm="vcx"):
        assert config.get().gemm == "vcx"
        linear.set_gemm_backend("lib")
        assert config.get().gemm == "lib"
    assert config.get().gemm == "lib"
    with pytest.raises(AttributeError):
        config.update(no_such_field=1)
    with pytest.raises(ValueError):
        config.update(p2p_backend="mpi")
    assert "VCX_GEMM" in config.describe()


def test_round6_compute_path_flags():
    """VCX_GEMM_FWD (forward GEMMs on gemm_f, opt-in) and VCX_CONV3X3_FWD (the stage-3/4 3x3 convolutions on
    gemm_f's implicit GEMM, default): parsed, validated, and refused by the CPU-side gates."""
    import torch

    import importlib

    from distributedvolunteercomputing_amd.models import resnet

    linear = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")
    c = config.from_env({"VCX_GEMM_FWD": "vcx", "VCX_CONV3X3_FWD": "lib"})
    assert c.gemm_fwd == "vcx" and c.conv3x3_fwd == "lib"
    d = config.RuntimeConfig()
    assert d.gemm_fwd == "lib" and d.conv3x3_fwd == "vcx"
    for env in ({"VCX_GEMM_FWD": "hipblaslt"}, {"VCX_CONV3X3_FWD": "miopen"}):
        with pytest.raises(ValueError):
            config.from_env(env)
    with config.override(gemm_fwd="vcx"):
        assert not linear.gemm_f_ok(65536, 2304, 768, torch.zeros(2, 2, dtype=torch.bfloat16))  # CPU tensor
    with config.override(conv3x3_fwd="lib"):
        assert not resnet._fwd_vcx(128, 14, 14, 256, 256, 1)  # off: no native call made
    m = resnet.Conv3x3(64, 256).to(torch.bfloat16)
    x = torch.randn(1, 64, 6, 6, dtype=torch.bfloat16)
    assert m(x).shape == (1, 256, 6, 6)  # CPU: nn.Conv2d
