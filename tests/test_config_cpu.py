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
