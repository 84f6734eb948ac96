"""Hot ops. On GPU every op here runs a hand-written gfx950 HIP kernel from ``_C``;
on CPU the same call runs the plain-PyTorch reference (used by tests and CPU volunteers)."""
from ._lib import available as native_available, native  # noqa: F401
from .activations import bias_gelu, gelu, swiglu  # noqa: F401
from .attention import causal_attention, fused_bias_grad_ok, gqa_attention  # noqa: F401
from .embedding import embed  # noqa: F401
from .linear import gemm_nt, linear, mlp_gelu, native_linear_ok, set_gemm_backend, wgrad  # noqa: F401
from .loss import cross_entropy, lm_head_cross_entropy  # noqa: F401
from .norm import add_layernorm, add_rmsnorm, layernorm, rmsnorm  # noqa: F401
from .rope import rope_qkv  # noqa: F401
from .optim import (adamw_step, axpy_bf16, f32_to_bf16, lsgd_apply, lsgd_delta, new_ostate,  # noqa: F401
                    reduce_bcast_bf16)
