"""Native HIP/CDNA4 compute ops (gfx950) with a bit-compatible PyTorch reference for CPU tensors."""
from . import _ext, reference  # noqa: F401
from .fused import (adam_flat, flatten_into, linear_fwd, mlp_fwd_logits,  # noqa: F401
                    sgd_flat, softmax_xent, unflatten_from, wgrad_grouped, xent_head)
from .autograd import FusedLinear, fused_linear, fused_cross_entropy  # noqa: F401
