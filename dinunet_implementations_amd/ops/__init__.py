"""Hot ops.  On a GPU every op below runs hand-written gfx950 kernels from the in-tree library
(``_native/libdinunet_kernels.so``); on CPU they run the reference math (``ops.reference``)."""
from . import _lib, capture, reference
from ._lib import native_available
from .gemm import PLAIN_BLAS, mm, mm_grouped, mm_plain
from .linear import linear_bias_relu
from .lstm import bilstm as _bilstm_fused, lstm_supported, padded_hidden
from .optim import (DeviceSource, FlatParams, FusedAdam, StepRecorder, cast_bf16_to_f32,
                    cast_f32_to_bf16, step_prologue)
from .heads import softmax_ce, log_softmax_nll
from .head import HeadSpec, head_loss
from .layernorm import LayerNorm, layer_norm


def bilstm(x, params, reduce: str = "none", modules=None, packed=None, xp=None,
           relu_input: bool = False):
    return _bilstm_fused(x, params, reduce=reduce, modules=modules, packed=packed, xp=xp,
                         relu_input=relu_input)


__all__ = [
    "LayerNorm", "layer_norm",
    "mm", "linear_bias_relu", "bilstm", "lstm_supported", "padded_hidden", "FlatParams",
    "DeviceSource", "StepRecorder", "FusedAdam", "cast_bf16_to_f32", "cast_f32_to_bf16", "step_prologue", "HeadSpec", "head_loss",
    "softmax_ce", "log_softmax_nll", "native_available", "capture", "reference",
]
