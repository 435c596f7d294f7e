"""ICA bi-LSTM classifier, reference ``comps/icalstm/models.py:5-110``.

Module tree and ``state_dict`` keys are identical to the reference:
``encoder.0.*``, ``lstm.lstms.{0,1}.{i2h,h2h}.*``, ``classifier.{1,2,4,6}.*`` (``classifier.2``
is a BatchNorm1d *with* running stats).  Numerics follow the reference quirks (double sigmoid on
i/f/o, per-direction hidden = hidden_size // 2, reverse outputs in processing order,
``num_layers`` ignored: SURVEY.md A1-A4).

Execution is MI355X-first: on a GPU the encoder runs as one ``[B*S, C*W] x [C*W, I]`` bf16 MFMA
GEMM with a fused bias+ReLU epilogue (no per-sample Python loop, reference ``models.py:107``),
the input projection of both directions is one GEMM hoisted out of the recurrence, and the
recurrence of both directions runs in one persistent HIP kernel whose recurrent weights stay
resident in VGPRs for all time steps (``ops.lstm``); classifier + softmax-CE are one fused
launch per direction (``ops.head``).  On CPU the module runs the reference math
(``ops.reference``), which is also the test oracle.
"""
from __future__ import annotations

import os
import warnings
from typing import Optional, Tuple

import torch
import torch.nn as nn

from .. import ops
from ..ops import reference as ref


class LSTMCell(nn.Module):
    """One LSTM direction built from two ``nn.Linear`` (``models.py:5-45``).

    Keeping ``i2h``/``h2h`` as real Linear modules matters for rank-dAD: the engine sees every
    Linear's inputs and output-gradients.
    """

    def __init__(self, input_size: int, hidden_size: int, bias: bool = True):
        super().__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.bias = bias
        self.i2h = nn.Linear(input_size, 4 * hidden_size, bias=bias)
        self.h2h = nn.Linear(hidden_size, 4 * hidden_size, bias=bias)

    def init_hidden(self, bz: int, device="cpu"):
        return (torch.zeros(bz, self.hidden_size, device=device),
                torch.zeros(bz, self.hidden_size, device=device))

    def params(self):
        return (self.i2h.weight, self.i2h.bias, self.h2h.weight, self.h2h.bias)

    def forward(self, x: torch.Tensor, h=None):
        return ref.lstm_cell_seq(x, *self.params(), h0=h)


class LSTM(nn.Module):
    """Bi-directional wrapper (``models.py:48-66``)."""

    def __init__(self, input_size: int, hidden_size: int, bidirectional: bool = True,
                 num_layers: int = 1, bias: bool = True):
        super().__init__()
        self.input_size = input_size
        self.num_layers = num_layers  # stored, ignored (reference quirk A3)
        self.bidirectional = bidirectional
        self.num_direction = 2 if bidirectional else 1
        self.hidden_size = hidden_size // self.num_direction
        self.bias = bias
        self.lstms = nn.ModuleList([LSTMCell(input_size, self.hidden_size, bias=bias)
                                    for _ in range(self.num_direction)])
        self.use_fused = True

    def fused_ok(self, x: torch.Tensor) -> bool:
        return (self.use_fused and x.is_cuda and self.bias
                and ops.lstm_supported(x.shape[0], self.input_size, self.hidden_size,
                                       self.num_direction, seq=x.shape[1]))

    def prepack(self, device, side: bool = True, casts=(), cast_out=None):
        """Pack the LSTM weights into the kernel layouts ahead of the forward (on the side
        stream when ``side``); ``casts`` get bf16 copies from the same launch."""
        from ..ops.lstm import pack_params
        flat = [t for cell in self.lstms for t in cell.params()]
        return pack_params(flat, self.input_size, device, side=side, casts=casts,
                           cast_out=cast_out)

    def forward(self, x: torch.Tensor, h=None, reduce: str = "none", packed=None, xp=None,
                relu_input: bool = False):
        """``reduce='none'`` returns ``(hidden_seq [B,S,H*dirs], (h, c))`` like the reference;
        ``reduce='mean'`` returns the temporal mean ``[B, H*dirs]`` instead of the sequence
        (what ``ICALstm`` consumes) so the fused kernel never materialises the sequence."""
        if h is None and self.fused_ok(x):
            params = [cell.params() for cell in self.lstms]
            return ops.bilstm(x, params, reduce=reduce, modules=list(self.lstms), packed=packed,
                              xp=xp, relu_input=relu_input)
        if x.is_cuda and self.use_fused and h is None and self.bias:
            # only the hidden size can push a default (zero-state, biased) LSTM off the fused
            # kernels; an explicit initial state or bias=False takes the reference loop by choice
            _slow_lstm_gate(self.hidden_size, x.shape[0])
        x = x.to(self.lstms[0].i2h.weight.dtype)  # the fused encoder hands over bf16
        if h is not None:
            hs, (h_t, c_t) = self.lstms[0](x, h)
            if self.bidirectional:
                rhs, (rh, rc) = self.lstms[1](torch.flip(x, (1,)), h)
                hs = torch.cat([hs, rhs], 2)
                h_t, c_t = torch.cat([h_t, rh], 1), torch.cat([c_t, rc], 1)
        else:
            hs, (h_t, c_t) = ref.bilstm(x, [c.params() for c in self.lstms], self.bidirectional,
                                        modules=list(self.lstms))
        if reduce == "mean":
            return hs.mean(1), (h_t, c_t)
        return hs, (h_t, c_t)


_SLOW_WARNED = False


def _slow_lstm_gate(hidden: int, batch: int):
    """A GPU LSTM the persistent kernels do not cover (per-direction hidden > 512; up to 192
    W_hh stays in the register file, up to 512 the kernels stream it from L2 every step) runs
    the reference's per-step loop of library ops, ~100x slower.  That is never silent: it raises unless ``DINUNET_ALLOW_SLOW_LSTM=1`` opts in, and
    then warns once."""
    global _SLOW_WARNED
    msg = (f"LSTM hidden {hidden} (batch {batch}) is outside the fused gfx950 kernels "
           f"(per-direction hidden <= 512); the step-by-step reference loop would run instead")
    if os.environ.get("DINUNET_ALLOW_SLOW_LSTM", "0") != "1":
        raise NotImplementedError(msg + ": set DINUNET_ALLOW_SLOW_LSTM=1 to accept it")
    if not _SLOW_WARNED:
        warnings.warn(msg, RuntimeWarning, stacklevel=3)
        _SLOW_WARNED = True


class ICALstm(nn.Module):
    # the encoder GEMM rounds its input to bf16 while staging: a bf16 batch is bit-identical
    accepts_bf16_input = True

    def __init__(self, input_size: int = 256, hidden_size: int = 256, bidirectional: bool = True,
                 num_cls: int = 2, num_comps: int = 53, window_size: int = 20,
                 num_layers: int = 1, norm_layer: str = "batch"):
        super().__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.num_comp = num_comps
        self.window_size = window_size
        self.encoder = nn.Sequential(nn.Linear(num_comps * window_size, input_size), nn.ReLU())
        self.lstm = LSTM(input_size=input_size, hidden_size=hidden_size,
                         bidirectional=bidirectional, num_layers=num_layers)
        # norm_layer "batch": the reference's BatchNorm1d (fused head kernels); "layer": the
        # optional LayerNorm on its own gfx950 kernels (ops.layernorm; the head then runs
        # module by module)
        if norm_layer not in ("batch", "layer"):
            raise ValueError(f"norm_layer {norm_layer!r}: expected 'batch' or 'layer'")
        self.classifier = nn.Sequential(
            nn.Dropout(0.25),
            nn.Linear(hidden_size, 256),
            nn.BatchNorm1d(256) if norm_layer == "batch" else ops.LayerNorm(256),
            nn.ReLU(),
            nn.Linear(256, 64),
            nn.ReLU(),
            nn.Linear(64, num_cls),
        )
        self.use_fused = True
        self._head: Optional[ops.HeadSpec] = None

    def head_spec(self) -> "ops.HeadSpec":
        if self._head is None:
            self._head = ops.HeadSpec(list(self.classifier))
        return self._head

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        """``[B, S, C, W] -> [B, S, I]``: one batched GEMM instead of the per-sample loop."""
        B, S = x.shape[:2]
        flat = x.reshape(B * S, -1)
        lin = self.encoder[0]
        if self.use_fused and x.is_cuda:
            enc = ops.linear_bias_relu(flat, lin.weight, lin.bias, module=lin)
        else:
            enc = torch.relu(lin(flat))  # module call: rank-dAD hooks see it
        return enc.view(B, S, -1)

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
        enc = self.encode(x)
        o, h = self.lstm(enc, reduce="mean")
        return self.classifier(o.flatten(1).to(self.classifier[1].weight.dtype)), h

    def forward_loss(self, x: torch.Tensor, y: torch.Tensor):
        """``(probs, ce_loss, argmax)`` (reference ``comps/icalstm/__init__.py:59-63``); on a GPU
        the classifier, softmax and cross-entropy are one fused launch each way."""
        return self.body_loss(self.stem(x), y)

    def stem(self, x: torch.Tensor) -> torch.Tensor:
        """First half of :meth:`forward_loss`: the encoder (``[B,S,C,W] -> [B,S,I]``).

        Its parameter gradients are the LAST ones the backward produces, so a training step can
        stop the backward at the stem output, start the all-reduce of every other gradient, and
        only then run the stem's backward (``runtime.step.TrainStep`` split capture)."""
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()  # host datasets are float64 (reference comps/icalstm/__init__.py:29)
        self._packed = None
        if self.use_fused and x.is_cuda and self.lstm.fused_ok(x) and ops.capture.active() is None:
            # in-stream: as a side-stream branch of the step graph the pack saved nothing (it
            # fills the chip anyway) and added a cross-queue wait before the input projection
            lin = self.encoder[0]
            casts = []
            want = lin.bias is not None
            if want and x.dtype == torch.float32:
                # eager callers: same operand values as the step graph's bf16 input (every GEMM
                # rounds to bf16 while staging), so eager and replayed steps agree
                x = x.to(torch.bfloat16)
            self._packed = self.lstm.prepack(
                x.device, side=False, casts=(lin.weight, lin.bias) if want else (),
                cast_out=casts)
            B, S = x.shape[:2]
            flat = x.reshape(B * S, -1)
            if casts:
                enc = ops.linear_bias_relu(flat, lin.weight, lin.bias, module=lin,
                                           bf16_params=tuple(casts))
                return enc.view(B, S, -1)
        return self.encode(x)

    def prologue_rides_pack(self, x: torch.Tensor) -> bool:
        """Will :meth:`stem` on ``x`` start with the LSTM weight-pack launch (which can also run
        a device-fed step prologue, ``ops.lstm.ride_pack``)?  Same test as in :meth:`stem`."""
        return bool(self.use_fused and x.is_cuda and self.lstm.fused_ok(x)
                    and ops.capture.active() is None)

    def stem_parameters(self):
        return self.encoder.parameters()

    def split_at_projection(self, x: torch.Tensor) -> bool:
        """Can a split step cut at the LSTM input projection (:meth:`proj_stem` /
        :meth:`proj_body_loss`) instead of the encoder output?  The fused GPU path only."""
        return bool(self.use_fused and x.is_cuda and self.lstm.fused_ok(x)
                    and ops.capture.active() is None)

    def proj_stem(self, x: torch.Tensor) -> torch.Tensor:
        """Encoder + the LSTM input projection of both directions (``ops.lstm.project``):
        ``[B,S,C,W] -> xp [B*S, ndir*4HD]``.  The backward of everything AFTER xp (recurrences,
        head, every LSTM and head weight gradient) runs before the backward of xp itself (the
        encoder input gradient and the encoder's weight gradients): the multi-site split step
        cuts there and all-reduces the LSTM + head gradients under the encoder backward.  The
        encoder output is kept (detached) for :meth:`proj_body_loss`."""
        from ..ops.lstm import project
        enc = self.stem(x)
        self._split_enc = enc.detach()
        return project(enc, self._packed, relu_input=True)

    def proj_body_loss(self, xp: torch.Tensor, y: torch.Tensor):
        """Second half of :meth:`proj_stem`: recurrences on the given projection, head, loss."""
        enc, self._split_enc = self._split_enc, None
        packed, self._packed = getattr(self, "_packed", None), None
        o, _ = self.lstm(enc, reduce="mean", packed=packed, xp=xp, relu_input=True)
        o = o.flatten(1).to(self.classifier[1].weight.dtype)
        if self.use_fused and o.is_cuda:
            return ops.head_loss(o, self.head_spec(), y, log_out=False)
        return ops.softmax_ce(self.classifier(o), y)

    def persistent_pack(self, device) -> Optional["ops.lstm.PersistentPack"]:
        """Step-persistent packed operands for a fused Adam that keeps them current
        (``runtime.step.TrainStep`` device-fed steps): the LSTM weight images and the encoder's
        bf16 weight / bias, i.e. exactly what :meth:`stem`'s pack launch would produce."""
        lin = self.encoder[0]
        if not (self.use_fused and lin.bias is not None and self.lstm.bias):
            return None
        from ..ops.lstm import PersistentPack
        flat = [t for cell in self.lstm.lstms for t in cell.params()]
        # + bf16 images of the classifier weights for the replicated head (ops.head, head_rep.hip)
        extra = [m.weight for m in self.classifier if isinstance(m, nn.Linear)]
        return PersistentPack(flat, self.lstm.input_size, device, casts=(lin.weight, lin.bias),
                              extra=extra)

    def body_loss(self, enc: torch.Tensor, y: torch.Tensor):
        """Second half of :meth:`forward_loss`: bi-LSTM, classifier, softmax-CE on ``enc``."""
        packed, self._packed = getattr(self, "_packed", None), None
        # enc = ReLU(encoder), consumed only by the LSTM: its mask joins the LSTM's dX GEMM
        o, _ = self.lstm(enc, reduce="mean", packed=packed, relu_input=True)
        o = o.flatten(1).to(self.classifier[1].weight.dtype)
        if self.use_fused and o.is_cuda:
            return ops.head_loss(o, self.head_spec(), y, log_out=False)
        logits = self.classifier(o)
        return ops.softmax_ce(logits, y)
