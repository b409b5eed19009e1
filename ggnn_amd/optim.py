"""The reference's optimizer step for the path's variables, on the GPU.

``chem_tensorflow.py:494-503``: ``tf.clip_by_norm(grad, clamp_gradient_norm)``
per variable, then ``tf.compat.v1.train.AdamOptimizer(learning_rate, beta1=0.9,
beta2=0.999)`` (epsilon 1e-8, TF1 bias correction folded into the step size).
One fused pair of HIP launches (``ggnn_adam_step``) updates every tensor;
PyTorch tensors are only the memory holders.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("m", ctypes.c_void_p),
                ("v", ctypes.c_void_p), ("n", ctypes.c_int64), ("sqnorm", ctypes.c_void_p)]


MAX_TENSORS = 16
SCRATCH_PER_TENSOR = 256   # GGNN_ADAM_SCRATCH_PER_TENSOR


class ClipAdam:
    """``step(grads)`` applies clip_by_norm + Adam to ``params`` in place.

    params: list of fp32 contiguous device tensors (the variables).
    grads:  matching list (or dict by position) of fp32 device tensors, e.g.
            ``FlatGradients.views`` values; ``grad_scale`` multiplies them first
            (1/N turns an N-rank all-reduce sum into the mean).
    """

    def __init__(self, params, learning_rate=0.003, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 clamp_gradient_norm=1.0):
        self.params = list(params)
        if not 1 <= len(self.params) <= MAX_TENSORS:
            raise ValueError("ClipAdam takes 1..%d tensors" % MAX_TENSORS)
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device.type != "cuda":
                raise ValueError("parameters must be contiguous fp32 tensors on the GPU")
        self.lr, self.b1, self.b2, self.eps = float(learning_rate), float(beta1), float(beta2), float(epsilon)
        self.clip = float(clamp_gradient_norm)
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0
        self._scratch = torch.zeros(MAX_TENSORS * SCRATCH_PER_TENSOR, dtype=torch.float32, device=self.params[0].device)
        self._lib = _lib.load()

    @torch.no_grad()
    def step(self, grads, grad_scale: float = 1.0, sqnorms=None, step_dev=None) -> None:
        """sqnorms: optional list (None entries allowed) of device scalars that
        replace ||grad||^2 in clip_by_norm -- the per-lookup norm of an
        embedding's IndexedSlices gradient (EmbeddingFrontEnd.backward).
        step_dev: a device int64 tensor holding the step count to use
        (ggnn_adam_step_dev, for hipGraph capture); the caller keeps ``t``
        (it is not advanced here)."""
        grads = list(grads)
        sqnorms = list(sqnorms) if sqnorms is not None else [None] * len(grads)
        if len(grads) != len(self.params):
            raise ValueError("expected %d gradients, got %d" % (len(self.params), len(grads)))
        tab = (AdamTensor * len(self.params))()
        for i, (p, g) in enumerate(zip(self.params, grads)):
            if g.shape != p.shape or g.dtype != torch.float32 or not g.is_contiguous():
                raise ValueError("gradient %d must be contiguous fp32 of shape %s" % (i, tuple(p.shape)))
            sq = sqnorms[i]
            tab[i] = AdamTensor(p.data_ptr(), g.data_ptr(), self.m[i].data_ptr(), self.v[i].data_ptr(), p.numel(),
                                None if sq is None else sq.data_ptr())
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        if step_dev is not None:
            if step_dev.dtype != torch.int64 or step_dev.device.type != "cuda":
                raise ValueError("step_dev must be a device int64 tensor")
            _lib.check(self._lib.ggnn_adam_step_dev(tab, len(self.params), self.lr, self.b1, self.b2, self.eps,
                                                    self.clip, ctypes.c_void_p(step_dev.data_ptr()),
                                                    float(grad_scale), ctypes.c_void_p(self._scratch.data_ptr()),
                                                    stream), "ggnn_adam_step_dev")
            return
        self.t += 1
        _lib.check(self._lib.ggnn_adam_step(tab, len(self.params), self.lr, self.b1, self.b2, self.eps, self.clip,
                                            self.t, float(grad_scale), ctypes.c_void_p(self._scratch.data_ptr()),
                                            stream), "ggnn_adam_step")
