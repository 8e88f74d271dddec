"""Python entry to the MFMA GEMM (K17, csrc/nn/gemm_mfma.hip): ONNX ``Gemm`` / ``MatMul`` and the FC
layers of the executor. Operands are torch CUDA tensors (fp32 / fp16 / bf16); strides are read from the
tensors, so transposed and batch-broadcast operands need no copy. fp32 runs on the exact f32-input
16x16x4 MFMA (no TF32-style rounding), fp16 / bf16 on 16x16x32 with fp32 accumulation."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import native

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def supported(*ts: torch.Tensor) -> bool:
    return all(t.is_cuda and t.dtype in _DT for t in ts) and len({t.dtype for t in ts}) == 1


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _mat(t: torch.Tensor) -> Tuple[torch.Tensor, int, int]:
    """(tensor, ld, trans) of a 2-D operand: row-major (ld = stride 0) or column-major (transposed view);
    anything else is made contiguous."""
    if t.stride(1) == 1 and t.stride(0) >= max(1, t.shape[1]):
        return t, t.stride(0), 0
    if t.stride(0) == 1 and t.stride(1) >= max(1, t.shape[0]):
        return t, t.stride(1), 1
    t = t.contiguous()
    return t, t.stride(0), 0


def gemm(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None, c: Optional[torch.Tensor] = None,
         alpha: float = 1.0, beta: float = 1.0, relu: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(alpha * a @ b + beta * (bias | c)) for 2-D ``a`` [M, K], ``b`` [K, N] (any strides: a transposed
    view is read in place). ``bias``: [N] fp32-castable; ``c``: [M, N] (broadcastable, materialised)."""
    M, K = a.shape
    K2, N = b.shape
    if K != K2:
        raise ValueError(f"gemm: inner dims {K} != {K2}")
    a, lda, ta = _mat(a)
    # b [K, N] row-major is the "NN" layout (trans_b = 0); a transposed view of an [N, K] weight is "NT"
    bt, ldb, tb = _mat(b)
    y = out if out is not None else torch.empty((M, N), device=a.device, dtype=a.dtype)
    bias32 = None if bias is None else bias.reshape(-1).to(a.device, torch.float32).contiguous()
    cm = None
    if c is not None:
        cm = torch.broadcast_to(c.to(a.device, a.dtype), (M, N)).contiguous()
    native.load("_nn").gemm(a.data_ptr(), bt.data_ptr(), y.data_ptr(), M, N, K, 1, lda, ldb, y.stride(0), 0, 0, 0,
                            ta, tb, float(alpha), float(beta), 0 if bias32 is None else bias32.data_ptr(),
                            0 if cm is None else cm.data_ptr(), N, 0, int(bool(relu)), _DT[a.dtype], _stream(a))
    return y


def matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """numpy/ONNX MatMul semantics (1-D promotion, batch broadcasting) on the MFMA GEMM: the batch is one
    launch (grid z); a broadcast operand gets batch stride 0 instead of a copy."""
    va, vb = a.dim() == 1, b.dim() == 1
    if va:
        a = a.unsqueeze(0)
    if vb:
        b = b.unsqueeze(1)
    M, K = a.shape[-2:]
    N = b.shape[-1]
    batch_shape = torch.broadcast_shapes(a.shape[:-2], b.shape[:-2])
    nb = 1
    for s in batch_shape:
        nb *= s
    A = a.expand(*batch_shape, M, K).reshape(nb, M, K) if a.dim() > 2 or batch_shape else a.reshape(1, M, K)
    B = b.expand(*batch_shape, K, N).reshape(nb, K, N) if b.dim() > 2 or batch_shape else b.reshape(1, K, N)

    def op3(t):  # (tensor, ld, trans, batch stride) of a [nb, R, C] operand
        if t.stride(2) == 1 and t.stride(1) >= max(1, t.shape[2]):
            return t, t.stride(1), 0, t.stride(0) if t.shape[0] > 1 else 0
        if t.stride(1) == 1 and t.stride(2) >= max(1, t.shape[1]):
            return t, t.stride(2), 1, t.stride(0) if t.shape[0] > 1 else 0
        t = t.contiguous()
        return t, t.stride(1), 0, t.stride(0)

    A, lda, ta, sa = op3(A)
    B, ldb, tb, sb = op3(B)
    y = torch.empty((nb, M, N), device=a.device, dtype=a.dtype)
    native.load("_nn").gemm(A.data_ptr(), B.data_ptr(), y.data_ptr(), M, N, K, nb, lda, ldb, N, sa, sb, M * N,
                            ta, tb, 1.0, 1.0, 0, 0, 0, 0, 0, _DT[a.dtype], _stream(a))
    y = y.reshape(*batch_shape, M, N)
    if va:
        y = y.squeeze(-2)
    if vb:
        y = y.squeeze(-1)
    return y
