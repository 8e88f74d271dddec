"""Python entry to the MFMA implicit-GEMM convolution (csrc/nn/conv_mfma.hip).

Tensors are torch CUDA tensors in channels_last memory (NHWC); weights are
packed once to [Cout, R, S, Cin]. Epilogue / prologue tensors are fp32. fp16/bf16 run on the 16x16x32
MFMA; fp32 either on the exact f32-input MFMA (16x16x4, 1/16 of the bf16 rate) or with every f32 operand
split over bf16 planes and the products rebuilt from 16x16x32 MFMAs (F32_MODES)."""
from __future__ import annotations

import os
from typing import Optional, Sequence, Tuple

import torch

from . import native

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}
_SPLITK = os.environ.get("SML_CONV_SPLITK", "0") not in ("", "0")
# fp32 convolution modes: exact f32 MFMAs (16x16x4, 1/16 of the bf16 rate on gfx950), or every f32 operand
# split into 2 / 3 bf16 planes with the products rebuilt from 3 / 6 bf16 MFMAs (16x16x32): ~16 / ~24
# significant bits per product (TF32 keeps 11), fp32 accumulation, fp32 in and out.
F32_MODES = {"exact": 0, "bf16x3": 3, "bf16x6": 4}


def f32_mode_default() -> str:
    import os

    # bf16x3 by default: ~16 significant bits per product, 2.9-4.3e-6 of max |y| against an fp64 convolution
    # and gated at <= 1e-5 on all 14 ResNet-50 layer shapes (tests/test_conv_mfma.py) - two orders of magnitude
    # tighter than TF32 (11 bits, ~1e-3), the fp32 conv math ORT's CUDA provider uses on tensor cores - at
    # +60 % ResNet-50 fp32 throughput over bf16x6 (11.9k -> 18.3k img/s at batch 128, profiles/r3/
    # conv_f32_modes). bf16x6 (error at the exact f32 MFMA's level) and exact stay selectable.
    m = os.environ.get("SML_CONV_F32", "bf16x3")
    if m not in F32_MODES:
        raise ValueError(f"SML_CONV_F32={m!r}: expected one of {sorted(F32_MODES)}")
    return m


def supported(cin: int, cout: int, groups: int, dtype: torch.dtype) -> bool:
    return dtype in _DT and bool(native.load("_nn").conv_supported(cin, cout, groups, _DT[dtype]))


_PLANES = {"bf16x3": 2, "bf16x6": 3}


def split_weight(wp: torch.Tensor, mode: str) -> torch.Tensor:
    """packed fp32 weights [Cout, R, S, C] -> [planes, Cout, R, S, C] bf16 with w = sum of the planes up to the
    last plane's rounding (each plane the RNE bf16 of what the earlier ones left: the kernel's own split)"""
    r = wp.float()
    planes = []
    for _ in range(_PLANES[mode]):
        h = r.to(torch.bfloat16)
        planes.append(h)
        r = r - h.float()
    return torch.stack(planes).contiguous()


def pack_weight(w: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """[Cout, Cin, R, S] -> contiguous [Cout, R, S, Cin] in ``dtype``."""
    return w.permute(0, 2, 3, 1).contiguous().to(dtype)


def out_hw(h: int, w: int, r: int, s: int, stride: Sequence[int], pad: Sequence[int], dil: Sequence[int]):
    """``pad`` = (top, left) symmetric or (top, left, bottom, right)."""
    pt, pl = pad[0], pad[1]
    pb, pr = (pad[2], pad[3]) if len(pad) == 4 else (pt, pl)
    oh = (h + pt + pb - dil[0] * (r - 1) - 1) // stride[0] + 1
    ow = (w + pl + pr - dil[1] * (s - 1) - 1) // stride[1] + 1
    return oh, ow


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def conv2d_nhwc(x: torch.Tensor, wp: torch.Tensor, r: int, s: int, stride=(1, 1), pad=(0, 0), dil=(1, 1),
                bias: Optional[torch.Tensor] = None, relu=False,
                in_affine: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, in_relu: bool = True,
                res: Optional[torch.Tensor] = None,
                out_affine: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, kernel: int = 0,
                f32_mode: Optional[str] = None, w_planes: Optional[torch.Tensor] = None):
    """y = conv(pro(x), w) + bias, ReLU, + res; optionally also y2 = relu(y * out_scale + out_shift).

    ``relu``: False/0 none, True/1 before the residual add, 2 after it. ``pad``: (top, left) or
    (top, left, bottom, right). ``x``: [B, C, H, W] channels_last, fp32/fp16/bf16 (C % 32 == 0 for fp32, % 64 otherwise). ``wp``: packed [Cout, R, S, C]
    (a channels_last [Cout, C, R, S] weight permuted to (0, 2, 3, 1) is exactly that). Returns y (and y2).
    ``kernel``: 0 picks the tile by shape; BM*1000+BN forces one (64064, 128064, 64128, 128128, 256128, 128256;
    128999 / 64999 = 8-wave 128x128 / 64x64; 256064 / 128164 = 256x64 / 128x64 with 64x64 wave tiles;
    128777 / 64777 / 256777 = LDS-DMA staged 128x128 / 64x64 / 256x64, f16/bf16 without in_affine).
    ``f32_mode`` (fp32 inputs): "exact" | "bf16x3" | "bf16x6" (see F32_MODES; default SML_CONV_F32 or bf16x6).
    ``w_planes``: split_weight(wp, mode) computed once per weight; the split modes then read the planes instead
    of splitting the weights in every block."""
    B, C, H, W = x.shape
    if not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv2d_nhwc expects a channels_last input")
    cout = wp.shape[0]
    if wp.shape != (cout, r, s, C) or wp.dtype != x.dtype or not wp.is_contiguous():
        raise ValueError(f"packed weight must be [Cout, {r}, {s}, {C}] {x.dtype}, got {tuple(wp.shape)} {wp.dtype}")
    oh, ow = out_hw(H, W, r, s, stride, pad, dil)
    y = torch.empty((B, cout, oh, ow), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    y2 = torch.empty_like(y) if out_affine is not None else None
    if res is not None and (res.shape != y.shape or not res.is_contiguous(memory_format=torch.channels_last)
                            or res.dtype != y.dtype):
        raise ValueError("residual must match the output shape / dtype in channels_last")
    for t in (bias,) + (in_affine or ()) + (out_affine or ()):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise ValueError("bias / affine vectors must be contiguous fp32")
    geom = [B, H, W, C, cout, r, s, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], oh, ow]
    mode = (f32_mode or f32_mode_default()) if x.dtype == torch.float32 else None
    dt = F32_MODES[mode] if mode else _DT[x.dtype]
    wptr = wp.data_ptr()
    if w_planes is not None and mode in _PLANES:
        if (w_planes.shape != (_PLANES[mode], cout, r, s, C) or w_planes.dtype != torch.bfloat16
                or not w_planes.is_contiguous()):
            raise ValueError(f"w_planes must be [{_PLANES[mode]}, {cout}, {r}, {s}, {C}] bf16 contiguous")
        dt, wptr = dt + 2, w_planes.data_ptr()
    nn = native.load("_nn")
    # split-K (deep layers with few output tiles): fp32 partial tiles + per-tile arrival counters, allocated
    # stream-ordered from the caching allocator (so concurrent streams and graph capture each get their own).
    # Opt-in (SML_CONV_SPLITK=auto or a split count): r4 measured it slower on every ResNet-50 layer it took
    # (profiles/r4/conv: the partial tiles' agent-scope release per block costs more than the fuller grid).
    sk, ws_floats, n_cnt = (nn.conv_split_plan(geom, dt, in_affine is not None, int(kernel)) if _SPLITK
                            else (1, 0, 0))
    ws = cnt = None
    if sk > 1:
        ws = torch.empty(ws_floats, device=x.device, dtype=torch.float32)
        cnt = torch.zeros(n_cnt, device=x.device, dtype=torch.int32)
    nn.conv_mfma(
        x.data_ptr(), wptr, y.data_ptr(), _ptr(in_affine[0] if in_affine else None),
        _ptr(in_affine[1] if in_affine else None), _ptr(bias), _ptr(res), _ptr(out_affine[0] if out_affine else None),
        _ptr(out_affine[1] if out_affine else None), _ptr(y2), geom, int(relu), int(in_relu), dt,
        torch.cuda.current_stream(x.device).cuda_stream, int(kernel), int(sk), _ptr(ws), _ptr(cnt))
    return (y, y2) if out_affine is not None else y


STEM_KP = 160  # padded K of the stem kernel (csrc/nn/conv_mfma.hip stem_conv_kernel)


def stem_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    """The dedicated few-channel stem kernel takes f16/bf16 NHWC inputs with C <= 4, R, S <= 8 and
    R * S * C <= 160."""
    return (x.is_cuda and x.dtype in (torch.float16, torch.bfloat16) and w.dim() == 4 and 1 <= x.shape[1] <= 4
            and w.shape[1] == x.shape[1] and w.shape[2] <= 8 and w.shape[3] <= 8
            and w.shape[1] * w.shape[2] * w.shape[3] <= STEM_KP)


STEM_WIDE_KP, STEM_WIDE_RP = 192, 24  # the row-run stem form (C = 3, S * 3 <= 24, R <= 8)
# SML_STEM_ROWRUN=1 makes the row-run form the default for 3-channel stems. Off: r4 pass 11 measured it at
# 426 us per ResNet-50 batch of 128 against 330 us for the 2-byte gathers - the texture path moves ~4 B per
# clock per CU for these scattered accesses whatever the width, and the 64-B windows fetch 1.5x the bytes.
_STEM_ROWRUN = os.environ.get("SML_STEM_ROWRUN", "0") == "1"


def stem_wide(w: torch.Tensor) -> bool:
    """Whether a stem weight fits the row-run kernel (C = 3, S * 3 <= 24, R <= 8): each (pixel, filter row)
    run of S * 3 input values fetched as aligned 16-B chunks instead of 2-byte gathers."""
    return w.shape[1] == 3 and w.shape[3] * 3 <= STEM_WIDE_RP and w.shape[2] <= 8


def pack_stem_weight(w: torch.Tensor, wide: Optional[bool] = None) -> torch.Tensor:
    """[Cout, C, R, S] -> [Cout, 160] with k = (r * S + s) * C + c, zero-padded; for the row-run form
    (``stem_wide``) [Cout, 192] with k = r * 24 + s * 3 + c, zero in every slot s * 3 + c >= S * 3 and past
    R * 24 (packed once per weight)."""
    cout = w.shape[0]
    if wide is None:
        wide = _STEM_ROWRUN and stem_wide(w)
    if wide:
        if not stem_wide(w):
            raise ValueError("row-run stem packing: C = 3, S * 3 <= 24, R <= 8")
        R, S = w.shape[2], w.shape[3]
        out = torch.zeros((cout, R, STEM_WIDE_RP), dtype=w.dtype, device=w.device)
        out[:, :, :S * 3] = w.permute(0, 2, 3, 1).reshape(cout, R, S * 3)
        full = torch.zeros((cout, STEM_WIDE_KP), dtype=w.dtype, device=w.device)
        full[:, :R * STEM_WIDE_RP] = out.reshape(cout, -1)
        return full
    k = w.permute(0, 2, 3, 1).reshape(cout, -1)
    out = torch.zeros((cout, STEM_KP), dtype=w.dtype, device=w.device)
    out[:, :k.shape[1]] = k
    return out


def stem_f32_supported(x: torch.Tensor, w: torch.Tensor, stride=(1, 1), pad=(0, 0), dil=(1, 1),
                       mode: str = "bf16x3") -> bool:
    """The fp32 stem kernel (bf16-plane products, csrc/nn/conv_mfma.hip stem_f32_kernel): fp32 NHWC input with
    3 channels, R <= 8, S <= 7, W % 4 == 0, output rows of <= 128 pixels, no dilation, pad_w <= 8, 16-B
    aligned rows (the row-staged geometry; the native launcher re-checks and refuses other shapes)."""
    if mode not in _PLANES or not (
            x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and w.dim() == 4 and x.shape[1] == 3
            and w.shape[1] == 3 and w.shape[2] <= 8 and w.shape[3] <= 7 and x.shape[3] % 4 == 0
            and tuple(dil) == (1, 1) and pad[1] <= 8 and x.data_ptr() % 16 == 0):
        return False
    H, W = x.shape[2], x.shape[3]
    r, s = w.shape[2], w.shape[3]
    oh, ow = out_hw(H, W, r, s, stride, pad, dil)
    return (0 < ow <= 128 and oh > 0 and (ow - 1) * stride[1] - pad[1] + s <= W + 8
            and _PLANES[mode] * r * (W + 16) * 3 * 2 <= 34 * 1024 and r * (W + 16) * 3 // 4 <= 2048)


def pack_stem_weight_f32(w: torch.Tensor, mode: str = "bf16x3", wide: bool = False) -> torch.Tensor:
    """fp32 [Cout, 3, R, S] -> [planes, Cout, 160] bf16 (pack_stem_weight, then split_weight's RNE planes:
    2 for bf16x3, 3 for bf16x6) - the fp32 stem kernel's weight operand, made once per model; ``wide``: the
    row-run K order [planes, Cout, 192] of the strip form (``stem_ring_ok``)."""
    return split_weight(pack_stem_weight(w.float(), wide=wide), mode)


# SML_STEM_RING=0: the row-staged stem forms instead of the strip form (one block per 8 output rows, input rows
# in an LDS ring, the weights in registers) for the stride-2 RGB stems
_STEM_RING = os.environ.get("SML_STEM_RING", "1") != "0"


def stem_ring_ok(x: torch.Tensor, w: torch.Tensor, stride=(1, 1), pad=(0, 0), dil=(1, 1), planes: int = 1) -> bool:
    """Whether the strip form of the stem (csrc/nn/conv_mfma.hip stem_ring_kernel, mirrors RingOk) takes this
    conv: 3 channels, an even horizontal stride <= 4, R <= 8, S * 3 <= 24, pad_w <= 8, no dilation, output
    rows of <= 128 pixels, 16-B aligned input rows and its LDS ring within 44 KB."""
    if not _STEM_RING or x.dim() != 4 or w.dim() != 4 or x.shape[1] != 3 or w.shape[1] != 3:
        return False
    esize = x.element_size()
    epc = 16 // esize
    H, W = x.shape[2], x.shape[3]
    r, s = w.shape[2], w.shape[3]
    sh, sw = stride
    if (sw % 2 or sw > 4 or s * 3 > STEM_WIDE_RP or not 1 <= r <= 8 or not 1 <= sh <= 4 or tuple(dil) != (1, 1)
            or pad[1] > 8 or (W * 3) % epc or x.data_ptr() % 16):
        return False
    oh, ow = out_hw(H, W, r, s, stride, pad, dil)
    cpr = W * 3 // epc
    sp = (max((pad[1] + W) * 3, (ow - 1) * sw * 3 + STEM_WIDE_RP) + 15) // 8 * 8
    return (0 < ow <= 128 and oh > 0 and r * cpr <= 2048 and sh * cpr <= 512
            and (planes * (r + sh) + 1) * sp * 2 <= 44 * 1024)


def stem_conv_nhwc(x: torch.Tensor, wk: torch.Tensor, r: int, s: int, stride=(1, 1), pad=(0, 0), dil=(1, 1),
                   bias: Optional[torch.Tensor] = None, relu: int = 0,
                   res: Optional[torch.Tensor] = None, in_affine=None, in_relu: bool = False,
                   form: int = 0) -> torch.Tensor:
    """y = relu?(conv(x', w) + bias (+ res)) for a few-channel input (the image stem): ``x`` [B, C, H, W]
    channels_last f16/bf16 with C <= 4, ``wk`` = pack_stem_weight(w). ``relu``: 0 none, 1 before the residual
    add, 2 after it. ``pad``: (top, left) or (top, left, bottom, right). ``in_affine`` = (scale, shift) per
    input channel: x' = x * scale + shift (ReLU'd with ``in_relu``) inside the kernel, padding taps 0 - an
    input BatchNormalization without its own pass. ``form`` (160-wide weights): 0 picks the row-staged kernel
    where it applies (3 channels, one block per output row of <= 128 pixels), 1 forces the 2-byte gather
    kernel, 2 the row-staged one; 192-wide weights: 0 picks the strip form (``stem_ring_ok``) where it applies,
    1 forces the row-run kernel, 3 the strip form. fp32 ``x``: ``wk`` = pack_stem_weight_f32(w, mode), the bf16-plane kernel
    (2 planes: 3 products per pair, 3 planes: 6), 3 channels and the row-staged geometry only (192-wide planes:
    the strip form)."""
    B, C, H, W = x.shape
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    if x.dtype == torch.float32:
        if wk.dim() != 3 or wk.shape[0] not in (2, 3) or wk.shape[2] not in (STEM_KP, STEM_WIDE_KP) \
                or wk.dtype != torch.bfloat16 \
                or not wk.is_contiguous():
            raise ValueError("fp32 stem weight must be pack_stem_weight_f32(w, mode)")
        cout = wk.shape[1]
        dt = 3 if wk.shape[0] == 2 else 4
    elif wk.dim() != 2 or wk.shape[1] not in (STEM_KP, STEM_WIDE_KP) or wk.dtype != x.dtype or not wk.is_contiguous():
        raise ValueError("stem weight must be pack_stem_weight(w) in the input dtype")
    else:
        cout = wk.shape[0]
        dt = _DT[x.dtype]
    if wk.shape[-1] == STEM_WIDE_KP and (C != 3 or s * 3 > STEM_WIDE_RP or r > 8):
        raise ValueError("row-run stem weight for a different filter shape")
    if C * r * s > STEM_KP or C > 4:
        raise ValueError("stem kernel: C <= 4 and R * S * C <= 160")
    oh, ow = out_hw(H, W, r, s, stride, pad, dil)
    y = torch.empty((B, cout, oh, ow), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    if res is not None:
        res = res.to(x.dtype).contiguous(memory_format=torch.channels_last)
    b32 = None if bias is None else bias.reshape(-1).to(x.device, torch.float32).contiguous()
    geom = [B, H, W, C, cout, r, s, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], oh, ow]
    sc = sh = None
    if in_affine is not None:
        sc = in_affine[0].reshape(-1).to(x.device, torch.float32).contiguous()
        sh = in_affine[1].reshape(-1).to(x.device, torch.float32).contiguous()
        if sc.numel() != C or sh.numel() != C:
            raise ValueError("stem in_affine: one scale / shift per input channel")
    native.load("_nn").stem_conv(x.data_ptr(), wk.data_ptr(), y.data_ptr(), _ptr(b32), _ptr(res), geom, int(relu),
                                 dt, torch.cuda.current_stream(x.device).cuda_stream, _ptr(sc), _ptr(sh),
                                 int(bool(in_relu)), int(wk.shape[-1]), int(form))
    return y


__all__ = ["supported", "pack_weight", "split_weight", "conv2d_nhwc", "out_hw", "F32_MODES", "stem_supported",
           "pack_stem_weight", "stem_conv_nhwc", "stem_wide", "stem_f32_supported", "pack_stem_weight_f32",
           "stem_ring_ok"]


def conv2d_nhwc_general(x: torch.Tensor, wp: torch.Tensor, r: int, s: int, stride=(1, 1), pad=(0, 0, 0, 0),
                        dil=(1, 1), groups: int = 1, bias: Optional[torch.Tensor] = None, relu: int = 0,
                        res: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Convolutions the tiled implicit-GEMM kernel does not take: any channel count (the 3-channel stem,
    C % 64 != 0) and grouped / depthwise layers. ``x`` [B, C, H, W] channels_last, ``wp`` packed
    [Cout, R, S, C / groups]. groups == 1, or groups whose per-group GEMM is at least 16 wide: the MFMA
    GEMM with an implicit-im2col A operand (one batch entry per group); otherwise (depthwise, narrow
    groups) the direct NHWC kernel. ``relu``: 0 none, 1 before the residual add, 2 after it."""
    B, C, H, W = x.shape
    cout = wp.shape[0]
    cg, ng = C // groups, cout // groups
    if wp.shape != (cout, r, s, cg) or not wp.is_contiguous() or wp.dtype != x.dtype:
        raise ValueError(f"packed weight must be [Cout, {r}, {s}, {cg}] {x.dtype}")
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    oh, ow = out_hw(H, W, r, s, stride, pad, dil)
    y = torch.empty((B, cout, oh, ow), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    if res is not None:
        res = res.to(x.dtype).contiguous(memory_format=torch.channels_last)
    b32 = None if bias is None else bias.reshape(-1).to(x.device, torch.float32).contiguous()
    nn = native.load("_nn")
    stream = torch.cuda.current_stream(x.device).cuda_stream
    K = r * s * cg
    if groups == 1 or (ng >= 16 and K >= 16):
        M = B * oh * ow
        # the GEMM epilogue adds the residual before its ReLU: relu=1 with a residual adds it afterwards
        act = 1 if relu else 0
        cm = None if (relu == 1 and res is not None) else res
        nn.gemm(x.data_ptr(), wp.data_ptr(), y.data_ptr(), M, ng, K, groups, 0, K, cout, cg, ng * K, ng, 0, 1, 1.0, 1.0,
                _ptr(b32), _ptr(cm), cout, ng, act, _DT[x.dtype], stream,
                [H, W, C, r, s, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], oh, ow], ng)
        if res is not None and cm is None:  # relu before the residual add (rare): add it after
            y.add_(res)
        return y
    nn.group_conv(x.data_ptr(), wp.data_ptr(), y.data_ptr(), _ptr(b32), _ptr(res),
                  [B, H, W, C, cout, r, s, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], oh, ow],
                  groups, int(relu), _DT[x.dtype], stream)
    return y
