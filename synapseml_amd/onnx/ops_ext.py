"""More of the ONNX operator set for arbitrary graphs (the reference runs any model through ONNX Runtime:
deep-learning/.../onnx/ONNXModel.scala:36-106, ONNXRuntime.scala:58-107):

* control flow: Loop, Scan (bodies run as cached sub-sessions, outer-scope values visible)
* sequences: SequenceEmpty / Construct / At / Length / Insert / Erase, ConcatFromSequence, SplitToSequence,
  Optional / OptionalHasElement / OptionalGetElement
* recurrent: LSTM, GRU, RNN (ONNX gate orders, forward / reverse / bidirectional, sequence_lens, peepholes,
  clip, input_forget, linear_before_reset, layout, per-gate activations)
* quantisation: QuantizeLinear, DequantizeLinear, DynamicQuantizeLinear, MatMulInteger, ConvInteger,
  QLinearMatMul, QLinearConv, com.microsoft QLinearAdd / QLinearMul / QLinearSigmoid /
  QLinearLeakyRelu / QLinearGlobalAveragePool (integer products accumulate exactly in fp64)
* tensors: NonZero, Compress, Unique, EyeLike, Shrink, ReverseSequence, MeanVarianceNormalization,
  GroupNormalization, RMSNormalization, Det, CenterCropPad, GridSample, NonMaxSuppression, GlobalLpPool,
  BitwiseAnd / Or / Xor, the window functions, DFT, random generators
* text: StringNormalizer, StringConcat, StringSplit, RegexFullMatch
* ai.onnx.ml: DictVectorizer, FeatureVectorizer, CategoryMapper
* com.microsoft transformer contrib ops emitted by ORT's graph optimizers: FusedMatMul, FastGelu,
  BiasGelu, QuickGelu, SkipLayerNormalization, SimplifiedLayerNormalization,
  SkipSimplifiedLayerNormalization, EmbedLayerNormalization, Attention, MultiHeadAttention

These are graph-coverage ops (the hot paths of the flagship graphs run on the HIP kernels in csrc/nn);
each follows the ONNX / contrib operator specification. Values: torch tensors (device or host), numpy object
arrays for strings, Python lists for sequences, None for empty optionals.
"""
from __future__ import annotations

import math
import re
from typing import List, Optional

import numpy as np
import torch
import torch.nn.functional as Fn

from . import proto as P
from .ops import OPS, TORCH_OF, _ints, _to_np, op

# ops whose outputs' shapes / control flow depend on tensor values (or that read values on the host): a graph
# containing one is run eagerly, never captured into a hipGraph (a host sync inside a capture invalidates it)
HOST_SYNC_OPS = {"Loop", "Scan", "If", "NonZero", "Compress", "Unique", "NonMaxSuppression", "SequenceAt",
                 "SequenceInsert", "SequenceErase", "SplitToSequence", "ReverseSequence", "CenterCropPad",
                 "DynamicQuantizeLinear", "MatMulInteger", "ConvInteger", "QLinearMatMul", "QLinearConv",
                 "LSTM", "GRU", "RNN", "Bernoulli", "Multinomial", "RandomNormal", "RandomUniform",
                 "RandomNormalLike", "RandomUniformLike", "StringNormalizer", "StringConcat", "StringSplit",
                 "RegexFullMatch", "CategoryMapper", "DictVectorizer", "FeatureVectorizer",
                 # ai.onnx.ml ops evaluated on the host (numpy maps / dicts): a capture would record nothing
                 "ZipMap", "LabelEncoder", "OneHotEncoder", "TfIdfVectorizer"}


def _t(v, device=None, dtype=None) -> torch.Tensor:
    if isinstance(v, torch.Tensor):
        t = v
    else:
        a = np.asarray(v)
        t = torch.from_numpy(np.ascontiguousarray(a))
    if device is not None and t.device != torch.device(device):
        t = t.to(device)
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t


def _dev(x):
    for v in x:
        if isinstance(v, torch.Tensor):
            return v.device
    return torch.device("cpu")


def _scalar(v, default=None):
    if v is None:
        return default
    return _to_np(v).reshape(-1)[0].item()


# ------------------------------------------------------------------ control flow
@op("Loop")
def _loop(rt, at, x):
    body = at["body"]
    M = _scalar(x[0]) if len(x) > 0 and x[0] is not None else None
    cond = bool(_scalar(x[1])) if len(x) > 1 and x[1] is not None else True
    vs = list(x[2:])
    n_carried = len(vs)
    names = [v.name for v in body.inputs]
    scans: List[list] = []
    i = 0
    while (M is None or i < M) and cond:
        feeds = {names[0]: torch.tensor(i, dtype=torch.int64), names[1]: torch.tensor(cond)}
        for k, v in enumerate(vs):
            feeds[names[2 + k]] = v
        outs = rt.run_subgraph(body, feeds)
        cond = bool(_scalar(outs[0]))
        vs = list(outs[1:1 + n_carried])
        rest = outs[1 + n_carried:]
        if not scans:
            scans = [[] for _ in rest]
        for k, v in enumerate(rest):
            scans[k].append(_t(v))
        i += 1
    n_scan = len(body.outputs) - 1 - n_carried
    res = list(vs)
    for k in range(n_scan):
        res.append(torch.stack(scans[k]) if scans and scans[k] else torch.zeros((0,)))
    return res


@op("Scan")
def _scan(rt, at, x):
    body = at["body"]
    M = int(at["num_scan_inputs"])
    N = len(x) - M
    states = list(x[:N])
    seqs = [_t(v) for v in x[N:]]
    in_axes = list(at.get("scan_input_axes", [0] * M))
    in_dirs = list(at.get("scan_input_directions", [0] * M))
    n_out = len(body.outputs) - N
    out_axes = list(at.get("scan_output_axes", [0] * n_out))
    out_dirs = list(at.get("scan_output_directions", [0] * n_out))
    in_axes = [a + seqs[j].dim() if a < 0 else a for j, a in enumerate(in_axes)]
    T = seqs[0].shape[in_axes[0]] if seqs else 0
    names = [v.name for v in body.inputs]
    outs_t: List[list] = [[] for _ in range(n_out)]
    for t in range(T):
        feeds = {names[k]: states[k] for k in range(N)}
        for j in range(M):
            idx = T - 1 - t if in_dirs[j] else t
            feeds[names[N + j]] = seqs[j].select(in_axes[j], idx)
        outs = rt.run_subgraph(body, feeds)
        states = list(outs[:N])
        for k in range(n_out):
            outs_t[k].append(_t(outs[N + k]))
    res = list(states)
    for k in range(n_out):
        items = outs_t[k][::-1] if out_dirs[k] else outs_t[k]
        st = torch.stack(items) if items else torch.zeros((0,))
        ax = out_axes[k]
        if ax < 0:
            ax += st.dim()
        res.append(st.movedim(0, ax) if items and ax != 0 else st)
    return res


# ------------------------------------------------------------------ sequences / optionals
@op("SequenceEmpty")
def _seq_empty(rt, at, x):
    return [[]]


@op("SequenceConstruct")
def _seq_construct(rt, at, x):
    return [list(x)]


@op("SequenceAt")
def _seq_at(rt, at, x):
    return [x[0][int(_scalar(x[1]))]]


@op("SequenceLength")
def _seq_len(rt, at, x):
    return [torch.tensor(len(x[0]), dtype=torch.int64)]


@op("SequenceInsert")
def _seq_insert(rt, at, x):
    s = list(x[0])
    pos = int(_scalar(x[2])) if len(x) > 2 and x[2] is not None else len(s)
    if pos < 0:
        pos += len(s)
    s.insert(pos, x[1])
    return [s]


@op("SequenceErase")
def _seq_erase(rt, at, x):
    s = list(x[0])
    pos = int(_scalar(x[1])) if len(x) > 1 and x[1] is not None else -1
    del s[pos]
    return [s]


@op("ConcatFromSequence")
def _concat_from_seq(rt, at, x):
    axis = int(at["axis"])
    items = [_t(v) for v in x[0]]
    if int(at.get("new_axis", 0)):
        if axis < 0:
            axis += items[0].dim() + 1
        return [torch.stack(items, axis)]
    return [torch.cat(items, axis)]


@op("SplitToSequence")
def _split_to_seq(rt, at, x):
    t = _t(x[0])
    axis = int(at.get("axis", 0))
    if axis < 0:
        axis += t.dim()
    split = x[1] if len(x) > 1 else None
    if split is None:
        parts = list(torch.split(t, 1, axis))
        if not int(at.get("keepdims", 1)):
            parts = [p.squeeze(axis) for p in parts]
        return [parts]
    sp = _to_np(split).reshape(-1)
    if _to_np(split).ndim == 0:
        return [list(torch.split(t, int(sp[0]), axis))]
    return [list(torch.split(t, [int(v) for v in sp], axis))]


@op("Optional")
def _optional(rt, at, x):
    return [x[0] if x else None]


@op("OptionalHasElement")
def _opt_has(rt, at, x):
    return [torch.tensor(bool(x) and x[0] is not None)]


@op("OptionalGetElement")
def _opt_get(rt, at, x):
    if x[0] is None:
        raise ValueError("OptionalGetElement on an empty optional")
    return [x[0]]


# ------------------------------------------------------------------ recurrent layers
def _act(name: str, alpha: Optional[float], beta: Optional[float]):
    n = name.lower()
    if n == "sigmoid":
        return torch.sigmoid
    if n == "tanh":
        return torch.tanh
    if n == "relu":
        return torch.relu
    if n == "affine":
        return lambda v: (alpha if alpha is not None else 1.0) * v + (beta or 0.0)
    if n == "leakyrelu":
        return lambda v: Fn.leaky_relu(v, alpha if alpha is not None else 0.01)
    if n == "thresholdedrelu":
        a = alpha if alpha is not None else 1.0
        return lambda v: torch.where(v > a, v, torch.zeros_like(v))
    if n == "scaledtanh":
        return lambda v: (alpha if alpha is not None else 1.0) * torch.tanh((beta if beta is not None else 1.0) * v)
    if n == "hardsigmoid":
        a, b = (alpha if alpha is not None else 0.2), (beta if beta is not None else 0.5)
        return lambda v: torch.clamp(a * v + b, 0.0, 1.0)
    if n == "elu":
        return lambda v: Fn.elu(v, alpha if alpha is not None else 1.0)
    if n == "softsign":
        return lambda v: v / (1 + v.abs())
    if n == "softplus":
        return Fn.softplus
    raise NotImplementedError(f"RNN activation {name}")


def _acts(at, defaults: List[str], num_dir: int):
    names = [a.decode() if isinstance(a, bytes) else a for a in at.get("activations", [])] or defaults * num_dir
    alphas = list(at.get("activation_alpha", []))
    betas = list(at.get("activation_beta", []))
    out, ai, bi = [], 0, 0
    for nm in names:
        n = nm.lower()
        takes_a = n in ("affine", "leakyrelu", "thresholdedrelu", "scaledtanh", "hardsigmoid", "elu")
        takes_b = n in ("affine", "scaledtanh", "hardsigmoid")
        a = alphas[ai] if takes_a and ai < len(alphas) else None
        b = betas[bi] if takes_b and bi < len(betas) else None
        ai += 1 if takes_a and ai < len(alphas) else 0
        bi += 1 if takes_b and bi < len(betas) else 0
        out.append(_act(nm, a, b))
    k = len(defaults)
    return [out[d * k:(d + 1) * k] for d in range(num_dir)]


def _rnn_common(at, x, gates: int):
    layout = int(at.get("layout", 0))
    X = _t(x[0])
    if layout:
        X = X.transpose(0, 1)  # -> [seq, batch, input]
    dt = X.dtype if X.is_floating_point() else torch.float32
    X = X.to(dt)
    dev = X.device
    W = _t(x[1], dev, dt)
    R = _t(x[2], dev, dt)
    nd, H = W.shape[0], W.shape[1] // gates
    B = _t(x[3], dev, dt) if len(x) > 3 and x[3] is not None else torch.zeros(nd, 2 * gates * H, device=dev, dtype=dt)
    T, N = X.shape[0], X.shape[1]
    lens = (_to_np(x[4]).astype(np.int64) if len(x) > 4 and x[4] is not None else np.full(N, T, np.int64))
    # (sequence_lens is read on the host once per call: the op sits in HOST_SYNC_OPS when it is an input)
    direction = at.get("direction", "forward")
    direction = direction.decode() if isinstance(direction, bytes) else direction
    if nd == 2 and direction != "bidirectional":
        direction = "bidirectional"
    clip = at.get("clip")
    return layout, X, W, R, B, nd, H, T, N, lens, direction, clip, dev, dt


def _rnn_outputs(rt, at, layout, Y, finals, n_states):
    outs = [Y.permute(2, 0, 1, 3) if layout else Y]
    for k in range(n_states):
        s = torch.stack([f[k] for f in finals])
        outs.append(s.transpose(0, 1) if layout else s)
    return outs[:max(1, rt.node_num_outputs)]


def _init_state(x, i, nd, N, H, dev, dt, layout):
    if len(x) > i and x[i] is not None:
        s = _t(x[i], dev, dt)
        return s.transpose(0, 1) if layout else s
    return torch.zeros(nd, N, H, device=dev, dtype=dt)


@op("LSTM")
def _lstm(rt, at, x):
    layout, X, W, R, B, nd, H, T, N, lens, direction, clip, dev, dt = _rnn_common(at, x, 4)
    h0 = _init_state(x, 5, nd, N, H, dev, dt, layout)
    c0 = _init_state(x, 6, nd, N, H, dev, dt, layout)
    Pp = _t(x[7], dev, dt) if len(x) > 7 and x[7] is not None else torch.zeros(nd, 3 * H, device=dev, dtype=dt)
    acts = _acts(at, ["Sigmoid", "Tanh", "Tanh"], nd)
    coupled = int(at.get("input_forget", 0))
    XW = [X @ W[d].t() + B[d, :4 * H] + B[d, 4 * H:] for d in range(nd)]  # [T, N, 4H]: gates i, o, f, c

    def step(d, xt, st):
        h, c = st
        f_, g_, h_ = acts[d]
        z = xt + h @ R[d].t()
        if clip is not None:
            z = z.clamp(-clip, clip)
        zi, zo, zf, zc = z.split(H, -1)
        pi, po, pf = Pp[d].split(H)
        i = f_(zi + pi * c)
        f = 1 - i if coupled else f_(zf + pf * c)
        cc = g_(zc)
        c_new = f * c + i * cc
        o = f_(zo + po * c_new)
        return [o * h_(c_new), c_new]

    Y, finals = _run_lstm(step, XW, nd, direction, T, N, H, lens, [h0, c0], dev, dt)
    return _rnn_outputs(rt, at, layout, Y, finals, 2)


def _run_lstm(step, XW, nd, direction, T, N, H, lens, init, dev, dt):
    """time loop of every direction over the precomputed input projections XW[d] [T, N, G]; each batch item
    walks its own valid prefix (backwards for the reverse direction) and keeps its state past its length.
    Returns Y [T, nd, N, H] (zeros past each length) and the final states per direction."""
    proj = torch.stack(XW, 0)  # [nd, T, N, G]

    Y = torch.zeros(T, nd, N, H, device=dev, dtype=dt)
    finals = []
    lens_t = torch.as_tensor(lens, device=dev)
    ar = torch.arange(N, device=dev)
    for d in range(nd):
        rev = direction == "reverse" or (direction == "bidirectional" and d == 1)
        st = [s[d].clone() for s in init]
        for stp in range(T):
            tt = (lens_t - 1 - stp) if rev else torch.full((N,), stp, device=dev, dtype=torch.long)
            valid = (tt >= 0) & (tt < lens_t)  # all-false steps are masked no-ops: no host sync in the loop
            ti = tt.clamp(0, T - 1)
            new = step(d, proj[d][ti, ar], st)
            m = valid.unsqueeze(1)
            st = [torch.where(m, nv, ov) for nv, ov in zip(new, st)]
            Y[ti, d, ar] = torch.where(m, st[0], Y[ti, d, ar])  # one (time, item) cell per item
        finals.append(st)
    return Y, finals


@op("GRU")
def _gru(rt, at, x):
    layout, X, W, R, B, nd, H, T, N, lens, direction, clip, dev, dt = _rnn_common(at, x, 3)
    h0 = _init_state(x, 5, nd, N, H, dev, dt, layout)
    acts = _acts(at, ["Sigmoid", "Tanh"], nd)
    lbr = int(at.get("linear_before_reset", 0))
    XW = [X @ W[d].t() + B[d, :3 * H] for d in range(nd)]  # gates z, r, h (input part + Wb)

    def step(d, xt, st):
        (h,) = st
        f_, g_ = acts[d]
        xz, xr, xh = xt.split(H, -1)
        Rz, Rr, Rh = R[d].split(H, 0)
        Rbz, Rbr, Rbh = B[d, 3 * H:].split(H)
        zpre = xz + h @ Rz.t() + Rbz
        rpre = xr + h @ Rr.t() + Rbr
        if clip is not None:
            zpre, rpre = zpre.clamp(-clip, clip), rpre.clamp(-clip, clip)
        z, r = f_(zpre), f_(rpre)
        if lbr:
            hpre = xh + r * (h @ Rh.t() + Rbh)
        else:
            hpre = xh + (r * h) @ Rh.t() + Rbh
        if clip is not None:
            hpre = hpre.clamp(-clip, clip)
        hh = g_(hpre)
        return [(1 - z) * hh + z * h]

    Y, finals = _run_lstm(step, XW, nd, direction, T, N, H, lens, [h0], dev, dt)
    return _rnn_outputs(rt, at, layout, Y, finals, 1)


@op("RNN")
def _rnn(rt, at, x):
    layout, X, W, R, B, nd, H, T, N, lens, direction, clip, dev, dt = _rnn_common(at, x, 1)
    h0 = _init_state(x, 5, nd, N, H, dev, dt, layout)
    acts = _acts(at, ["Tanh"], nd)
    XW = [X @ W[d].t() + B[d, :H] + B[d, H:] for d in range(nd)]

    def step(d, xt, st):
        (h,) = st
        z = xt + h @ R[d].t()
        if clip is not None:
            z = z.clamp(-clip, clip)
        return [acts[d][0](z)]

    Y, finals = _run_lstm(step, XW, nd, direction, T, N, H, lens, [h0], dev, dt)
    return _rnn_outputs(rt, at, layout, Y, finals, 1)


# ------------------------------------------------------------------ quantisation
_QRANGE = {torch.uint8: (0, 255), torch.int8: (-128, 127), torch.int16: (-32768, 32767),
           torch.int32: (-2 ** 31, 2 ** 31 - 1)}


def _per_axis(v: torch.Tensor, ref: torch.Tensor, axis: int) -> torch.Tensor:
    """broadcast a per-tensor scalar or a per-axis 1-D parameter against `ref`"""
    if v.dim() == 0 or v.numel() == 1:
        return v.reshape(())
    if axis < 0:
        axis += ref.dim()
    shape = [1] * ref.dim()
    shape[axis] = v.numel()
    return v.reshape(shape)


def _quantize(xf: torch.Tensor, scale: torch.Tensor, zp: torch.Tensor, qdtype, axis: int = 1) -> torch.Tensor:
    lo, hi = _QRANGE[qdtype]
    s = _per_axis(scale.to(torch.float64), xf, axis)
    z = _per_axis(zp.to(torch.float64), xf, axis)
    q = torch.round(xf.to(torch.float64) / s) + z  # round half to even
    return q.clamp(lo, hi).to(qdtype)


def _dequantize(q: torch.Tensor, scale: torch.Tensor, zp: Optional[torch.Tensor], axis: int = 1) -> torch.Tensor:
    s = _per_axis(scale.to(torch.float32), q, axis)
    qf = q.to(torch.float32)
    if zp is not None:
        qf = qf - _per_axis(zp.to(torch.float32), q, axis)
    return qf * s


@op("QuantizeLinear")
def _quantize_linear(rt, at, x):
    xf = _t(x[0])
    dev = xf.device
    scale = _t(x[1], dev)
    zp = _t(x[2], dev) if len(x) > 2 and x[2] is not None else None
    qd = zp.dtype if zp is not None else torch.uint8
    if zp is None:
        zp = torch.zeros((), dtype=qd, device=dev)
    return [_quantize(xf, scale, zp, qd, int(at.get("axis", 1)))]


@op("DequantizeLinear")
def _dequantize_linear(rt, at, x):
    q = _t(x[0])
    dev = q.device
    zp = _t(x[2], dev) if len(x) > 2 and x[2] is not None else None
    return [_dequantize(q, _t(x[1], dev), zp, int(at.get("axis", 1)))]


@op("DynamicQuantizeLinear")
def _dyn_quantize(rt, at, x):
    xf = _t(x[0]).to(torch.float32)
    lo = min(0.0, float(xf.min())) if xf.numel() else 0.0
    hi = max(0.0, float(xf.max())) if xf.numel() else 0.0
    scale = (hi - lo) / 255.0 if hi > lo else 1.0
    zp = float(np.clip(np.round(0.0 - lo / scale), 0, 255))
    sc = torch.tensor(scale, dtype=torch.float32, device=xf.device)
    z = torch.tensor(zp, dtype=torch.uint8, device=xf.device)
    return [_quantize(xf, sc, z, torch.uint8), sc, z]


def _int_matmul(a: torch.Tensor, b: torch.Tensor, azp, bzp) -> torch.Tensor:
    """(A - a_zp) @ (B - b_zp), exact (fp64 accumulation of integer products); a_zp per row, b_zp per column"""
    af = a.to(torch.float64)
    bf = b.to(torch.float64)
    if azp is not None:
        az = azp.to(torch.float64)
        af = af - (az.reshape(-1, 1) if az.numel() > 1 else az.reshape(()))
    if bzp is not None:
        bz = bzp.to(torch.float64)
        bf = bf - (bz.reshape(1, -1) if bz.numel() > 1 else bz.reshape(()))
    dev = af.device
    if dev.type != "cpu":  # fp64 GEMM exactness on any backend: run it on the host
        return torch.matmul(af.cpu(), bf.cpu()).to(dev)
    return torch.matmul(af, bf)


@op("MatMulInteger")
def _matmul_integer(rt, at, x):
    a, b = _t(x[0]), _t(x[1])
    b = b.to(a.device)
    azp = _t(x[2], a.device) if len(x) > 2 and x[2] is not None else None
    bzp = _t(x[3], a.device) if len(x) > 3 and x[3] is not None else None
    return [_int_matmul(a, b, azp, bzp).to(torch.int32)]


def _conv_f64(xf, wf, at, bias=None):
    """exact integer convolution in fp64 on the host (inputs already centred on their zero points, so the
    zero padding is the zero point's padding)"""
    from .ops import _sym_pad, conv_args

    nd, strides, dil, pb, pe = conv_args(at, xf.shape, wf.shape)
    dev = xf.device
    xp, pad = _sym_pad(xf.cpu(), pb, pe)
    fn = {1: Fn.conv1d, 2: Fn.conv2d, 3: Fn.conv3d}[nd]
    out = fn(xp, wf.cpu(), None if bias is None else bias.cpu(), stride=strides, padding=pad, dilation=dil,
             groups=at.get("group", 1))
    return out.to(dev)


@op("ConvInteger")
def _conv_integer(rt, at, x):
    xq, w = _t(x[0]), _t(x[1])
    xf = xq.to(torch.float64)
    wf = w.to(torch.float64).to(xf.device)
    if len(x) > 2 and x[2] is not None:
        xf = xf - _t(x[2], xf.device).to(torch.float64).reshape(())
    if len(x) > 3 and x[3] is not None:
        wz = _t(x[3], xf.device).to(torch.float64)
        wf = wf - (wz.reshape([-1] + [1] * (wf.dim() - 1)) if wz.numel() > 1 else wz.reshape(()))
    return [_conv_f64(xf, wf, at).round().to(torch.int32)]


def _requant(acc: torch.Tensor, mult: torch.Tensor, y_scale, y_zp) -> torch.Tensor:
    """int32 accumulator (fp64) x (a_scale * b_scale) / y_scale, round half to even, + y_zp, saturate"""
    ys = _t(y_scale, acc.device).to(torch.float64)
    yz = _t(y_zp, acc.device)
    qd = yz.dtype
    lo, hi = _QRANGE[qd]
    q = torch.round(acc * mult / ys.reshape(())) + yz.to(torch.float64).reshape(())
    return q.clamp(lo, hi).to(qd)


@op("QLinearMatMul")
def _qlinear_matmul(rt, at, x):
    a = _t(x[0])
    dev = a.device
    a_s, a_z, b, b_s, b_z = (_t(v, dev) for v in x[1:6])
    acc = _int_matmul(a, b, a_z, b_z)
    bs = b_s.to(torch.float64)
    mult = a_s.to(torch.float64).reshape(()) * (bs.reshape(1, -1) if bs.numel() > 1 else bs.reshape(()))
    return [_requant(acc, mult, x[6], x[7])]


@op("QLinearConv")
def _qlinear_conv(rt, at, x):
    xq = _t(x[0])
    dev = xq.device
    x_s, x_z, w, w_s, w_z = (_t(v, dev) for v in x[1:6])
    xf = xq.to(torch.float64) - x_z.to(torch.float64).reshape(())
    wf = w.to(torch.float64)
    wz = w_z.to(torch.float64)
    wf = wf - (wz.reshape([-1] + [1] * (wf.dim() - 1)) if wz.numel() > 1 else wz.reshape(()))
    bias = _t(x[8], dev).to(torch.float64) if len(x) > 8 and x[8] is not None else None
    acc = _conv_f64(xf, wf, at, bias)
    ws = w_s.to(torch.float64)
    wsb = ws.reshape([1, -1] + [1] * (acc.dim() - 2)) if ws.numel() > 1 else ws.reshape(())
    return [_requant(acc, x_s.to(torch.float64).reshape(()) * wsb, x[6], x[7])]


def _qbinary(fn):
    def impl(rt, at, x):
        a = _t(x[0])
        dev = a.device
        af = _dequantize(a, _t(x[1], dev), _t(x[2], dev) if x[2] is not None else None)
        b = _t(x[3], dev)
        bf = _dequantize(b, _t(x[4], dev), _t(x[5], dev) if x[5] is not None else None)
        yz = _t(x[7], dev) if len(x) > 7 and x[7] is not None else torch.zeros((), dtype=a.dtype, device=dev)
        return [_quantize(fn(af, bf), _t(x[6], dev), yz, yz.dtype)]

    return impl


OPS["QLinearAdd"] = _qbinary(torch.add)
OPS["QLinearMul"] = _qbinary(torch.mul)


def _qunary(fn):
    def impl(rt, at, x):
        a = _t(x[0])
        dev = a.device
        af = _dequantize(a, _t(x[1], dev), _t(x[2], dev) if x[2] is not None else None)
        yz = _t(x[4], dev) if len(x) > 4 and x[4] is not None else torch.zeros((), dtype=a.dtype, device=dev)
        return [_quantize(fn(af, at), _t(x[3], dev), yz, yz.dtype)]

    return impl


OPS["QLinearSigmoid"] = _qunary(lambda v, at: torch.sigmoid(v))
OPS["QLinearLeakyRelu"] = _qunary(lambda v, at: Fn.leaky_relu(v, float(at.get("alpha", 0.01))))
OPS["QLinearGlobalAveragePool"] = _qunary(
    lambda v, at: v.mean(dim=tuple(range(1, v.dim() - 1)) if int(at.get("channels_last", 0))
                         else tuple(range(2, v.dim())), keepdim=True))


# ------------------------------------------------------------------ tensor ops
@op("NonZero")
def _nonzero(rt, at, x):
    t = _t(x[0])
    if t.dim() == 0:
        t = t.reshape(1)
    return [torch.nonzero(t).t().contiguous().to(torch.int64)]


@op("Compress")
def _compress(rt, at, x):
    t = _t(x[0])
    cond = _t(x[1], t.device).to(torch.bool).reshape(-1)
    axis = at.get("axis")
    if axis is None:
        flat = t.reshape(-1)
        return [flat[:cond.numel()][cond[:flat.numel()]]]
    axis = int(axis) % t.dim()
    idx = torch.nonzero(cond[:t.shape[axis]]).reshape(-1)
    return [t.index_select(axis, idx)]


@op("Unique")
def _unique(rt, at, x):
    t = _t(x[0])
    a = t.detach().cpu().numpy()
    axis = at.get("axis")
    srt = int(at.get("sorted", 1))
    if axis is None:
        vals, first, inv, counts = np.unique(a.reshape(-1), return_index=True, return_inverse=True, return_counts=True)
    else:
        vals, first, inv, counts = np.unique(a, axis=int(axis), return_index=True, return_inverse=True,
                                             return_counts=True)
    inv = inv.reshape(-1)
    if not srt:  # order of first occurrence
        order = np.argsort(first, kind="stable")
        rank = np.empty_like(order)
        rank[order] = np.arange(len(order))
        vals = np.take(vals, order, axis=0 if axis is None else int(axis))
        first, counts, inv = first[order], counts[order], rank[inv]
    dev = t.device
    return [torch.from_numpy(np.ascontiguousarray(vals)).to(dev),
            torch.from_numpy(first.astype(np.int64)).to(dev), torch.from_numpy(inv.astype(np.int64)).to(dev),
            torch.from_numpy(counts.astype(np.int64)).to(dev)]


@op("EyeLike")
def _eyelike(rt, at, x):
    t = _t(x[0])
    dt = TORCH_OF[int(at["dtype"])] if "dtype" in at else t.dtype
    r, c = t.shape
    k = int(at.get("k", 0))
    out = torch.zeros(r, c, dtype=dt, device=t.device)
    i = torch.arange(max(0, -k), min(r, c - k), device=t.device)
    if len(i):
        out[i, i + k] = 1
    return [out]


@op("Shrink")
def _shrink(rt, at, x):
    t = _t(x[0])
    lam, bias = float(at.get("lambd", 0.5)), float(at.get("bias", 0.0))
    return [torch.where(t < -lam, t + bias, torch.where(t > lam, t - bias, torch.zeros_like(t))).to(t.dtype)]


@op("ReverseSequence")
def _reverse_sequence(rt, at, x):
    t = _t(x[0])
    lens = _to_np(x[1]).astype(np.int64)
    ba, ta = int(at.get("batch_axis", 1)), int(at.get("time_axis", 0))
    out = t.clone()
    for b, L in enumerate(lens):
        if L <= 1:
            continue
        src = t.select(ba, b)
        ta_ = ta if ta < ba else ta - 1
        seg = src.narrow(ta_, 0, int(L)).flip(ta_)
        out.select(ba, b).narrow(ta_, 0, int(L)).copy_(seg)
    return [out]


@op("MeanVarianceNormalization")
def _mvn(rt, at, x):
    t = _t(x[0])
    axes = tuple(at.get("axes", [0, 2, 3]))
    mean = t.mean(dim=axes, keepdim=True)
    var = (t * t).mean(dim=axes, keepdim=True) - mean * mean
    return [(t - mean) / (torch.sqrt(var) + 1e-9)]


@op("GroupNormalization")
def _group_norm(rt, at, x):
    t = _t(x[0])
    dev = t.device
    G = int(at["num_groups"])
    eps = float(at.get("epsilon", 1e-5))
    N, C = t.shape[0], t.shape[1]
    g = t.reshape(N, G, -1).to(torch.float32)
    mean = g.mean(-1, keepdim=True)
    var = g.var(-1, unbiased=False, keepdim=True)
    y = ((g - mean) / torch.sqrt(var + eps)).reshape(t.shape)
    sc, bi = _t(x[1], dev, torch.float32), _t(x[2], dev, torch.float32)
    if sc.numel() == G and G != C:  # opset 18: per-group scale / bias
        sc = sc.repeat_interleave(C // G)
        bi = bi.repeat_interleave(C // G)
    shape = [1, C] + [1] * (t.dim() - 2)
    return [(y * sc.reshape(shape) + bi.reshape(shape)).to(t.dtype)]


def _rms(t: torch.Tensor, scale, axis: int, eps: float):
    axis = axis % t.dim()
    dims = tuple(range(axis, t.dim()))
    tf = t.to(torch.float32)
    inv = torch.rsqrt((tf * tf).mean(dim=dims, keepdim=True) + eps)
    y = tf * inv
    if scale is not None:
        y = y * _t(scale, t.device, torch.float32)
    return y.to(t.dtype), inv


@op("RMSNormalization", "SimplifiedLayerNormalization")
def _rmsnorm(rt, at, x):
    y, inv = _rms(_t(x[0]), x[1] if len(x) > 1 else None, int(at.get("axis", -1)), float(at.get("epsilon", 1e-5)))
    return [y, inv][:max(1, rt.node_num_outputs)]


@op("Det")
def _det(rt, at, x):
    t = _t(x[0])
    return [torch.linalg.det(t.to(torch.float64)).to(t.dtype)]


@op("CenterCropPad")
def _center_crop_pad(rt, at, x):
    t = _t(x[0])
    shape = _ints(x[1])
    axes = at.get("axes") or list(range(t.dim()))
    axes = [a % t.dim() for a in axes]
    for a, target in zip(axes, shape):
        size = t.shape[a]
        if target < size:
            t = t.narrow(a, (size - target) // 2, target)
        elif target > size:
            before = (target - size) // 2
            pad_shape = list(t.shape)
            pad_shape[a] = target
            out = torch.zeros(pad_shape, dtype=t.dtype, device=t.device)
            out.narrow(a, before, size).copy_(t)
            t = out
    return [t]


@op("GridSample")
def _grid_sample(rt, at, x):
    t = _t(x[0])
    grid = _t(x[1], t.device, t.dtype if t.is_floating_point() else torch.float32)
    mode = at.get("mode", "linear")
    mode = mode.decode() if isinstance(mode, bytes) else mode
    mode = {"linear": "bilinear", "bilinear": "bilinear", "nearest": "nearest", "cubic": "bicubic",
            "bicubic": "bicubic"}[mode]
    pm = at.get("padding_mode", "zeros")
    pm = pm.decode() if isinstance(pm, bytes) else pm
    return [Fn.grid_sample(t.to(grid.dtype), grid, mode=mode, padding_mode=pm,
                           align_corners=bool(int(at.get("align_corners", 0)))).to(t.dtype)]


@op("NonMaxSuppression")
def _nms(rt, at, x):
    boxes = _to_np(x[0]).astype(np.float64)
    scores = _to_np(x[1]).astype(np.float64)
    max_out = int(_scalar(x[2], 0)) if len(x) > 2 and x[2] is not None else 0
    iou_thr = float(_scalar(x[3], 0.0)) if len(x) > 3 and x[3] is not None else 0.0
    score_thr = float(_scalar(x[4])) if len(x) > 4 and x[4] is not None else None
    center = int(at.get("center_point_box", 0))
    sel = []
    if max_out > 0:
        for b in range(scores.shape[0]):
            bx = boxes[b]
            if center:
                xc, yc, w, h = bx[:, 0], bx[:, 1], bx[:, 2], bx[:, 3]
                y1, x1, y2, x2 = yc - h / 2, xc - w / 2, yc + h / 2, xc + w / 2
            else:
                y1 = np.minimum(bx[:, 0], bx[:, 2]); y2 = np.maximum(bx[:, 0], bx[:, 2])
                x1 = np.minimum(bx[:, 1], bx[:, 3]); x2 = np.maximum(bx[:, 1], bx[:, 3])
            area = (y2 - y1) * (x2 - x1)
            for c in range(scores.shape[1]):
                s = scores[b, c]
                cand = np.argsort(-s, kind="stable")
                if score_thr is not None:
                    cand = cand[s[cand] > score_thr]
                kept = []
                for i in cand:
                    if len(kept) >= max_out:
                        break
                    ok = True
                    for j in kept:
                        ih = max(0.0, min(y2[i], y2[j]) - max(y1[i], y1[j]))
                        iw = max(0.0, min(x2[i], x2[j]) - max(x1[i], x1[j]))
                        inter = ih * iw
                        union = area[i] + area[j] - inter
                        if union > 0 and inter / union > iou_thr:
                            ok = False
                            break
                    if ok:
                        kept.append(int(i))
                sel += [[b, c, i] for i in kept]
    return [torch.tensor(sel, dtype=torch.int64).reshape(-1, 3)]


@op("GlobalLpPool")
def _global_lp_pool(rt, at, x):
    t = _t(x[0])
    p = float(at.get("p", 2))
    dims = tuple(range(2, t.dim()))
    return [(t.abs() ** p).sum(dim=dims, keepdim=True) ** (1.0 / p)]


def _bitwise(fn):
    return lambda rt, at, x: [fn(_t(x[0]), _t(x[1], _dev(x)))]


OPS["BitwiseAnd"] = _bitwise(torch.bitwise_and)
OPS["BitwiseOr"] = _bitwise(torch.bitwise_or)
OPS["BitwiseXor"] = _bitwise(torch.bitwise_xor)


def _window(kind: str):
    def impl(rt, at, x):
        n = int(_scalar(x[0]))
        periodic = int(at.get("periodic", 1))
        N = n if periodic else n - 1
        k = np.arange(n, dtype=np.float64)
        if kind == "hann":
            w = 0.5 - 0.5 * np.cos(2 * np.pi * k / N)
        elif kind == "hamming":
            w = 25.0 / 46.0 - (21.0 / 46.0) * np.cos(2 * np.pi * k / N)
        else:
            w = 0.42 - 0.5 * np.cos(2 * np.pi * k / N) + 0.08 * np.cos(4 * np.pi * k / N)
        dt = TORCH_OF[int(at.get("output_datatype", P.FLOAT32))]
        return [torch.from_numpy(w).to(dt)]

    return impl


OPS["HannWindow"] = _window("hann")
OPS["HammingWindow"] = _window("hamming")
OPS["BlackmanWindow"] = _window("blackman")


@op("DFT")
def _dft(rt, at, x):
    t = _t(x[0])
    opset = rt.opset.get("", 17) if isinstance(rt.opset, dict) else 17
    if opset >= 20:
        axis = int(_scalar(x[2], -2)) if len(x) > 2 and x[2] is not None else -2
    else:
        axis = int(at.get("axis", 1))
    axis = axis % t.dim()
    n = int(_scalar(x[1])) if len(x) > 1 and x[1] is not None else None
    comp = torch.complex(t[..., 0], t[..., 1]) if t.shape[-1] == 2 else t[..., 0].to(torch.complex64)
    comp = comp.to(torch.complex128 if t.dtype == torch.float64 else torch.complex64)
    inverse, onesided = int(at.get("inverse", 0)), int(at.get("onesided", 0))
    y = torch.fft.ifft(comp, n=n, dim=axis) if inverse else torch.fft.fft(comp, n=n, dim=axis)
    if onesided:
        y = y.narrow(axis, 0, y.shape[axis] // 2 + 1)
    return [torch.stack([y.real, y.imag], -1).to(t.dtype)]


def _rng(at):
    g = torch.Generator()
    if "seed" in at:
        g.manual_seed(int(float(at["seed"]) * 1000003) & 0x7FFFFFFF)
    else:
        g.seed()
    return g


def _random(kind: str, like: bool):
    def impl(rt, at, x):
        if like:
            ref = _t(x[0])
            shape, dt = list(ref.shape), TORCH_OF[int(at["dtype"])] if "dtype" in at else ref.dtype
        else:
            shape, dt = list(at["shape"]), TORCH_OF[int(at.get("dtype", P.FLOAT32))]
        g = _rng(at)
        if kind == "normal":
            v = torch.randn(shape, generator=g, dtype=torch.float64) * float(at.get("scale", 1.0)) + float(at.get("mean", 0.0))
        else:
            lo, hi = float(at.get("low", 0.0)), float(at.get("high", 1.0))
            v = torch.rand(shape, generator=g, dtype=torch.float64) * (hi - lo) + lo
        return [v.to(dt).to(rt.device)]

    return impl


OPS["RandomNormal"] = _random("normal", False)
OPS["RandomUniform"] = _random("uniform", False)
OPS["RandomNormalLike"] = _random("normal", True)
OPS["RandomUniformLike"] = _random("uniform", True)


@op("Bernoulli")
def _bernoulli(rt, at, x):
    p = _t(x[0])
    dt = TORCH_OF[int(at["dtype"])] if "dtype" in at else p.dtype
    v = torch.bernoulli(p.detach().cpu().to(torch.float64), generator=_rng(at))
    return [v.to(dt).to(p.device)]


@op("Multinomial")
def _multinomial(rt, at, x):
    logits = _t(x[0]).detach().cpu().to(torch.float64)
    n = int(at.get("sample_size", 1))
    dt = TORCH_OF[int(at.get("dtype", P.INT32))]
    probs = torch.softmax(logits, -1)
    return [torch.multinomial(probs, n, replacement=True, generator=_rng(at)).to(dt).to(rt.device)]


# ------------------------------------------------------------------ strings
def _strs(v) -> np.ndarray:
    a = np.asarray(v, dtype=object)
    return np.vectorize(lambda s: s.decode("utf-8") if isinstance(s, bytes) else str(s), otypes=[object])(a) \
        if a.size else a


@op("StringNormalizer")
def _string_normalizer(rt, at, x):
    a = _strs(x[0])
    action = at.get("case_change_action", "NONE")
    action = action.decode() if isinstance(action, bytes) else action
    sens = int(at.get("is_case_sensitive", 0))
    stop = [s.decode() if isinstance(s, bytes) else s for s in at.get("stopwords", [])]
    stop_set = set(stop) if sens else {s.lower() for s in stop}
    shape = a.shape
    rows = a.reshape(-1, shape[-1]) if a.ndim == 2 else a.reshape(1, -1)
    out_rows = []
    for r in rows:
        keep = [s for s in r if (s if sens else s.lower()) not in stop_set]
        if action == "LOWER":
            keep = [s.lower() for s in keep]
        elif action == "UPPER":
            keep = [s.upper() for s in keep]
        out_rows.append(keep)
    width = max((len(k) for k in out_rows), default=0)
    if width == 0:
        return [np.array([[""]] if a.ndim == 2 else [""], dtype=object)]
    res = np.array([k + [""] * (width - len(k)) for k in out_rows], dtype=object)
    return [res if a.ndim == 2 else res.reshape(-1)]


@op("StringConcat")
def _string_concat(rt, at, x):
    a, b = _strs(x[0]), _strs(x[1])
    return [np.vectorize(lambda u, v: u + v, otypes=[object])(a, b)]


@op("RegexFullMatch")
def _regex_full_match(rt, at, x):
    pat = at["pattern"]
    rx = re.compile(pat.decode() if isinstance(pat, bytes) else pat)
    a = _strs(x[0])
    return [torch.from_numpy(np.vectorize(lambda s: rx.fullmatch(s) is not None, otypes=[bool])(a)
                             if a.size else np.zeros(a.shape, bool))]


@op("StringSplit")
def _string_split(rt, at, x):
    a = _strs(x[0])
    d = at.get("delimiter")
    d = (d.decode() if isinstance(d, bytes) else d) or None
    maxsplit = int(at.get("maxsplit", -1)) if "maxsplit" in at else -1
    parts = [s.split(d, maxsplit) if d else s.split(None, maxsplit) for s in a.reshape(-1)]
    width = max((len(p) for p in parts), default=0)
    out = np.array([p + [""] * (width - len(p)) for p in parts], dtype=object).reshape(a.shape + (width,))
    counts = np.array([len(p) for p in parts], dtype=np.int64).reshape(a.shape)
    return [out, torch.from_numpy(counts)]


# ------------------------------------------------------------------ ai.onnx.ml
@op("DictVectorizer")
def _dict_vectorizer(rt, at, x):
    vocab = at.get("string_vocabulary") or at.get("int64_vocabulary") or []
    vocab = [v.decode() if isinstance(v, bytes) else v for v in vocab]
    pos = {v: i for i, v in enumerate(vocab)}
    maps = x[0] if isinstance(x[0], (list, tuple)) else [x[0]]
    out = np.zeros((len(maps), len(vocab)), dtype=np.float32)
    for r, m in enumerate(maps):
        for k, v in m.items():
            k = k.decode() if isinstance(k, bytes) else k
            j = pos.get(k)
            if j is not None:
                out[r, j] = float(v)
    return [torch.from_numpy(out)]


@op("FeatureVectorizer")
def _feature_vectorizer(rt, at, x):
    dims = list(at.get("inputdimensions", []))
    cols = []
    for i, v in enumerate(x):
        t = _t(v).to(torch.float32)
        t = t.reshape(t.shape[0], -1) if t.dim() > 1 else t.reshape(1, -1)
        d = dims[i] if i < len(dims) else t.shape[1]
        if t.shape[1] < d:
            t = Fn.pad(t, (0, d - t.shape[1]))
        cols.append(t[:, :d].cpu())
    return [torch.cat(cols, 1)]


@op("CategoryMapper")
def _category_mapper(rt, at, x):
    ints = [int(v) for v in at.get("cats_int64s", [])]
    strs = [v.decode() if isinstance(v, bytes) else v for v in at.get("cats_strings", [])]
    dint = int(at.get("default_int64", -1))
    dstr = at.get("default_string", "_Unused")
    dstr = dstr.decode() if isinstance(dstr, bytes) else dstr
    v = x[0]
    if isinstance(v, np.ndarray) and v.dtype == object:
        m = dict(zip(strs, ints))
        return [torch.from_numpy(np.vectorize(lambda s: m.get(s.decode() if isinstance(s, bytes) else s, dint),
                                              otypes=[np.int64])(v) if v.size else np.zeros(v.shape, np.int64))]
    m = dict(zip(ints, strs))
    a = _to_np(v)
    return [np.vectorize(lambda i: m.get(int(i), dstr), otypes=[object])(a) if a.size else a.astype(object)]


# ------------------------------------------------------------------ com.microsoft transformer contrib ops
def _gelu_tanh(v):
    return 0.5 * v * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (v + 0.044715 * v * v * v)))


@op("FusedMatMul")
def _fused_matmul(rt, at, x):
    a, b = _t(x[0]), _t(x[1], _dev(x))
    if int(at.get("transBatchA", 0)) and a.dim() > 2:
        a = a.movedim(0, -2)
    if int(at.get("transBatchB", 0)) and b.dim() > 2:
        b = b.movedim(0, -2)
    if int(at.get("transA", 0)):
        a = a.transpose(-1, -2)
    if int(at.get("transB", 0)):
        b = b.transpose(-1, -2)
    return [float(at.get("alpha", 1.0)) * torch.matmul(a, b.to(a.dtype))]


@op("FastGelu")
def _fast_gelu(rt, at, x):
    v = _t(x[0])
    if len(x) > 1 and x[1] is not None:
        v = v + _t(x[1], v.device, v.dtype)
    return [_gelu_tanh(v)]


@op("BiasGelu")
def _bias_gelu(rt, at, x):
    v = _t(x[0]) + _t(x[1], _dev(x))
    return [Fn.gelu(v)]


@op("QuickGelu")
def _quick_gelu(rt, at, x):
    v = _t(x[0])
    return [v * torch.sigmoid(float(at.get("alpha", 1.702)) * v)]


def _skip_sum(x):
    s = _t(x[0])
    s = s + _t(x[1], s.device, s.dtype)
    bias = x[4] if len(x) > 4 else None
    if bias is not None:
        s = s + _t(bias, s.device, s.dtype)
    return s


@op("SkipLayerNormalization")
def _skip_ln(rt, at, x):
    s = _skip_sum(x)
    eps = float(at.get("epsilon", 1e-12))
    sf = s.to(torch.float32)
    mean = sf.mean(-1, keepdim=True)
    var = ((sf - mean) ** 2).mean(-1, keepdim=True)
    inv = torch.rsqrt(var + eps)
    y = (sf - mean) * inv * _t(x[2], s.device, torch.float32)
    if len(x) > 3 and x[3] is not None:
        y = y + _t(x[3], s.device, torch.float32)
    return [y.to(s.dtype), mean, inv, s][:max(1, rt.node_num_outputs)]


@op("SkipSimplifiedLayerNormalization")
def _skip_rms(rt, at, x):
    xs = list(x) + [None] * (5 - len(x))
    s = _skip_sum([xs[0], xs[1], None, None, xs[3]])  # inputs: input, skip, gamma, bias
    y, inv = _rms(s, xs[2], -1, float(at.get("epsilon", 1e-12)))
    return [y, None, inv, s][:max(1, rt.node_num_outputs)]


@op("EmbedLayerNormalization")
def _embed_ln(rt, at, x):
    xs = list(x) + [None] * (10 - len(x))
    ids = _t(xs[0]).long()
    dev = _dev([xs[2]])
    ids = ids.to(dev)
    word = _t(xs[2], dev)
    emb = word[ids]
    B, S = ids.shape
    pos_ids = _t(xs[8], dev).long() if xs[8] is not None else torch.arange(S, device=dev).expand(B, S)
    emb = emb + _t(xs[3], dev, emb.dtype)[pos_ids]
    if xs[1] is not None and xs[4] is not None:
        emb = emb + _t(xs[4], dev, emb.dtype)[_t(xs[1], dev).long()]
    y = Fn.layer_norm(emb.to(torch.float32), (emb.shape[-1],), _t(xs[5], dev, torch.float32),
                      _t(xs[6], dev, torch.float32), float(at.get("epsilon", 1e-12))).to(emb.dtype)
    if xs[7] is not None:
        mask_index = _t(xs[7], dev).to(torch.int32).sum(-1).to(torch.int32)
    else:
        mask_index = torch.full((B,), S, dtype=torch.int32, device=dev)
    return [y, mask_index, emb][:max(1, rt.node_num_outputs)]


def _attend(q, k, v, heads: int, scale: Optional[float], mask_add: Optional[torch.Tensor], causal: bool):
    """q [B, S, Dq], k [B, L, Dq], v [B, L, Dv] -> [B, S, Dv]; mask_add broadcastable to [B, heads, S, L]"""
    B, S, Dq = q.shape
    L, Dv = k.shape[1], v.shape[2]
    hq, hv = Dq // heads, Dv // heads
    qh = q.reshape(B, S, heads, hq).transpose(1, 2).to(torch.float32)
    kh = k.reshape(B, L, heads, hq).transpose(1, 2).to(torch.float32)
    vh = v.reshape(B, L, heads, hv).transpose(1, 2).to(torch.float32)
    sc = scale if scale else 1.0 / math.sqrt(hq)
    s = torch.matmul(qh, kh.transpose(-1, -2)) * sc
    if mask_add is not None:
        s = s + mask_add
    if causal:
        cm = torch.ones(S, L, dtype=torch.bool, device=s.device).tril(L - S)
        s = s.masked_fill(~cm, float("-inf"))
    p = torch.softmax(s, -1)
    return torch.matmul(p, vh).transpose(1, 2).reshape(B, S, Dv).to(q.dtype)


def _mask_to_add(mask, B, S, L, dev, filt: float):
    """contrib attention masks -> additive [B, 1, S|1, L]: 1-D [B] valid lengths (right padding), 2-D
    [B, L] 1/0 key mask, 3-D [B, S, L]"""
    if mask is None:
        return None
    m = _t(mask, dev)
    if m.dim() == 1 and m.numel() == B:
        keep = torch.arange(L, device=dev).unsqueeze(0) < m.reshape(B, 1).to(torch.long)
        return torch.where(keep, 0.0, filt).reshape(B, 1, 1, L)
    if m.dim() == 2:
        return torch.where(m.to(torch.bool), 0.0, filt).reshape(B, 1, 1, L)
    if m.dim() == 3:
        return torch.where(m.to(torch.bool), 0.0, filt).reshape(B, 1, S, L)
    raise NotImplementedError(f"attention mask of shape {tuple(m.shape)}")


@op("Attention")
def _attention(rt, at, x):
    xs = list(x) + [None] * (8 - len(x))
    inp = _t(xs[0])
    dev = inp.device
    w = _t(xs[1], dev, inp.dtype)
    qkv = torch.matmul(inp, w)
    if xs[2] is not None:
        qkv = qkv + _t(xs[2], dev, inp.dtype)
    heads = int(at["num_heads"])
    sizes = list(at.get("qkv_hidden_sizes", [])) or [qkv.shape[-1] // 3] * 3
    q, k, v = torch.split(qkv, sizes, -1)
    B, S = inp.shape[0], inp.shape[1]
    present = None
    if xs[4] is not None:  # past [2, B, heads, P, head] -> prepend to k / v
        past = _t(xs[4], dev, inp.dtype)
        pk = past[0].transpose(1, 2).reshape(B, -1, sizes[1])
        pv = past[1].transpose(1, 2).reshape(B, -1, sizes[2])
        k, v = torch.cat([pk, k], 1), torch.cat([pv, v], 1)
    L = k.shape[1]
    if rt.node_num_outputs > 1:
        present = torch.stack([k.reshape(B, L, heads, -1).transpose(1, 2), v.reshape(B, L, heads, -1).transpose(1, 2)])
    filt = float(at.get("mask_filter_value", -10000.0))
    mask_add = _mask_to_add(xs[3], B, S, L, dev, filt)
    if xs[5] is not None:  # relative position bias [B|1, heads, S, L]
        rb = _t(xs[5], dev, torch.float32)
        mask_add = rb if mask_add is None else mask_add + rb
    out = _attend(q, k, v, heads, at.get("scale"), mask_add, bool(int(at.get("unidirectional", 0))))
    return [out, present][:max(1, rt.node_num_outputs)]


@op("MultiHeadAttention")
def _mha(rt, at, x):
    xs = list(x) + [None] * (8 - len(x))
    q = _t(xs[0])
    dev = q.device
    k, v = _t(xs[1], dev, q.dtype), _t(xs[2], dev, q.dtype)
    if xs[3] is not None:
        b = _t(xs[3], dev, q.dtype)
        D, Dv = q.shape[-1], v.shape[-1]
        q, k, v = q + b[:D], k + b[D:2 * D], v + b[2 * D:2 * D + Dv]
    B, S, L = q.shape[0], q.shape[1], k.shape[1]
    mask_add = _mask_to_add(xs[4], B, S, L, dev, float(at.get("mask_filter_value", -10000.0)))
    if xs[5] is not None:
        rb = _t(xs[5], dev, torch.float32)
        mask_add = rb if mask_add is None else mask_add + rb
    out = _attend(q, k, v, int(at["num_heads"]), at.get("scale"), mask_add, bool(int(at.get("unidirectional", 0))))
    return [out]
