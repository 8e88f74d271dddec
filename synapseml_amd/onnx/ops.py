"""ONNX operator set executed on torch tensors (ROCm device or CPU).

Each op is ``fn(rt, attrs, inputs) -> list of outputs``. Values are torch
tensors, numpy ``object`` arrays (string tensors stay on the host), Python
lists (sequences) or dicts (maps). Shape-valued tensors (``Shape`` and the
integer arithmetic on them) are kept on the host so dynamic-shape chains
never force a device synchronisation.

Heavy ops (Conv, Gemm/MatMul) are placed on the device in the session's
compute dtype; the fused conv/epilogue variants produced by the optimizer
(``_FusedConv``, ``_AddBnRelu``, ``_ScaleShiftAct``) call the HIP kernels in
``csrc/nn`` on the GPU (see ``synapseml_amd/onnx/session.py``).
"""
from __future__ import annotations

import math
from typing import Any, Callable, Dict, List

import numpy as np
import torch
import torch.nn.functional as Fn

from . import proto as P

OPS: Dict[str, Callable] = {}

TORCH_OF = {P.FLOAT32: torch.float32, P.UINT8: torch.uint8, P.INT8: torch.int8, P.INT16: torch.int16,
            P.INT32: torch.int32, P.INT64: torch.int64, P.BOOL: torch.bool, P.FLOAT16: torch.float16,
            P.DOUBLE_T: torch.float64, P.BFLOAT16: torch.bfloat16, P.UINT16: torch.int32, P.UINT32: torch.int64,
            P.UINT64: torch.int64}


def op(*names):
    def deco(fn):
        for n in names:
            OPS[n] = fn
        return fn

    return deco


def _same_dev(a, b):
    if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and a.device != b.device:
        if a.device.type == "cpu" and a.dim() <= 1 and a.numel() <= 8 and b.device.type != "cpu" and b.numel() > 8:
            return a.to(b.device), b
        if b.device.type == "cpu":
            return a, b.to(a.device)
        return a.to(b.device), b
    return a, b


def _ints(t) -> List[int]:
    if t is None:
        return []
    if isinstance(t, torch.Tensor):
        return [int(v) for v in t.detach().cpu().reshape(-1).tolist()]
    return [int(v) for v in np.asarray(t).reshape(-1).tolist()]


def _promote(a, b):
    if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
        a, b = _same_dev(a, b)
        if a.dtype != b.dtype:
            # ONNX requires equal types; tolerate compute-dtype mixes (fp16 activations vs fp32 constants)
            if a.is_floating_point() and b.is_floating_point():
                t = a.dtype if a.numel() >= b.numel() else b.dtype
                a, b = a.to(t), b.to(t)
            elif a.is_floating_point():
                b = b.to(a.dtype)
            elif b.is_floating_point():
                a = a.to(b.dtype)
            else:
                t = torch.promote_types(a.dtype, b.dtype)
                a, b = a.to(t), b.to(t)
    return a, b


# ------------------------------------------------------------------ elementwise
def _binary(fn):
    def run(rt, at, x):
        a, b = _promote(x[0], x[1])
        return [fn(a, b)]

    return run


OPS["Add"] = _binary(torch.add)
OPS["Sub"] = _binary(torch.sub)
OPS["Mul"] = _binary(torch.mul)
OPS["Pow"] = lambda rt, at, x: [torch.pow(*_same_dev(x[0], x[1].to(x[0].dtype) if x[0].is_floating_point()
                                                       else x[1]))]
OPS["Equal"] = _binary(torch.eq)
OPS["Greater"] = _binary(torch.gt)
OPS["Less"] = _binary(torch.lt)
OPS["GreaterOrEqual"] = _binary(torch.ge)
OPS["LessOrEqual"] = _binary(torch.le)
OPS["And"] = _binary(torch.logical_and)
OPS["Or"] = _binary(torch.logical_or)
OPS["Xor"] = _binary(torch.logical_xor)
OPS["BitShift"] = lambda rt, at, x: [torch.bitwise_left_shift(*_promote(x[0], x[1])) if at.get("direction") == "LEFT"
                                     else torch.bitwise_right_shift(*_promote(x[0], x[1]))]


@op("Div")
def _div(rt, at, x):
    a, b = _promote(x[0], x[1])
    if not a.is_floating_point():
        return [torch.div(a, b, rounding_mode="trunc")]
    return [a / b]


@op("Mod")
def _mod(rt, at, x):
    a, b = _promote(x[0], x[1])
    return [torch.fmod(a, b) if at.get("fmod", 0) else torch.remainder(a, b)]


def _unary(fn):
    return lambda rt, at, x: [fn(x[0])]


for _n, _f in {"Abs": torch.abs, "Neg": torch.neg, "Exp": torch.exp, "Log": torch.log, "Sqrt": torch.sqrt,
               "Reciprocal": torch.reciprocal, "Floor": torch.floor, "Ceil": torch.ceil, "Round": torch.round,
               "Sin": torch.sin, "Cos": torch.cos, "Tan": torch.tan, "Asin": torch.asin, "Acos": torch.acos,
               "Atan": torch.atan, "Sinh": torch.sinh, "Cosh": torch.cosh, "Asinh": torch.asinh,
               "Acosh": torch.acosh, "Atanh": torch.atanh, "Tanh": torch.tanh, "Sigmoid": torch.sigmoid,
               "Relu": torch.relu, "Erf": torch.erf, "Not": torch.logical_not, "Sign": torch.sign,
               "Softsign": Fn.softsign, "Softplus": Fn.softplus, "IsNaN": torch.isnan,
               "BitwiseNot": torch.bitwise_not}.items():
    OPS[_n] = _unary(_f)

OPS["IsInf"] = lambda rt, at, x: [(torch.isposinf(x[0]) & bool(at.get("detect_positive", 1))) |
                                  (torch.isneginf(x[0]) & bool(at.get("detect_negative", 1)))]
OPS["LeakyRelu"] = lambda rt, at, x: [Fn.leaky_relu(x[0], at.get("alpha", 0.01))]
OPS["Elu"] = lambda rt, at, x: [Fn.elu(x[0], at.get("alpha", 1.0))]
OPS["Celu"] = lambda rt, at, x: [Fn.celu(x[0], at.get("alpha", 1.0))]
OPS["Selu"] = lambda rt, at, x: [at.get("gamma", 1.0507009873554805) *
                                 torch.where(x[0] > 0, x[0], at.get("alpha", 1.6732632423543772) *
                                             (torch.exp(x[0]) - 1))]
OPS["ThresholdedRelu"] = lambda rt, at, x: [torch.where(x[0] > at.get("alpha", 1.0), x[0], torch.zeros_like(x[0]))]
OPS["HardSigmoid"] = lambda rt, at, x: [torch.clamp(at.get("alpha", 0.2) * x[0] + at.get("beta", 0.5), 0, 1)]
OPS["HardSwish"] = lambda rt, at, x: [Fn.hardswish(x[0])]
OPS["Mish"] = lambda rt, at, x: [Fn.mish(x[0])]
OPS["Gelu"] = lambda rt, at, x: [Fn.gelu(x[0], approximate="tanh" if at.get("approximate") == "tanh" else "none")]
OPS["PRelu"] = lambda rt, at, x: [torch.where(x[0] >= 0, x[0], x[0] * _same_dev(x[1].to(x[0].dtype), x[0])[0])]
OPS["Identity"] = lambda rt, at, x: [x[0]]
OPS["Dropout"] = lambda rt, at, x: [x[0], torch.ones_like(x[0], dtype=torch.bool)]


@op("Clip")
def _clip(rt, at, x):
    lo = x[1] if len(x) > 1 and x[1] is not None else at.get("min")
    hi = x[2] if len(x) > 2 and x[2] is not None else at.get("max")
    lo = float(lo) if lo is not None else None
    hi = float(hi) if hi is not None else None
    return [torch.clamp(x[0], lo, hi)]


def _variadic(fn):
    def run(rt, at, x):
        out = x[0]
        for y in x[1:]:
            out, y = _promote(out, y)
            out = fn(out, y)
        return [out]

    return run


OPS["Sum"] = _variadic(torch.add)
OPS["Max"] = _variadic(torch.maximum)
OPS["Min"] = _variadic(torch.minimum)
OPS["Mean"] = lambda rt, at, x: [_variadic(torch.add)(rt, at, x)[0] / len(x)]


@op("Where")
def _where(rt, at, x):
    c, a = _same_dev(x[0], x[1])
    a, b = _promote(a, x[2])
    c = c.to(a.device)
    return [torch.where(c.bool(), a, b)]


@op("Cast", "CastLike")
def _cast(rt, at, x):
    to = at.get("to") if "to" in at else None
    if to is None:  # CastLike
        target = x[1]
        if isinstance(target, np.ndarray) and target.dtype == object:
            to = P.STRING_T
        else:
            return [x[0].to(target.dtype)]
    v = x[0]
    if to == P.STRING_T:
        arr = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
        return [arr.astype(str).astype(object)]
    if isinstance(v, np.ndarray) and v.dtype == object:
        np_t = P.NP_OF[to]
        return [torch.as_tensor(v.astype(np.float64).astype(np_t))]
    return [v.to(TORCH_OF[to])]


# ------------------------------------------------------------------ shape ops
@op("Shape")
def _shape(rt, at, x):
    shp = list(x[0].shape)
    s, e = at.get("start", 0), at.get("end", None)
    return [torch.tensor(shp[s:e] if e is not None else shp[s:], dtype=torch.int64)]


OPS["Size"] = lambda rt, at, x: [torch.tensor(int(np.prod(x[0].shape)), dtype=torch.int64)]


@op("Reshape")
def _reshape(rt, at, x):
    shape = _ints(x[1])
    inp = x[0]
    if not at.get("allowzero", 0):
        shape = [inp.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return [inp.reshape(shape)]


@op("Flatten")
def _flatten(rt, at, x):
    a = at.get("axis", 1)
    t = x[0]
    if a < 0:
        a += t.dim()
    lead = int(np.prod(t.shape[:a])) if a > 0 else 1
    return [t.reshape(lead, -1)]


@op("Squeeze")
def _squeeze(rt, at, x):
    axes = _ints(x[1]) if len(x) > 1 and x[1] is not None else at.get("axes")
    t = x[0]
    if axes is None:
        return [t.squeeze()]
    axes = sorted([a + t.dim() if a < 0 else a for a in axes], reverse=True)
    for a in axes:
        t = t.squeeze(a)
    return [t]


@op("Unsqueeze")
def _unsqueeze(rt, at, x):
    axes = _ints(x[1]) if len(x) > 1 and x[1] is not None else at.get("axes")
    t = x[0]
    r = t.dim() + len(axes)
    for a in sorted([a + r if a < 0 else a for a in axes]):
        t = t.unsqueeze(a)
    return [t]


@op("Transpose")
def _transpose(rt, at, x):
    perm = at.get("perm") or list(range(x[0].dim()))[::-1]
    return [x[0].permute(*perm)]


@op("Concat")
def _concat(rt, at, x):
    xs = [v for v in x if v is not None and (not isinstance(v, torch.Tensor) or v.numel() > 0 or v.dim() > 1)]
    if xs and isinstance(xs[0], np.ndarray):
        return [np.concatenate(xs, axis=at.get("axis", 0))]
    devs = {v.device for v in xs}
    if len(devs) > 1:
        dev = [d for d in devs if d.type != "cpu"][0]
        xs = [v.to(dev) for v in xs]
    if len({v.dtype for v in xs}) > 1:
        t = xs[0].dtype
        for v in xs[1:]:
            t = torch.promote_types(t, v.dtype)
        xs = [v.to(t) for v in xs]
    return [torch.cat(xs, dim=at.get("axis", 0))]


@op("Split")
def _split(rt, at, x):
    axis = at.get("axis", 0)
    t = x[0]
    if len(x) > 1 and x[1] is not None:
        sizes = _ints(x[1])
    elif "split" in at:
        sizes = at["split"]
    else:
        n = at.get("num_outputs", rt.node_num_outputs)
        d = t.shape[axis]
        chunk = -(-d // n)
        sizes = [min(chunk, d - i * chunk) for i in range(n)]
    return list(torch.split(t, sizes, dim=axis))


@op("Slice")
def _slice(rt, at, x):
    t = x[0]
    if len(x) > 1:
        starts, ends = _ints(x[1]), _ints(x[2])
        axes = _ints(x[3]) if len(x) > 3 and x[3] is not None else list(range(len(starts)))
        steps = _ints(x[4]) if len(x) > 4 and x[4] is not None else [1] * len(starts)
    else:
        starts, ends = at["starts"], at["ends"]
        axes = at.get("axes", list(range(len(starts))))
        steps = [1] * len(starts)
    idx = [slice(None)] * t.dim()
    flips = []
    for s, e, a, st in zip(starts, ends, axes, steps):
        a = a + t.dim() if a < 0 else a
        d = t.shape[a]
        if st > 0:
            s = max(0, min(d, s + d if s < 0 else s))
            e = max(0, min(d, e + d if e < 0 else e))
            idx[a] = slice(s, e, st)
        else:
            # negative step: slice forward then flip
            s = max(-1, min(d - 1, s + d if s < 0 else s))
            e = max(-1, min(d - 1, e + d if e < -d else (e + d if e < 0 else e)))
            lo = e + 1
            hi = s + 1
            if hi <= lo:
                idx[a] = slice(0, 0)
            else:
                idx[a] = slice(lo, hi)
                flips.append((a, -st))
    out = t[tuple(idx)]
    for a, st in flips:
        out = out.flip(a)
        if st != 1:
            sl = [slice(None)] * out.dim()
            sl[a] = slice(None, None, st)
            out = out[tuple(sl)]
    return [out]


@op("Gather")
def _gather(rt, at, x):
    axis = at.get("axis", 0)
    data, ind = x[0], x[1]
    if isinstance(data, np.ndarray):
        return [np.take(data, _to_np(ind).astype(np.int64), axis=axis)]
    ind = ind.to(data.device).long()
    d = data.shape[axis]
    ind = torch.where(ind < 0, ind + d, ind)
    out = torch.index_select(data, axis, ind.reshape(-1))
    shp = list(data.shape[:axis]) + list(ind.shape) + list(data.shape[axis + 1:])
    return [out.reshape(shp)]


@op("GatherElements")
def _gather_el(rt, at, x):
    axis = at.get("axis", 0)
    ind = x[1].to(x[0].device).long()
    ind = torch.where(ind < 0, ind + x[0].shape[axis], ind)
    return [torch.gather(x[0], axis, ind)]


@op("GatherND")
def _gather_nd(rt, at, x):
    data, ind = x[0], x[1].to(x[0].device).long()
    b = at.get("batch_dims", 0)
    if b != 0:
        raise NotImplementedError("GatherND batch_dims != 0")
    k = ind.shape[-1]
    flat = ind.reshape(-1, k)
    out = data[tuple(flat[:, i] for i in range(k))]
    return [out.reshape(list(ind.shape[:-1]) + list(data.shape[k:]))]


@op("ScatterElements", "Scatter")
def _scatter_el(rt, at, x):
    axis = at.get("axis", 0)
    red = at.get("reduction", "none")
    out = x[0].clone()
    ind = x[1].to(out.device).long()
    ind = torch.where(ind < 0, ind + out.shape[axis], ind)
    if red == "none":
        return [out.scatter(axis, ind, x[2].to(out.dtype))]
    return [out.scatter_reduce(axis, ind, x[2].to(out.dtype), {"add": "sum", "mul": "prod"}.get(red, red))]


@op("ScatterND")
def _scatter_nd(rt, at, x):
    out = x[0].clone()
    ind = x[1].to(out.device).long()
    k = ind.shape[-1]
    flat = ind.reshape(-1, k)
    upd = x[2].reshape([flat.shape[0]] + list(out.shape[k:])).to(out.dtype)
    out[tuple(flat[:, i] for i in range(k))] = upd
    return [out]


@op("Expand")
def _expand(rt, at, x):
    shape = _ints(x[1])
    t = x[0]
    tgt = list(torch.broadcast_shapes(tuple(t.shape), tuple(shape)))
    return [t.expand(tgt).contiguous()]


@op("Tile")
def _tile(rt, at, x):
    return [x[0].repeat(*_ints(x[1]))]


@op("ConstantOfShape")
def _const_of_shape(rt, at, x):
    v = at.get("value")
    val = np.asarray(v).reshape(-1)[0] if v is not None else np.float32(0)
    dt = torch.from_numpy(np.asarray([val])).dtype
    return [torch.full(_ints(x[0]), val.item(), dtype=dt, device=rt.device)]


@op("Constant")
def _constant(rt, at, x):
    for k in ("value", "value_float", "value_floats", "value_int", "value_ints", "value_string", "value_strings"):
        if k in at:
            v = at[k]
            if k == "value":
                arr = v
            elif k in ("value_string", "value_strings"):
                return [np.asarray(v, dtype=object)]
            else:
                arr = np.asarray(v, dtype=np.float32 if "float" in k else np.int64)
            if isinstance(arr, np.ndarray) and arr.dtype == object:
                return [arr]
            return [torch.from_numpy(np.array(arr, copy=True))]
    raise ValueError("Constant without value")


@op("Range")
def _range(rt, at, x):
    s, l, d = (v.item() for v in x[:3])
    return [torch.arange(s, l, d, dtype=x[0].dtype)]


@op("OneHot")
def _onehot(rt, at, x):
    ind, depth, vals = x[0], int(_ints(x[1])[0]), x[2]
    axis = at.get("axis", -1)
    ind = ind.long()
    ind = torch.where(ind < 0, ind + depth, ind)
    oh = Fn.one_hot(ind.clamp(0, depth - 1), depth) * ((ind >= 0) & (ind < depth)).unsqueeze(-1)
    vals = vals.to(ind.device)
    out = torch.where(oh.bool(), vals[1], vals[0])
    if axis != -1 and axis != out.dim() - 1:
        out = out.movedim(-1, axis)
    return [out]


@op("Trilu")
def _trilu(rt, at, x):
    k = int(_ints(x[1])[0]) if len(x) > 1 and x[1] is not None else 0
    return [torch.triu(x[0], k) if at.get("upper", 1) else torch.tril(x[0], k)]


@op("CumSum")
def _cumsum(rt, at, x):
    axis = int(_ints(x[1])[0])
    t = x[0]
    if at.get("reverse", 0):
        t = t.flip(axis)
    out = torch.cumsum(t, axis)
    if at.get("exclusive", 0):
        out = out - t
    if at.get("reverse", 0):
        out = out.flip(axis)
    return [out]


@op("DepthToSpace")
def _d2s(rt, at, x):
    b = at["blocksize"]
    t = x[0]
    n, c, h, w = t.shape
    if at.get("mode", "DCR") == "DCR":
        t = t.reshape(n, b, b, c // (b * b), h, w).permute(0, 3, 4, 1, 5, 2)
    else:
        t = t.reshape(n, c // (b * b), b, b, h, w).permute(0, 1, 4, 2, 5, 3)
    return [t.reshape(n, c // (b * b), h * b, w * b)]


@op("SpaceToDepth")
def _s2d(rt, at, x):
    b = at["blocksize"]
    t = x[0]
    n, c, h, w = t.shape
    t = t.reshape(n, c, h // b, b, w // b, b).permute(0, 3, 5, 1, 2, 4)
    return [t.reshape(n, c * b * b, h // b, w // b)]


# ------------------------------------------------------------------ reductions
def _axes(at, x, t):
    if len(x) > 1 and x[1] is not None:
        axes = _ints(x[1])
    else:
        axes = at.get("axes")
    if not axes:
        if at.get("noop_with_empty_axes", 0):
            return None
        return list(range(t.dim()))
    return [a + t.dim() if a < 0 else a for a in axes]


def _reduce(fn):
    def run(rt, at, x):
        t = x[0]
        axes = _axes(at, x, t)
        if axes is None:
            return [t]
        keep = bool(at.get("keepdims", 1))
        return [fn(t, axes, keep)]

    return run


OPS["ReduceSum"] = _reduce(lambda t, a, k: torch.sum(t, dim=a, keepdim=k))
OPS["ReduceMean"] = _reduce(lambda t, a, k: torch.mean(t, dim=a, keepdim=k))
OPS["ReduceMax"] = _reduce(lambda t, a, k: torch.amax(t, dim=a, keepdim=k))
OPS["ReduceMin"] = _reduce(lambda t, a, k: torch.amin(t, dim=a, keepdim=k))
OPS["ReduceProd"] = _reduce(lambda t, a, k: _prod(t, a, k))
OPS["ReduceL1"] = _reduce(lambda t, a, k: torch.sum(t.abs(), dim=a, keepdim=k))
OPS["ReduceL2"] = _reduce(lambda t, a, k: torch.sqrt(torch.sum(t * t, dim=a, keepdim=k)))
OPS["ReduceSumSquare"] = _reduce(lambda t, a, k: torch.sum(t * t, dim=a, keepdim=k))
OPS["ReduceLogSum"] = _reduce(lambda t, a, k: torch.log(torch.sum(t, dim=a, keepdim=k)))
OPS["ReduceLogSumExp"] = _reduce(lambda t, a, k: torch.logsumexp(t, dim=a, keepdim=k))


def _prod(t, axes, keep):
    for a in sorted(axes, reverse=True):
        t = torch.prod(t, dim=a, keepdim=keep)
    return t


def _arg(is_min):
    def run(rt, at, x):
        t = x[0]
        axis = at.get("axis", 0)
        keep = bool(at.get("keepdims", 1))
        if at.get("select_last_index", 0):
            t = t.flip(axis)
            r = (torch.argmin if is_min else torch.argmax)(t, dim=axis, keepdim=keep)
            r = t.shape[axis] - 1 - r
        else:
            r = (torch.argmin if is_min else torch.argmax)(t, dim=axis, keepdim=keep)
        return [r]

    return run


OPS["ArgMax"] = _arg(False)
OPS["ArgMin"] = _arg(True)


@op("TopK")
def _topk(rt, at, x):
    k = int(_ints(x[1])[0])
    axis = at.get("axis", -1)
    v, i = torch.topk(x[0], k, dim=axis, largest=bool(at.get("largest", 1)), sorted=bool(at.get("sorted", 1)))
    return [v, i]


def _softmax_like(kind):
    def run(rt, at, x):
        t = x[0]
        axis = at.get("axis", -1 if rt.opset >= 13 else 1)
        if rt.opset < 13:
            # coerce to 2D at axis
            a = axis + t.dim() if axis < 0 else axis
            shp = t.shape
            t2 = t.reshape(int(np.prod(shp[:a])) if a else 1, -1)
            return [run13(t2, -1).reshape(shp)]
        return [run13(t, axis)]

    def run13(t, axis):
        if kind == "soft":
            return torch.softmax(t, dim=axis)
        if kind == "log":
            return torch.log_softmax(t, dim=axis)
        idx = torch.argmax(t, dim=axis, keepdim=True)
        return torch.zeros_like(t).scatter_(axis, idx, 1.0)

    return run


OPS["Softmax"] = _softmax_like("soft")
OPS["LogSoftmax"] = _softmax_like("log")
OPS["Hardmax"] = _softmax_like("hard")


# ------------------------------------------------------------------ linear algebra
def _mfma_gemm_ok(rt, *ts) -> bool:
    """K17 on the device: float operands of one dtype on the GPU with the _nn module loaded."""
    from ..ops import gemm as G

    return getattr(getattr(rt, "session", None), "_nn", None) is not None and G.supported(*ts)


@op("MatMul")
def _matmul(rt, at, x):
    a, b = _promote(x[0], x[1])
    if _mfma_gemm_ok(rt, a, b) and a.dim() >= 1 and b.dim() >= 1:
        from ..ops import gemm as G

        return [G.matmul(a, b)]  # one batched MFMA launch (broadcast operands read with batch stride 0)
    return [torch.matmul(a, b)]  # host / integer graphs


@op("Gemm")
def _gemm(rt, at, x):
    a, b = _promote(x[0], x[1])
    if at.get("transA", 0):
        a = a.t()  # a view: the GEMM reads the transposed layout in place
    if at.get("transB", 0):
        b = b.t()
    alpha, beta = at.get("alpha", 1.0), at.get("beta", 1.0)
    c = x[2] if len(x) > 2 and x[2] is not None else None
    if _mfma_gemm_ok(rt, a, b) and a.dim() == 2 and b.dim() == 2:
        from ..ops import gemm as G

        N = b.shape[1]
        act = at.get("__act", 0)
        if c is not None and c.numel() == N and (c.dim() == 1 or c.shape[0] == 1):
            return [G.gemm(a, b, bias=c, alpha=alpha, beta=beta, relu=act == 1)]  # FC bias in the epilogue
        return [G.gemm(a, b, c=c, alpha=alpha, beta=beta if c is not None else 0.0, relu=act == 1)]
    y = torch.matmul(a, b)
    if alpha != 1.0:
        y = y * alpha
    if c is not None:
        c = c.to(y.device, y.dtype)
        y = y + (c * beta if beta != 1.0 else c)
    if at.get("__act", 0) == 1:
        y = torch.relu(y)
    return [y]


@op("Einsum")
def _einsum(rt, at, x):
    ts = list(x)
    for i in range(1, len(ts)):
        ts[0], ts[i] = _promote(ts[0], ts[i])
    return [torch.einsum(at["equation"], *ts)]


# ------------------------------------------------------------------ conv / pool / norm
def _pads_for(at, in_spatial, kernel, strides, dilations):
    auto = at.get("auto_pad", "NOTSET")
    nd = len(kernel)
    if auto in ("SAME_UPPER", "SAME_LOWER"):
        pads_b, pads_e = [], []
        for i in range(nd):
            out = -(-in_spatial[i] // strides[i])
            total = max(0, (out - 1) * strides[i] + (kernel[i] - 1) * dilations[i] + 1 - in_spatial[i])
            lo = total // 2 if auto == "SAME_UPPER" else total - total // 2
            pads_b.append(lo)
            pads_e.append(total - lo)
        return pads_b, pads_e
    if auto == "VALID":
        return [0] * nd, [0] * nd
    pads = at.get("pads", [0] * (2 * nd))
    return pads[:nd], pads[nd:]


def conv_args(at, x_shape, w_shape):
    nd = len(w_shape) - 2
    kernel = at.get("kernel_shape") or list(w_shape[2:])
    strides = at.get("strides", [1] * nd)
    dil = at.get("dilations", [1] * nd)
    pb, pe = _pads_for(at, list(x_shape[2:]), kernel, strides, dil)
    return nd, strides, dil, pb, pe


def _sym_pad(t, pb, pe, value=0.0):
    if pb == pe:
        return t, list(pb)
    pad = []
    for b, e in zip(reversed(pb), reversed(pe)):
        pad += [b, e]
    return Fn.pad(t, pad, value=value), [0] * len(pb)


@op("Conv")
def _conv(rt, at, x):
    inp, w = x[0], x[1]
    inp, w = _promote(inp, w)
    b = x[2].to(inp.device, inp.dtype) if len(x) > 2 and x[2] is not None else None
    nd, strides, dil, pb, pe = conv_args(at, inp.shape, w.shape)
    inp, pad = _sym_pad(inp, pb, pe)
    f = {1: Fn.conv1d, 2: Fn.conv2d, 3: Fn.conv3d}[nd]
    return [f(inp, w, b, stride=strides, padding=pad, dilation=dil, groups=at.get("group", 1))]


@op("ConvTranspose")
def _convT(rt, at, x):
    inp, w = _promote(x[0], x[1])
    b = x[2].to(inp.device, inp.dtype) if len(x) > 2 and x[2] is not None else None
    nd = w.dim() - 2
    strides = at.get("strides", [1] * nd)
    dil = at.get("dilations", [1] * nd)
    pads = at.get("pads", [0] * (2 * nd))
    outpad = at.get("output_padding", [0] * nd)
    f = {1: Fn.conv_transpose1d, 2: Fn.conv_transpose2d, 3: Fn.conv_transpose3d}[nd]
    return [f(inp, w, b, stride=strides, padding=pads[:nd], output_padding=outpad, groups=at.get("group", 1),
              dilation=dil)]


@op("MaxPool")
def _maxpool(rt, at, x):
    t = x[0]
    # executor fusion (session._move_epilogue_past_pool): x[1] = the producing conv's bias and
    # at["__act"] = 1 its ReLU, applied to the pooled maxima (max commutes with both exactly)
    shift = x[1] if len(x) > 1 else None
    act = at.get("__act", 0)
    k = at["kernel_shape"]
    nd = len(k)
    strides = at.get("strides", [1] * nd)
    dil = at.get("dilations", [1] * nd)
    pb, pe = _pads_for(at, list(t.shape[2:]), k, strides, dil)
    ceil = bool(at.get("ceil_mode", 0))
    nn = getattr(getattr(rt, "session", None), "_nn", None)
    if (nn is not None and nd == 2 and t.is_cuda and t.dim() == 4 and not ceil and list(dil) == [1, 1]
            and list(pb) == list(pe) and t.shape[1] % 8 == 0 and t.dtype in (torch.float16, torch.bfloat16, torch.float32)
            and t.is_contiguous(memory_format=torch.channels_last) and t.data_ptr() % 16 == 0
            and not (len(rt.node_outputs) > 1 and rt.node_outputs[1])):
        # K16: NHWC max pool on the HIP kernel (csrc/nn/nn_ops.hip), output stays channels-last
        from .session import _dtype_code, _stream

        N, C, H, W = t.shape
        OH = (H + 2 * pb[0] - k[0]) // strides[0] + 1
        OW = (W + 2 * pb[1] - k[1]) // strides[1] + 1
        y = torch.empty((N, C, OH, OW), dtype=t.dtype, device=t.device, memory_format=torch.channels_last)
        sh = shift.to(t.device, torch.float32).contiguous() if shift is not None else None
        nn.maxpool_nhwc(t.data_ptr(), N, H, W, C, k[0], k[1], strides[0], strides[1], pb[0], pb[1], OH, OW,
                        _dtype_code(t), y.data_ptr(), _stream(t), sh.data_ptr() if sh is not None else 0, int(act == 1))
        return [y]
    t, pad = _sym_pad(t, pb, pe, value=-math.inf)
    f = {1: Fn.max_pool1d, 2: Fn.max_pool2d, 3: Fn.max_pool3d}[nd]
    if len(rt.node_outputs) > 1 and rt.node_outputs[1]:
        y, i = f(t, k, strides, pad, dil, ceil_mode=ceil, return_indices=True)
        return [y, i]
    y = f(t, k, strides, pad, dil, ceil_mode=ceil)
    if shift is not None or act == 1:
        yf = y.float()
        if shift is not None:
            yf = yf + shift.to(y.device, torch.float32).reshape([1, -1] + [1] * (y.dim() - 2))
        y = (torch.relu(yf) if act == 1 else yf).to(y.dtype)
    return [y]


@op("AveragePool")
def _avgpool(rt, at, x):
    t = x[0]
    k = at["kernel_shape"]
    nd = len(k)
    strides = at.get("strides", [1] * nd)
    pb, pe = _pads_for(at, list(t.shape[2:]), k, strides, [1] * nd)
    incl = bool(at.get("count_include_pad", 0))
    ceil = bool(at.get("ceil_mode", 0))
    if pb != pe:
        if incl:
            t, pad = _sym_pad(t, pb, pe)
        else:
            # exclude padding: average of valid entries = pooled sum / pooled count
            ones = torch.ones_like(t[:1, :1])
            tp, _ = _sym_pad(t, pb, pe)
            op_, _ = _sym_pad(ones, pb, pe)
            f = {1: Fn.avg_pool1d, 2: Fn.avg_pool2d, 3: Fn.avg_pool3d}[nd]
            return [f(tp, k, strides, 0, ceil) / f(op_, k, strides, 0, ceil)]
    else:
        pad = pb
    f = {1: Fn.avg_pool1d, 2: Fn.avg_pool2d, 3: Fn.avg_pool3d}[nd]
    if nd == 1:
        return [f(t, k, strides, pad, ceil, incl)]
    return [f(t, k, strides, pad, ceil, incl)]


@op("LpPool")
def _lppool(rt, at, x):
    p = at.get("p", 2)
    k = at["kernel_shape"]
    nd = len(k)
    f = {1: Fn.lp_pool1d, 2: Fn.lp_pool2d}[nd]
    return [f(x[0], p, k, at.get("strides", k))]


@op("GlobalAveragePool")
def _gap(rt, at, x):
    t = x[0]
    nn = getattr(getattr(rt, "session", None), "_nn", None)
    if (nn is not None and t.is_cuda and t.dim() == 4 and t.dtype in (torch.float16, torch.bfloat16, torch.float32)
            and t.is_contiguous(memory_format=torch.channels_last)):
        # K16: NHWC global average pool on the HIP kernel, output in the input dtype ([N, C, 1, 1] is both
        # layouts at once), fp32 accumulation
        from .session import _dtype_code, _stream

        N, C, H, W = t.shape
        y = torch.empty((N, C, 1, 1), dtype=t.dtype, device=t.device)
        nn.gap_nhwc(t.data_ptr(), N, H * W, C, _dtype_code(t), y.data_ptr(), _stream(t))
        return [y]
    return [t.mean(dim=tuple(range(2, t.dim())), keepdim=True)]


@op("GlobalMaxPool")
def _gmp(rt, at, x):
    t = x[0]
    return [t.amax(dim=tuple(range(2, t.dim())), keepdim=True)]


@op("BatchNormalization")
def _bn(rt, at, x):
    t = x[0]
    sc, bi, mean, var = (v.to(t.device, t.dtype) for v in x[1:5])
    return [Fn.batch_norm(t, mean, var, sc, bi, training=False, eps=at.get("epsilon", 1e-5))]


@op("InstanceNormalization")
def _inorm(rt, at, x):
    t = x[0]
    return [Fn.instance_norm(t, weight=x[1].to(t.device, t.dtype), bias=x[2].to(t.device, t.dtype),
                             eps=at.get("epsilon", 1e-5))]


@op("LayerNormalization")
def _lnorm(rt, at, x):
    t = x[0]
    axis = at.get("axis", -1)
    axis = axis + t.dim() if axis < 0 else axis
    shp = t.shape[axis:]
    w = x[1].to(t.device, t.dtype) if len(x) > 1 and x[1] is not None else None
    b = x[2].to(t.device, t.dtype) if len(x) > 2 and x[2] is not None else None
    return [Fn.layer_norm(t, shp, w, b, at.get("epsilon", 1e-5))]


@op("LRN")
def _lrn(rt, at, x):
    return [Fn.local_response_norm(x[0], at["size"], at.get("alpha", 1e-4), at.get("beta", 0.75), at.get("bias", 1.0))]


@op("LpNormalization")
def _lpnorm(rt, at, x):
    return [Fn.normalize(x[0], p=at.get("p", 2), dim=at.get("axis", -1))]


@op("Pad")
def _pad(rt, at, x):
    t = x[0]
    pads = _ints(x[1]) if len(x) > 1 and x[1] is not None else at.get("pads")
    val = float(x[2].item()) if len(x) > 2 and x[2] is not None and x[2].numel() else float(at.get("value", 0.0))
    mode = at.get("mode", "constant")
    nd = t.dim()
    if len(x) > 3 and x[3] is not None:
        axes = [a + nd if a < 0 else a for a in _ints(x[3])]
        full = [0] * (2 * nd)
        for i, a in enumerate(axes):
            full[a] = pads[i]
            full[a + nd] = pads[i + len(axes)]
        pads = full
    tp = []
    for i in reversed(range(nd)):
        tp += [pads[i], pads[i + nd]]
    while len(tp) > 2 and tp[-1] == 0 and tp[-2] == 0:
        tp = tp[:-2]
    tmode = {"constant": "constant", "reflect": "reflect", "edge": "replicate", "wrap": "circular"}[mode]
    if tmode == "constant":
        return [Fn.pad(t, tp, mode="constant", value=val)]
    return [Fn.pad(t, tp, mode=tmode)]


@op("Resize", "Upsample")
def _resize(rt, at, x):
    t = x[0]
    mode = at.get("mode", "nearest")
    sizes = None
    scales = None
    if rt.op_type == "Upsample":
        scales = _floats(x[1]) if len(x) > 1 else at.get("scales")
    else:
        if len(x) > 3 and x[3] is not None and x[3].numel():
            sizes = _ints(x[3])
        elif len(x) > 2 and x[2] is not None and x[2].numel():
            scales = _floats(x[2])
    spatial = t.dim() - 2
    if sizes is not None:
        out = sizes[2:]
    else:
        out = [int(math.floor(t.shape[2 + i] * scales[2 + i])) for i in range(spatial)]
    ctm = at.get("coordinate_transformation_mode", "half_pixel")
    if mode == "nearest":
        return [Fn.interpolate(t, size=out, mode="nearest")]
    tmode = {1: "linear", 2: "bilinear", 3: "trilinear"}[spatial] if mode == "linear" else "bicubic"
    return [Fn.interpolate(t, size=out, mode=tmode, align_corners=(ctm == "align_corners"))]


def _floats(t):
    if isinstance(t, torch.Tensor):
        return [float(v) for v in t.detach().cpu().reshape(-1).tolist()]
    return [float(v) for v in np.asarray(t).reshape(-1)]


def _to_np(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    return np.asarray(v)


# ------------------------------------------------------------------ ai.onnx.ml + text
@op("ZipMap")
def _zipmap(rt, at, x):
    probs = _to_np(x[0])
    keys = at.get("classlabels_int64s") or at.get("classlabels_strings")
    return [[{k: float(v) for k, v in zip(keys, row)} for row in probs]]


def _post(kind, s):
    if kind == "SOFTMAX":
        return torch.softmax(s, dim=1)
    if kind == "LOGISTIC":
        return torch.sigmoid(s)
    if kind == "SOFTMAX_ZERO":
        e = torch.where(s == 0, torch.zeros_like(s), torch.exp(s - s.max(dim=1, keepdim=True).values))
        return e / e.sum(dim=1, keepdim=True).clamp_min(1e-30)
    if kind == "PROBIT":
        return math.sqrt(2) * torch.erfinv(2 * s - 1)
    return s


def _attr_const(at, dev, key, make):
    """A device tensor built once per (node attributes, device) and kept in the attribute dict (like the
    compiled tree ensembles): no host->device copy per run, so the op can sit inside a HIP-graph capture."""
    cache = at.setdefault("__dev_consts__", {})
    k = (key, str(dev))
    t = cache.get(k)
    if t is None:
        t = make()
        cache[k] = t
    return t


def _labels_of(at, dev, labels, idx):
    """class labels for argmax indices: on the device for integer labels, host objects for strings"""
    if isinstance(labels[0], str):
        return np.asarray(labels)[idx.cpu().numpy()].astype(object)
    lt = _attr_const(at, dev, "labels", lambda: torch.tensor([int(v) for v in labels], dtype=torch.int64, device=dev))
    return lt[idx]


@op("LinearClassifier")
def _linclf(rt, at, x):
    X = x[0].to(torch.float32)
    labels = at.get("classlabels_ints") or at.get("classlabels_strings")
    nc = len(labels)
    dev = X.device
    coef = _attr_const(at, dev, "coef", lambda: torch.tensor(at["coefficients"], dtype=torch.float32,
                                                             device=dev).reshape(-1, X.shape[1]))
    inter = _attr_const(at, dev, "inter", lambda: torch.tensor(at.get("intercepts", [0.0] * coef.shape[0]),
                                                               dtype=torch.float32, device=dev))
    s = X @ coef.t() + inter
    if coef.shape[0] == 1 and nc == 2:
        s = torch.cat([-s, s], dim=1)
        if at.get("post_transform", "NONE") == "LOGISTIC":
            p = torch.sigmoid(s[:, 1:2])
            s = torch.cat([1 - p, p], 1)
            post = s
        else:
            post = _post(at.get("post_transform", "NONE"), s)
    else:
        post = _post(at.get("post_transform", "NONE"), s)
    return [_labels_of(at, dev, labels, torch.argmax(s, dim=1)), post]


@op("LinearRegressor")
def _linreg(rt, at, x):
    X = x[0].to(torch.float32)
    t = at.get("targets", 1)
    coef = _attr_const(at, X.device, "coef", lambda: torch.tensor(at["coefficients"], dtype=torch.float32,
                                                                  device=X.device).reshape(t, -1))
    inter = _attr_const(at, X.device, "inter", lambda: torch.tensor(at.get("intercepts", [0.0] * t),
                                                                    dtype=torch.float32, device=X.device))
    return [_post(at.get("post_transform", "NONE"), X @ coef.t() + inter)]


@op("Normalizer")
def _normalizer(rt, at, x):
    X = x[0].to(torch.float32)
    n = at.get("norm", "MAX")
    if n == "MAX":
        d = X.abs().amax(dim=1, keepdim=True)
    elif n == "L1":
        d = X.abs().sum(dim=1, keepdim=True)
    else:
        d = X.pow(2).sum(dim=1, keepdim=True).sqrt()
    return [X / d.clamp_min(1e-30)]


@op("Scaler")
def _scaler(rt, at, x):
    X = x[0].to(torch.float32)
    off = _attr_const(at, X.device, "off", lambda: torch.tensor(at.get("offset", [0.0]), dtype=torch.float32,
                                                                device=X.device))
    sc = _attr_const(at, X.device, "sc", lambda: torch.tensor(at.get("scale", [1.0]), dtype=torch.float32,
                                                              device=X.device))
    return [(X - off) * sc]


@op("ArrayFeatureExtractor")
def _afe(rt, at, x):
    data = x[0]
    ind = _ints(x[1])
    if isinstance(data, np.ndarray):
        return [data[..., ind]]
    key = ("ind",) + tuple(int(i) for i in np.ravel(ind))
    return [data[..., _attr_const(at, data.device, key, lambda: torch.tensor(ind, device=data.device))]]


@op("Binarizer")
def _binarizer(rt, at, x):
    return [(x[0] > at.get("threshold", 0.0)).to(x[0].dtype)]


@op("LabelEncoder")
def _label_encoder(rt, at, x):
    keys = at.get("keys_strings") or at.get("keys_int64s") or at.get("keys_floats")
    vals = at.get("values_strings") or at.get("values_int64s") or at.get("values_floats")
    default = at.get("default_string", at.get("default_int64", at.get("default_float", -1)))
    m = dict(zip(keys, vals))
    arr = _to_np(x[0])
    out = np.vectorize(lambda k: m.get(k, default), otypes=[object])(arr)
    if isinstance(vals[0], str):
        return [out]
    return [torch.from_numpy(out.astype(np.int64 if isinstance(vals[0], int) else np.float32))]


@op("OneHotEncoder")
def _ohe(rt, at, x):
    cats = at.get("cats_strings") or at.get("cats_int64s")
    arr = _to_np(x[0])
    idx = {c: i for i, c in enumerate(cats)}
    out = np.zeros(arr.shape + (len(cats),), np.float32)
    for pos, v in np.ndenumerate(arr):
        j = idx.get(v if isinstance(cats[0], str) else int(v))
        if j is not None:
            out[pos + (j,)] = 1.0
        elif not at.get("zeros", 1):
            raise ValueError(f"unknown category {v}")
    return [torch.from_numpy(out)]


@op("Imputer")
def _imputer(rt, at, x):
    X = x[0]
    vals = _attr_const(at, X.device, ("vals", str(X.dtype)), lambda: torch.tensor(
        at.get("imputed_value_floats") or at.get("imputed_value_int64s"), device=X.device, dtype=X.dtype))
    rep = at.get("replaced_value_float", float("nan"))
    mask = torch.isnan(X) if math.isnan(rep) else (X == rep)
    return [torch.where(mask, vals.expand_as(X) if vals.numel() > 1 else vals, X)]


@op("TreeEnsembleRegressor", "TreeEnsembleClassifier")
def _tree_ensemble(rt, at, x):
    from .tree_ensemble import run_tree_ensemble

    return run_tree_ensemble(rt, at, x)


@op("TfIdfVectorizer")
def _tfidf(rt, at, x):
    """TF/IDF/TFIDF n-gram counts over string or int64 token tensors (1-D or 2-D)."""
    data = _to_np(x[0])
    pool = at.get("pool_strings") or at.get("pool_int64s")
    counts = at["ngram_counts"]
    idxs = at["ngram_indexes"]
    mn, mx = at.get("min_gram_length", 1), at.get("max_gram_length", 1)
    skip = at.get("max_skip_count", 0)
    weights = at.get("weights")
    mode = at.get("mode", "TF")
    out_dim = max(idxs) + 1 if idxs else 0
    # n-gram table: n -> {tuple: output index}
    table: Dict[tuple, int] = {}
    bounds = list(counts) + [len(pool)]
    k = 0
    for gi in range(len(counts)):
        n = gi + 1
        for p in range(bounds[gi], bounds[gi + 1], n):
            table[tuple(pool[p:p + n])] = idxs[k]
            k += 1
    rows = data.reshape(1, -1) if data.ndim == 1 else data
    res = np.zeros((rows.shape[0], out_dim), np.float32)
    for r, toks in enumerate(rows):
        toks = [t if isinstance(t, str) else int(t) for t in toks]
        for n in range(mn, mx + 1):
            for s in range(skip + 1):
                step = s + 1
                for i in range(len(toks)):
                    g = tuple(toks[i + j * step] for j in range(n) if i + j * step < len(toks))
                    if len(g) != n:
                        continue
                    j = table.get(g)
                    if j is not None:
                        res[r, j] += 1.0
                if n == 1:
                    break
    if mode == "IDF":
        res = (res > 0).astype(np.float32) * (np.asarray(weights, np.float32) if weights else 1.0)
    elif mode == "TFIDF" and weights:
        res = res * np.asarray(weights, np.float32)
    return [torch.from_numpy(res.reshape(-1) if data.ndim == 1 else res)]


# ------------------------------------------------------------------ control flow
@op("If")
def _if(rt, at, x):
    cond = bool(_to_np(x[0]).reshape(-1)[0])
    g = at["then_branch"] if cond else at["else_branch"]
    return rt.run_subgraph(g, {})
