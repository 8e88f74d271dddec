"""ONNX inference session for the MI355X (replaces ONNX Runtime; reference:
deep-learning/.../onnx/ONNXRuntime.scala:25-107).

Compile pipeline (``optimization_level`` BASIC/EXTENDED/ALL_OPT, NO_OPT skips
2-4):

1. decode + topologically order the graph (graph.py);
2. constant folding — every node whose inputs are all constants is evaluated
   once on the host (shape arithmetic, weight transposes, ...);
3. Conv→BatchNormalization folding into the conv weights/bias;
4. epilogue fusion: Conv[+bias][+residual Add][+Relu/LeakyRelu/Sigmoid/Clip]
   → one conv + one fused epilogue pass; standalone BatchNormalization[+act]
   → one affine pass; the pre-activation pattern ``s = a + b; y = act(bn(s))``
   (ResNet v2) → one pass writing both ``s`` and ``y``. On the GPU the
   epilogues run as the HIP kernels of csrc/nn (module ``_nn``); on the host
   they run as torch ops with identical math.

Execution: activations live on the session's device in the compute dtype
(fp32 by default for ORT parity; fp16/bf16 selectable), 4-D activations in
channels-last layout on the GPU; dead intermediates are freed at their last
use. For fixed input shapes the whole plan is captured once into a HIP graph
(``torch.cuda.CUDAGraph`` drives hipGraph on ROCm) and replayed, so a batch
costs one graph launch instead of one launch per node.
"""
from __future__ import annotations

import math
import os
import threading
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import proto as P
from .graph import Graph, Node, ValueInfo
from .ops import OPS, TORCH_OF, conv_args, _sym_pad
from . import ops_ext  # noqa: F401  (registers the extended operator set)

OPT_LEVELS = ("NO_OPT", "BASIC_OPT", "EXTENDED_OPT", "ALL_OPT")
_ACTS = {"Relu": 1, "LeakyRelu": 2, "Sigmoid": 3, "Clip": 4}
_NONDETERMINISTIC = {"RandomNormal", "RandomUniform", "RandomNormalLike", "RandomUniformLike", "Multinomial",
                     "Bernoulli"}
_MAX_FOLD_ELEMS = 1 << 24


def _is_const_tensor(v) -> bool:
    return isinstance(v, (torch.Tensor, np.ndarray))


def _outer_refs(g: Graph) -> set:
    """names a graph (and its nested subgraphs) reads without producing them: its outer-scope references"""
    produced = set(g.initializers) | {v.name for v in g.inputs}
    refs = set()
    for n in g.nodes:
        for x in n.inputs:
            if x and x not in produced:
                refs.add(x)
        for v in n.attrs.values():
            if isinstance(v, Graph):
                refs |= {x for x in _outer_refs(v) if x not in produced}
        produced.update(o for o in n.outputs if o)
    return refs


class _RT:
    """Per-node runtime context handed to op implementations."""

    __slots__ = ("device", "opset", "op_type", "node_outputs", "node_num_outputs", "session")

    def __init__(self, session, node: Node):
        self.device = session.device
        self.opset = session.opset
        self.op_type = node.op_type
        self.node_outputs = node.outputs
        self.node_num_outputs = len(node.outputs)
        self.session = session

    def run_subgraph(self, g: Graph, feeds: Dict[str, Any]):
        """Run a graph attribute (If branch, Loop / Scan body) with this graph's live values as its outer
        scope. The sub-session is built once per graph and reused across iterations and runs."""
        cache = self.session.__dict__.setdefault("_sub_sessions", {})
        sub = cache.get(id(g))
        if sub is None or sub.graph is not g:
            sub = InferenceSession.from_graph(g, device=self.device, optimization_level="NO_OPT",
                                              outer=self.session._live_values)
            cache[id(g)] = sub
        sub._outer = self.session._live_values
        return sub.run_values(feeds)


class InferenceSession:
    def __init__(self, model: bytes, device: Optional[str] = None, precision: str = "fp32",
                 optimization_level: str = "ALL_OPT", use_graph: bool = True, channels_last: Optional[bool] = None):
        g = Graph.from_bytes(model)
        self._init(g, device, precision, optimization_level, use_graph, channels_last)

    @classmethod
    def from_graph(cls, g: Graph, device=None, precision="fp32", optimization_level="ALL_OPT", use_graph=False,
                   outer: Optional[Dict[str, Any]] = None):
        s = cls.__new__(cls)
        s._outer = outer or {}
        s._init(g, device, precision, optimization_level, use_graph, None)
        return s

    # ------------------------------------------------------------------ setup
    def _init(self, g: Graph, device, precision, optimization_level, use_graph, channels_last):
        if not hasattr(self, "_outer"):
            self._outer = {}
        self.graph = g
        if device is None or str(device).upper() in ("GPU", "CUDA", "ROCM", "AUTO"):
            device = "cuda" if torch.cuda.is_available() else "cpu"
        elif str(device).upper() == "CPU":
            device = "cpu"
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.gpu = self.device.type == "cuda"
        self.opset = int(g.opset.get("", g.opset.get("ai.onnx", 13)))
        # "fp32" | "fp16" | "bf16", or "fp32-<mode>" choosing how fp32 convolutions use the matrix cores
        # (ops.conv.F32_MODES: exact f32 MFMAs, or f32 operands split over bf16 planes; default SML_CONV_F32)
        base, _, mode = str(precision).partition("-")
        self.compute_dtype = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[base]
        from ..ops.conv import F32_MODES

        if mode and (base != "fp32" or mode not in F32_MODES):
            raise ValueError(f"precision {precision!r}: fp32 modes are {['fp32-' + m for m in F32_MODES]}")
        self.f32_conv_mode = mode or None
        self.channels_last = self.gpu if channels_last is None else channels_last
        lvl = optimization_level.upper()
        if lvl not in OPT_LEVELS:
            raise ValueError(f"optimizationLevel must be one of {OPT_LEVELS}")
        self.optimization_level = lvl
        self.use_graph = use_graph and self.gpu
        self.inputs: List[ValueInfo] = list(g.inputs)
        self.outputs: List[ValueInfo] = list(g.outputs)
        self._nn = None
        if self.gpu:
            from ..ops import native

            self._nn = native.load("_nn")  # loud failure if the HIP kernels are missing on a GPU box
        self._consts: Dict[str, Any] = {}
        for k, v in g.initializers.items():
            self._consts[k] = v if v.dtype == object else torch.from_numpy(np.array(v, copy=True))
        nodes = g.toposort(outer=g.outer_refs() if self._outer else ())
        if lvl != "NO_OPT":
            nodes = self._fold_constants(nodes)
            nodes = self._fold_conv_bn(nodes)
            nodes = self._fuse_epilogues(nodes)
            if self._nn is not None and self.channels_last:
                nodes = self._fuse_prologues(nodes)
            if self._nn is not None:
                nodes = self._move_epilogue_past_pool(nodes)
        self.nodes = nodes
        self._place_constants()
        self._plan_liveness()
        self._graphs: Dict[tuple, Any] = {}
        self._graph_lock = threading.Lock()
        self._live_values: Dict[str, Any] = {}

    def _fold_constants(self, nodes: List[Node]) -> List[Node]:
        out = []
        for n in nodes:
            if (n.op_type not in _NONDETERMINISTIC and n.op_type in OPS and n.inputs
                    and all((not x) or x in self._consts for x in n.inputs)
                    and not any(isinstance(v, Graph) for v in n.attrs.values())
                    and all(_numel(self._consts[x]) <= _MAX_FOLD_ELEMS for x in n.inputs if x)):
                try:
                    rt = _RT(self, n)
                    rt.device = torch.device("cpu")
                    vals = OPS[n.op_type](rt, n.attrs, [self._consts[x] if x else None for x in n.inputs])
                    if all(_is_const_tensor(v) for v in vals):
                        for name, v in zip(n.outputs, vals):
                            if name:
                                self._consts[name] = v.cpu() if isinstance(v, torch.Tensor) else v
                        continue
                except Exception:
                    pass
            elif n.op_type == "Constant":
                vals = OPS["Constant"](_RT(self, n), n.attrs, [])
                self._consts[n.outputs[0]] = vals[0]
                continue
            out.append(n)
        return out

    def _consumers(self, nodes: List[Node]) -> Dict[str, int]:
        cnt: Dict[str, int] = {}
        for n in nodes:
            for x in n.inputs:
                if x:
                    cnt[x] = cnt.get(x, 0) + 1
        for o in self.outputs:
            cnt[o.name] = cnt.get(o.name, 0) + 1
        return cnt

    def _fold_conv_bn(self, nodes: List[Node]) -> List[Node]:
        cnt = self._consumers(nodes)
        prod = {o: n for n in nodes for o in n.outputs}
        drop = set()
        for n in nodes:
            if n.op_type != "BatchNormalization" or len(n.outputs) > 1 and any(n.outputs[1:]):
                continue
            src = prod.get(n.inputs[0])
            if src is None or src.op_type != "Conv" or cnt.get(src.outputs[0], 0) != 1:
                continue
            if src.inputs[1] not in self._consts or not all(x in self._consts for x in n.inputs[1:5]):
                continue
            if len(src.inputs) > 2 and src.inputs[2] and src.inputs[2] not in self._consts:
                continue
            w = self._consts[src.inputs[1]].double()
            gamma, beta, mean, var = (self._consts[x].double() for x in n.inputs[1:5])
            s = gamma / torch.sqrt(var + n.attrs.get("epsilon", 1e-5))
            b = self._consts[src.inputs[2]].double() if len(src.inputs) > 2 and src.inputs[2] else torch.zeros_like(mean)
            wn = (w * s.reshape(-1, *([1] * (w.dim() - 1)))).float()
            bn = ((b - mean) * s + beta).float()
            wname, bname = src.inputs[1] + "__bnfold", src.outputs[0] + "__bnfold_bias"
            self._consts[wname] = wn
            self._consts[bname] = bn
            src.inputs = [src.inputs[0], wname, bname]
            src.outputs = [n.outputs[0]]
            drop.add(id(n))
        return [n for n in nodes if id(n) not in drop]

    def _fuse_epilogues(self, nodes: List[Node]) -> List[Node]:
        cnt = self._consumers(nodes)
        by_input: Dict[str, List[Node]] = {}
        for n in nodes:
            for x in n.inputs:
                by_input.setdefault(x, []).append(n)
        drop = set()
        out_nodes = []

        def sole_consumer(name) -> Optional[Node]:
            cs = by_input.get(name, [])
            if len(cs) == 1 and cnt.get(name, 0) == 1 and id(cs[0]) not in drop:
                return cs[0]
            return None

        def act_of(n: Node) -> Tuple[int, float]:
            if n.op_type == "Clip":
                lo = n.attrs.get("min") if len(n.inputs) < 2 or not n.inputs[1] else _scalar(self._consts.get(n.inputs[1]))
                hi = n.attrs.get("max") if len(n.inputs) < 3 or not n.inputs[2] else _scalar(self._consts.get(n.inputs[2]))
                if lo == 0.0 and hi is not None:
                    return 4, float(hi)
                return 0, 0.0
            if n.op_type == "LeakyRelu":
                return 2, float(n.attrs.get("alpha", 0.01))
            return _ACTS.get(n.op_type, 0), 0.0

        for n in nodes:
            if id(n) in drop:
                continue
            if n.op_type == "Gemm":
                # Gemm -> Relu: the ReLU runs in the MFMA GEMM's epilogue (K17)
                nxt = sole_consumer(n.outputs[0])
                if nxt is not None and nxt.op_type == "Relu" and not n.attrs.get("__act", 0):
                    g = Node("Gemm", list(n.inputs), [nxt.outputs[0]], dict(n.attrs, __act=1), n.name)
                    drop.add(id(nxt))
                    out_nodes.append(g)
                    continue
            if n.op_type == "Conv" and n.inputs[1] in self._consts and len(self._consts[n.inputs[1]].shape) == 4:
                fused = Node("_FusedConv", list(n.inputs[:3]) + [""] * (3 - len(n.inputs[:3])), list(n.outputs),
                             dict(n.attrs), n.name)
                cur = n.outputs[0]
                nxt = sole_consumer(cur)
                # optional broadcast bias add (mnist style: Conv -> Add(const [C,1,1]))
                if nxt is not None and nxt.op_type == "Add" and not fused.inputs[2]:
                    other = nxt.inputs[1] if nxt.inputs[0] == cur else nxt.inputs[0]
                    c = self._consts.get(other)
                    cout = self._consts[n.inputs[1]].shape[0]
                    if isinstance(c, torch.Tensor) and c.numel() == cout and c.dim() >= 1 and \
                            (c.dim() < 3 or c.shape[-1] == 1):
                        bname = other + "__as_bias"
                        self._consts[bname] = c.reshape(-1).float()
                        fused.inputs[2] = bname
                        drop.add(id(nxt))
                        cur = nxt.outputs[0]
                        nxt = sole_consumer(cur)
                # residual add of another tensor
                # (an Add feeding a BatchNormalization is left to the one-pass _AddAffineAct instead)
                if nxt is not None and nxt.op_type == "Add" and not any(
                        c.op_type == "BatchNormalization" for c in by_input.get(nxt.outputs[0], [])):
                    other = nxt.inputs[1] if nxt.inputs[0] == cur else nxt.inputs[0]
                    if other not in self._consts and other != cur:
                        fused.inputs.append(other)
                        drop.add(id(nxt))
                        cur = nxt.outputs[0]
                        nxt = sole_consumer(cur)
                if nxt is not None:
                    a, alpha = act_of(nxt)
                    if a:
                        fused.attrs["__act"] = a
                        fused.attrs["__alpha"] = alpha
                        drop.add(id(nxt))
                        cur = nxt.outputs[0]
                fused.outputs = [cur]
                out_nodes.append(fused)
                continue
            if n.op_type == "Add" and len(n.inputs) == 2 and all(x not in self._consts for x in n.inputs):
                bn = None
                for c in by_input.get(n.outputs[0], []):
                    if c.op_type == "BatchNormalization" and all(x in self._consts for x in c.inputs[1:5]) and \
                            (len(c.outputs) == 1 or not any(c.outputs[1:])):
                        bn = c
                        break
                if bn is not None:
                    nxt = sole_consumer(bn.outputs[0])
                    a, alpha = act_of(nxt) if nxt is not None else (0, 0.0)
                    scale, shift = self._bn_affine(bn)
                    out_name = nxt.outputs[0] if a == 1 else bn.outputs[0]
                    fn = Node("_AddAffineAct", list(n.inputs) + [scale, shift], [n.outputs[0], out_name],
                              {"__act": 1 if a == 1 else 0}, n.name)
                    drop.add(id(bn))
                    if a == 1:
                        drop.add(id(nxt))
                    out_nodes.append(fn)
                    continue
            if n.op_type == "BatchNormalization" and all(x in self._consts for x in n.inputs[1:5]) and \
                    (len(n.outputs) == 1 or not any(n.outputs[1:])):
                scale, shift = self._bn_affine(n)
                nxt = sole_consumer(n.outputs[0])
                a, alpha = act_of(nxt) if nxt is not None else (0, 0.0)
                outs = [nxt.outputs[0]] if a else [n.outputs[0]]
                if a:
                    drop.add(id(nxt))
                out_nodes.append(Node("_AffineAct", [n.inputs[0], scale, shift], outs, {"__act": a, "__alpha": alpha},
                                      n.name))
                continue
            out_nodes.append(n)
        return self._reorder([n for n in out_nodes if id(n) not in drop])

    def _stem_conv_node(self, n: Node) -> bool:
        """A _FusedConv the few-channel stem kernel runs (f16 / bf16 GPU session, C <= 4, R, S <= 8,
        R * S * C <= 160, one group): its input affine can ride the kernel's im2col (padding stays 0)."""
        if (not _STEM_KERNEL or n.op_type != "_FusedConv" or n.inputs[1] not in self._consts or not self.gpu
                or self.compute_dtype not in (torch.float16, torch.bfloat16, torch.float32)):
            return False
        w = self._consts[n.inputs[1]]
        if self.compute_dtype == torch.float32:  # the bf16-plane fp32 stem kernel: 3 channels, S <= 7
            from ..ops.conv import f32_mode_default

            if (self.f32_conv_mode or f32_mode_default()) == "exact" or not isinstance(w, torch.Tensor) \
                    or w.dim() != 4 or w.shape[1] != 3 or w.shape[3] > 7:
                return False
        return (isinstance(w, torch.Tensor) and w.dim() == 4 and n.attrs.get("group", 1) == 1
                and 1 <= w.shape[1] <= 4 and w.shape[2] <= 8 and w.shape[3] <= 8
                and w.shape[1] * w.shape[2] * w.shape[3] <= 160 and n.attrs.get("__act", 0) in (0, 1))

    def _mfma_conv(self, n: Node) -> bool:
        """A _FusedConv the MFMA implicit-GEMM kernel runs (2-D, one group, C % 64 == 0, relu-or-none act)."""
        if n.op_type != "_FusedConv" or n.inputs[1] not in self._consts:
            return False
        w = self._consts[n.inputs[1]]
        return (isinstance(w, torch.Tensor) and w.dim() == 4 and n.attrs.get("group", 1) == 1
                and w.shape[1] % 64 == 0 and n.attrs.get("__act", 0) in (0, 1))

    def _fuse_prologues(self, nodes: List[Node]) -> List[Node]:
        """MFMA-conv fusions (GPU, channels_last; fp32 runs the exact f32-input MFMA form):

        * a per-channel BN(+ReLU) whose every consumer is an MFMA conv is applied in those convs' A-tile
          loaders (prologue) instead of being materialised — the pre-activation of ResNet-v2 blocks;
        * an ``_AddAffineAct`` whose activated output is consumed that way becomes a plain Add, which then
          folds into the producing conv's epilogue as the residual add.
        Input layout of a fused conv: [x, w, b, res, pro_scale, pro_shift]."""
        outs = {o.name for o in self.outputs}
        by_input: Dict[str, List[Node]] = {}
        for n in nodes:
            for x in n.inputs:
                by_input.setdefault(x, []).append(n)
        prod = {o: n for n in nodes for o in n.outputs}
        drop = set()

        def absorb(value: str, src: str, scale: str, shift: str, relu: bool) -> bool:
            cs = by_input.get(value, [])
            if value in outs or not cs or not all((self._mfma_conv(c) or self._stem_conv_node(c)) and c.inputs[0] == value and
                                                  c.inputs[1:].count(value) == 0 and len(c.inputs) <= 4
                                                  for c in cs):
                return False
            for c in cs:
                while len(c.inputs) < 4:
                    c.inputs.append("")
                c.inputs[0] = src
                c.inputs += [scale, shift]
                c.attrs["__pro_relu"] = 1 if relu else 0
                by_input.setdefault(src, []).append(c)
            return True

        new_nodes = []
        for n in nodes:
            if n.op_type == "_AffineAct" and n.attrs.get("__act", 0) in (0, 1):
                if absorb(n.outputs[0], n.inputs[0], n.inputs[1], n.inputs[2], n.attrs.get("__act", 0) == 1):
                    drop.add(id(n))
                    continue
            if n.op_type == "_AddAffineAct" and len(n.outputs) > 1 and n.outputs[1]:
                if absorb(n.outputs[1], n.outputs[0], n.inputs[2], n.inputs[3], n.attrs.get("__act", 0) == 1):
                    add = Node("Add", n.inputs[:2], [n.outputs[0]], {}, n.name)
                    # residual epilogue: the conv producing one addend (sole consumer, no act, no residual yet)
                    for k in (0, 1):
                        c = prod.get(add.inputs[k])
                        other = add.inputs[1 - k]
                        if (c is not None and self._mfma_conv(c) and c.attrs.get("__act", 0) == 0
                                and (len(c.inputs) < 4 or not c.inputs[3]) and c.outputs[0] not in outs
                                and len(by_input.get(c.outputs[0], [])) == 1 and other != c.outputs[0]):
                            while len(c.inputs) < 4:
                                c.inputs.append("")
                            c.inputs[3] = other
                            c.outputs = [add.outputs[0]]
                            add = None
                            break
                    if add is not None:
                        new_nodes.append(add)
                    drop.add(id(n))
                    continue
            if n.op_type == "_AddAffineAct" and n.attrs.get("__act", 0) == 1 and len(n.outputs) > 1 and n.outputs[1]:
                # activated output not consumed by MFMA convs (e.g. the last block's post-activation before the
                # pooling): the producing conv adds the residual and writes relu(y * scale + shift) as its
                # second output from registers, instead of a separate add + BN + ReLU pass
                for k in (0, 1):
                    c = prod.get(n.inputs[k])
                    other = n.inputs[1 - k]
                    if (c is not None and self._mfma_conv(c) and c.attrs.get("__act", 0) == 0
                            and len(c.inputs) <= 6 and (len(c.inputs) < 4 or not c.inputs[3])
                            and c.outputs[0] not in outs and len(by_input.get(c.outputs[0], [])) == 1
                            and other != c.outputs[0] and id(c) not in drop):
                        while len(c.inputs) < 6:
                            c.inputs.append("")
                        c.inputs[3] = other
                        c.inputs += [n.inputs[2], n.inputs[3]]
                        c.outputs = [n.outputs[0], n.outputs[1]]
                        drop.add(id(n))
                        break
                if id(n) in drop:
                    continue
            new_nodes.append(n)
        return self._reorder([n for n in new_nodes if id(n) not in drop])

    def _move_epilogue_past_pool(self, nodes: List[Node]) -> List[Node]:
        """A library conv (not the MFMA kernel, e.g. the 3-channel ResNet stem) whose bias(+ReLU) epilogue
        feeds only a MaxPool: the epilogue runs on the pooled maxima inside the pool kernel instead of as a
        full-resolution pass. Exact: x -> round(x + b) and ReLU are monotone, so they commute with max."""
        outs = {o.name for o in self.outputs}
        by_input: Dict[str, List[Node]] = {}
        for n in nodes:
            for x in n.inputs:
                by_input.setdefault(x, []).append(n)
        for n in nodes:
            if (n.op_type != "_FusedConv" or self._mfma_conv(n) or n.attrs.get("__act", 0) not in (0, 1)
                    or len(n.inputs) < 3 or not n.inputs[2] or any(n.inputs[3:]) or n.outputs[0] in outs):
                continue
            cs = by_input.get(n.outputs[0], [])
            if len(cs) != 1 or cs[0].op_type != "MaxPool" or len(cs[0].inputs) != 1 or \
                    (len(cs[0].outputs) > 1 and cs[0].outputs[1]):
                continue
            pool = cs[0]
            pool.inputs = [pool.inputs[0], n.inputs[2]]
            pool.attrs = dict(pool.attrs, __act=n.attrs.get("__act", 0))
            n.inputs = [n.inputs[0], n.inputs[1], ""]
            n.attrs["__act"] = 0
        return nodes

    def _reorder(self, nodes: List[Node]) -> List[Node]:
        """Stable topological re-order (a fused node may read a value produced
        after the node it replaced, e.g. a ResNet v1 shortcut conv)."""
        avail = set(self._consts) | {i.name for i in self.inputs} | set(self._outer) | {""}
        pending, order = list(nodes), []
        while pending:
            rest = []
            for n in pending:
                if all(x in avail for x in n.inputs):
                    order.append(n)
                    avail.update(n.outputs)
                else:
                    rest.append(n)
            if len(rest) == len(pending):
                order.extend(rest)  # subgraph outer references: keep original order
                break
            pending = rest
        return order

    def _bn_affine(self, bn: Node) -> Tuple[str, str]:
        gamma, beta, mean, var = (self._consts[x].double() for x in bn.inputs[1:5])
        s = gamma / torch.sqrt(var + bn.attrs.get("epsilon", 1e-5))
        sname, tname = bn.outputs[0] + "__scale", bn.outputs[0] + "__shift"
        self._consts[sname] = s.float()
        self._consts[tname] = (beta - mean * s).float()
        return sname, tname

    def _place_constants(self):
        """Move constants used by device ops to the device (weights in the compute dtype)."""
        weight_inputs = set()
        for n in self.nodes:
            if n.op_type in ("_FusedConv", "Conv", "ConvTranspose", "Gemm", "MatMul"):
                for x in n.inputs[1:2]:
                    if x:
                        weight_inputs.add(x)
        host_only = set()
        for n in self.nodes:
            # shape-like operands stay on the host
            if n.op_type in ("Reshape", "Expand", "Tile", "Slice", "Squeeze", "Unsqueeze", "ConstantOfShape", "Range",
                             "TopK", "Pad", "Resize", "Upsample", "Split", "OneHot", "Trilu", "CumSum"):
                for x in n.inputs[1:]:
                    host_only.add(x)
        for k, v in list(self._consts.items()):
            if not isinstance(v, torch.Tensor) or k in host_only:
                continue
            if not self.gpu:
                if k in weight_inputs and v.is_floating_point():
                    self._consts[k] = v.to(self.compute_dtype)
                continue
            if v.numel() <= 8 and not v.is_floating_point() and k not in weight_inputs:
                continue  # tiny integer constants (axes, shapes) stay on the host
            t = v.to(self.device)
            if k in weight_inputs and t.is_floating_point():
                t = t.to(self.compute_dtype)
                if self.channels_last and t.dim() == 4:
                    t = t.contiguous(memory_format=torch.channels_last)
            self._consts[k] = t

    def _plan_liveness(self):
        last: Dict[str, int] = {}
        for i, n in enumerate(self.nodes):
            for x in n.inputs:
                if x:
                    last[x] = i
            # values a subgraph (If / Loop / Scan body) reads from this scope stay alive until that node
            for v in n.attrs.values():
                if isinstance(v, Graph):
                    for x in _outer_refs(v):
                        last[x] = i
        outs = {o.name for o in self.outputs}
        self._free_after: List[List[str]] = [[] for _ in self.nodes]
        for name, i in last.items():
            if name not in outs and name not in self._consts:
                self._free_after[i].append(name)

    # ------------------------------------------------------------------ execution
    def _to_value(self, vi: Optional[ValueInfo], v):
        if isinstance(v, torch.Tensor):
            t = v
        elif isinstance(v, np.ndarray) and (v.dtype == object or v.dtype.kind in "US"):
            return v.astype(object)
        else:
            a = np.asarray(v)
            if a.dtype == object or a.dtype.kind in "US":
                return a.astype(object)
            if vi is not None and vi.kind == "tensor" and vi.elem_type in P.NP_OF and P.NP_OF[vi.elem_type] is not object:
                a = a.astype(P.NP_OF[vi.elem_type], copy=False)
            t = torch.from_numpy(a if a.flags.c_contiguous and a.flags.writeable else np.array(a, copy=True))
        if self.gpu:
            t = t.to(self.device, non_blocking=True)
        if t.is_floating_point() and t.dtype != self.compute_dtype:
            t = t.to(self.compute_dtype)
        if self.gpu and self.channels_last and t.dim() == 4:
            t = t.contiguous(memory_format=torch.channels_last)
        return t

    def run_values(self, feeds: Dict[str, Any], fetch: Optional[Sequence[str]] = None) -> List[Any]:
        vals: Dict[str, Any] = dict(self._outer)
        vals.update(self._consts)
        for vi in self.inputs:
            if vi.name in feeds:
                vals[vi.name] = self._to_value(vi, feeds[vi.name])
        for k, v in feeds.items():
            if k not in vals:
                vals[k] = self._to_value(None, v)
        self._live_values = vals
        keep = set(fetch) if fetch else ()
        for i, n in enumerate(self.nodes):
            fn = OPS.get(n.op_type) or _FUSED.get(n.op_type)
            if fn is None:
                raise NotImplementedError(f"ONNX operator {n.domain + '.' if n.domain else ''}{n.op_type} is not "
                                          f"supported")
            ins = []
            for x in n.inputs:
                if not x:
                    ins.append(None)
                    continue
                if x not in vals:
                    raise ValueError(f"missing value {x} for node {n.name} ({n.op_type})")
                ins.append(vals[x])
            res = fn(_RT(self, n), n.attrs, ins)
            for name, v in zip(n.outputs, res):
                if name:
                    vals[name] = v
            for name in self._free_after[i]:
                if name not in keep:
                    vals.pop(name, None)
        names = list(fetch) if fetch else [o.name for o in self.outputs]
        return [vals[nm] for nm in names]

    def run(self, output_names: Optional[Sequence[str]], feeds: Dict[str, Any]) -> List[Any]:
        """ORT-style ``run``: returns numpy arrays (float outputs as fp32), lists for sequences."""
        fetch = list(output_names) if output_names else [o.name for o in self.outputs]
        if self.use_graph and self._graphable(feeds):
            res = self._run_graph(feeds, fetch)
        else:
            res = self.run_values(feeds, fetch)
        return [_to_host(v) for v in res]

    def run_async(self, output_names: Optional[Sequence[str]], feeds: Dict[str, Any]) -> "_Pending":
        """``run`` whose device->host copies are queued behind the graph replay: ``.result()`` waits and
        returns what ``run`` would. The caller submits batch k+1 before collecting batch k, so the GPU
        never idles while the host turns batch k's outputs into rows."""
        fetch = list(output_names) if output_names else [o.name for o in self.outputs]
        if not self.gpu:
            return _Pending(self.run(fetch, feeds), None)
        res = self._run_graph(feeds, fetch) if self.use_graph and self._graphable(feeds) else self.run_values(feeds, fetch)
        if not all(isinstance(v, torch.Tensor) for v in res):
            return _Pending([_to_host(v) for v in res], None)
        outs = []
        for v in res:
            t = v.detach()
            if t.is_floating_point() and t.dtype != torch.float64:
                t = t.float()
            if t.dim() == 4 and not t.is_contiguous():
                t = t.contiguous()
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            outs.append(h)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return _Pending(outs, ev)

    # ------------------------------------------------------------------ HIP graphs
    def _graphable(self, feeds) -> bool:
        if any(vi.kind != "tensor" or vi.elem_type == P.STRING_T for vi in self.inputs + self.outputs):
            return False
        if any(n.op_type in ops_ext.HOST_SYNC_OPS for n in self.nodes):
            return False  # value-dependent shapes / control flow: eager (a sync inside a capture breaks it)
        return all(not (isinstance(v, np.ndarray) and v.dtype == object) for v in feeds.values())

    def _run_graph(self, feeds, fetch):
        key = tuple((k, tuple(np.shape(v)), str(getattr(v, "dtype", ""))) for k, v in sorted(feeds.items())) + \
            tuple(fetch)
        with self._graph_lock:
            entry = self._graphs.get(key)
            if entry is None:
                entry = self._capture(feeds, fetch)
                self._graphs[key] = entry
        if entry == "eager":
            return self.run_values(feeds, fetch)
        g, static_in, static_out = entry
        for k, t in static_in.items():
            v = feeds[k]
            if (t.is_floating_point() and tuple(np.shape(v)) == tuple(t.shape)
                    and (isinstance(v, torch.Tensor) and v.is_floating_point()
                         or isinstance(v, np.ndarray) and v.dtype.kind == "f")):
                # one pass straight into the captured input: host->device, dtype and layout conversion in a
                # single copy (instead of cast, channels_last copy and this copy as three passes)
                t.copy_(v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v)),
                        non_blocking=True)
            else:
                t.copy_(self._to_value(next((vi for vi in self.inputs if vi.name == k), None), v), non_blocking=True)
        g.replay()
        return [o.clone() for o in static_out]

    def _capture(self, feeds, fetch):
        try:
            static_in = {k: self._to_value(next((vi for vi in self.inputs if vi.name == k), None), v).clone()
                         for k, v in feeds.items()}
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                for _ in range(2):
                    self.run_values(static_in, fetch)
            torch.cuda.current_stream(self.device).wait_stream(s)
            g = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(g):
                static_out = self.run_values(static_in, fetch)
            if not all(isinstance(o, torch.Tensor) for o in static_out):
                return "eager"
            # a plan whose work never reached the capture stream (host-computed values, kernels on another
            # stream) records an empty graph: replaying it would hand back the capture-time buffers, so such a
            # plan runs eagerly instead
            if _graph_num_nodes(g) == 0:
                return "eager"
            g.instantiate()
            return g, static_in, static_out
        except Exception:
            torch.cuda.synchronize(self.device)
            return "eager"


_HIP = None


def _graph_num_nodes(g) -> int:
    """nodes of a captured graph (hipGraphGetNodes on the raw hipGraph_t); -1 when it cannot be queried"""
    global _HIP
    import ctypes

    try:
        if _HIP is None:
            _HIP = ctypes.CDLL("libamdhip64.so")
            _HIP.hipGraphGetNodes.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
            _HIP.hipGraphGetNodes.restype = ctypes.c_int
        n = ctypes.c_size_t(0)
        if _HIP.hipGraphGetNodes(ctypes.c_void_p(int(g.raw_cuda_graph())), None, ctypes.byref(n)) != 0:
            return -1
        return int(n.value)
    except Exception:  # noqa: BLE001 - no HIP runtime symbol / older torch: treat as unknown
        return -1


# ---------------------------------------------------------------------- fused ops
def _dtype_code(t: torch.Tensor) -> int:
    return {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[t.dtype]


def _layout(t: torch.Tensor) -> Optional[int]:
    """1 = NHWC (channels-last dense), 0 = NCHW dense, None = other."""
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last) and not t.is_contiguous():
        return 1
    if t.is_contiguous():
        return 0
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return 1
    return None


def _kernel_ok(*ts) -> bool:
    return all(t is None or (t.is_cuda and t.data_ptr() % 16 == 0 and t.dtype in (torch.float32, torch.float16,
                                                                               torch.bfloat16)) for t in ts)


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _affine_act_torch(x, scale, shift, res, act, alpha):
    shp = [1, -1] + [1] * (x.dim() - 2)
    y = x.float()
    if scale is not None:
        y = y * scale.reshape(shp).float()
    if shift is not None:
        y = y + shift.reshape(shp).float()
    if res is not None:
        y = y + res.float()
    if act == 1:
        y = torch.relu(y)
    elif act == 2:
        y = torch.nn.functional.leaky_relu(y, alpha)
    elif act == 3:
        y = torch.sigmoid(y)
    elif act == 4:
        y = torch.clamp(y, 0.0, alpha)
    return y.to(x.dtype)


def _affine_act(rt, x, scale, shift, res, act, alpha, out=None):
    nn = rt.session._nn
    if nn is not None and _kernel_ok(x, res) and x.dim() >= 2:
        lay = _layout(x)
        if res is not None and (res.shape != x.shape or _layout(res) != lay):
            res = res.contiguous(memory_format=torch.channels_last) if lay == 1 else res.contiguous()
        if lay is not None:
            y = out if out is not None else torch.empty_like(x)
            C = x.shape[1]
            HW = int(np.prod(x.shape[2:])) if x.dim() > 2 else 1
            sc = scale.to(x.device, torch.float32) if scale is not None else None
            sh = shift.to(x.device, torch.float32) if shift is not None else None
            nn.affine_act(x.data_ptr(), x.numel(), C, HW, lay, sc.data_ptr() if sc is not None else 0,
                          sh.data_ptr() if sh is not None else 0, res.data_ptr() if res is not None else 0, act,
                          float(alpha), _dtype_code(x), y.data_ptr(), _stream(x))
            return y
    return _affine_act_torch(x, scale, shift, res, act, alpha)


def _mfma_ok(rt, at, inp, w) -> bool:
    return (rt.session._nn is not None and inp.is_cuda and inp.dim() == 4
            and inp.dtype in (torch.float32, torch.float16, torch.bfloat16)
            and inp.dtype == w.dtype and w.dim() == 4 and at.get("group", 1) == 1 and inp.shape[1] % 64 == 0
            and inp.is_contiguous(memory_format=torch.channels_last) and w.permute(0, 2, 3, 1).is_contiguous()
            and at.get("__act", 0) in (0, 1) and inp.data_ptr() % 16 == 0
            and inp.numel() * inp.element_size() < 2 ** 31 and w.numel() * w.element_size() < 2 ** 31
            and w.shape[2] * w.shape[3] <= 64)


def _fused_conv(rt, at, x):
    inp, w, b = x[0], x[1], x[2]
    res = x[3] if len(x) > 3 else None
    pro = (x[4], x[5]) if len(x) > 5 and x[4] is not None else None
    post = (x[6], x[7]) if len(x) > 7 and x[6] is not None else None  # second output relu(y * s + t)
    if inp.dtype != w.dtype:
        inp = inp.to(w.dtype)
    act = at.get("__act", 0)
    if _mfma_ok(rt, at, inp, w):
        from ..ops.conv import conv2d_nhwc

        nd, strides, dil, pb, pe = conv_args(at, inp.shape, w.shape)
        if res is not None:
            res = res.to(inp.dtype).contiguous(memory_format=torch.channels_last)
        dev = inp.device
        f32 = lambda t: None if t is None else t.to(dev, torch.float32).contiguous()  # noqa: E731
        wp = w.permute(0, 2, 3, 1)
        planes = None
        if inp.dtype == torch.float32:
            from ..ops.conv import f32_mode_default, split_weight

            mode = rt.session.f32_conv_mode or f32_mode_default()
            if mode != "exact":  # fp32 weights split into bf16 planes once per model (the kernel reads them)
                cache = rt.session.__dict__.setdefault("_w_planes", {})
                key = (w.data_ptr(), tuple(w.shape), mode)
                planes = cache.get(key)
                if planes is None:
                    planes = cache[key] = split_weight(wp, mode)
        y = conv2d_nhwc(inp, wp, w.shape[2], w.shape[3], strides, (pb[0], pb[1], pe[0], pe[1]),
                        dil, bias=f32(b), relu=2 if act == 1 else 0, w_planes=planes,
                        in_affine=(f32(pro[0]), f32(pro[1])) if pro is not None else None,
                        in_relu=bool(at.get("__pro_relu", 1)), res=res,
                        out_affine=(f32(post[0]), f32(post[1])) if post is not None else None,
                        f32_mode=rt.session.f32_conv_mode)
        return list(y) if post is not None else [y]
    if _STEM_KERNEL and (_stem_kernel_ok(rt, at, inp, w) or _stem_f32_ok(rt, at, inp, w)):
        ys = [_stem_kernel_conv(rt, at, inp, w, b, res, act, pro)]
        if post is not None:
            return ys + [_affine_act(rt, ys[0], post[0], post[1], None, 1, 0.0)]
        return ys
    if _STEM_MFMA and pro is None and post is None and _stem_ok(rt, at, inp, w):
        return [_stem_conv(rt, at, inp, w, b, res, act)]
    ys = _fused_conv_fallback(rt, at, inp, w, b, res, pro, act)
    if post is not None:
        return ys + [_affine_act(rt, ys[0], post[0], post[1], None, 1, 0.0)]
    return ys


# The few-channel image stem (C <= 4, R * S * C <= 160, f16 / bf16) runs on its dedicated kernel (im2col rows
# built in LDS from the input's contiguous (s, c) runs, K padded to 160): csrc/nn/conv_mfma.hip
# stem_conv_kernel. SML_STEM_KERNEL=0 falls back to the generic implicit-GEMM gather.
_STEM_KERNEL = os.environ.get("SML_STEM_KERNEL", "1") != "0"


def _stem_kernel_ok(rt, at, inp, w) -> bool:
    from ..ops.conv import stem_supported

    return (rt.session._nn is not None and inp.dim() == 4 and inp.dtype == w.dtype and at.get("group", 1) == 1
            and at.get("__act", 0) in (0, 1) and stem_supported(inp, w)
            and inp.numel() * inp.element_size() < 2 ** 31)


def _stem_f32_mode(rt) -> str:
    from ..ops.conv import f32_mode_default

    return rt.session.f32_conv_mode or f32_mode_default()


def _stem_f32_ok(rt, at, inp, w) -> bool:
    """The 3-channel stem of an fp32 graph in a bf16-plane mode (bf16x3 / bf16x6; "exact" keeps the exact-f32
    gather GEMM): csrc/nn/conv_mfma.hip stem_f32_kernel, the input affine fused, for the row-staged geometry."""
    if rt.session._nn is None or inp.dtype != torch.float32 or w.dtype != torch.float32 or inp.dim() != 4:
        return False
    if at.get("group", 1) != 1 or at.get("__act", 0) not in (0, 1) or w.dim() != 4:
        return False
    mode = _stem_f32_mode(rt)
    if mode == "exact":
        return False
    from ..ops.conv import stem_f32_supported

    if not inp.is_contiguous(memory_format=torch.channels_last):
        return False
    nd, strides, dil, pb, pe = conv_args(at, inp.shape, w.shape)
    return stem_f32_supported(inp, w, strides, (pb[0], pb[1], pe[0], pe[1]), dil, mode)


def _stem_kernel_conv(rt, at, inp, w, b, res, act, pro=None):
    from ..ops.conv import _PLANES, pack_stem_weight, pack_stem_weight_f32, stem_conv_nhwc, stem_ring_ok

    cache = rt.session.__dict__.setdefault("_stem_wk", {})
    f32 = inp.dtype == torch.float32
    mode = _stem_f32_mode(rt) if f32 else None
    nd, strides, dil, pb, pe = conv_args(at, inp.shape, w.shape)
    if not inp.is_contiguous(memory_format=torch.channels_last):
        inp = inp.contiguous(memory_format=torch.channels_last)
    # the strip form (row-run K order) where it applies: stride-2 RGB stems
    wide = stem_ring_ok(inp, w, strides, (pb[0], pb[1], pe[0], pe[1]), dil, _PLANES[mode] if f32 else 1)
    key = (w.data_ptr(), tuple(w.shape), w.dtype, mode, wide)
    wk = cache.get(key)
    if wk is None:  # packed (fp32: and split into bf16 planes) once per weight
        wk = cache[key] = pack_stem_weight_f32(w, mode, wide) if f32 else pack_stem_weight(w, wide=True if wide else None)
    return stem_conv_nhwc(inp, wk, w.shape[2], w.shape[3], strides, (pb[0], pb[1], pe[0], pe[1]), dil,
                          bias=b, relu=2 if act == 1 else 0, res=res, in_affine=pro,
                          in_relu=bool(at.get("__pro_relu", 1)))


# SML_STEM_MFMA=1: run the 3-channel stem on the packed MFMA form. Off by default: ResNet-50 fp16 measured
# 39.7k -> 38.0k img/s with it (profiles/r2_s3/stem/: the zero-padded 4-channel input copy and the 256-wide
# padded K cost more than MIOpen's stem kernel saves).
_STEM_MFMA = os.environ.get("SML_STEM_MFMA", "0") == "1"


def _stem_ok(rt, at, inp, w) -> bool:
    """A few-channel conv (the 3-channel image stem) the MFMA kernel runs in its packed form: C <= 4 and
    R, S <= 8 zero-padded to [Cout][8][8][4], input padded to 4 channels."""
    return (rt.session._nn is not None and inp.is_cuda and inp.dim() == 4 and inp.dtype in (torch.float16, torch.bfloat16)
            and inp.dtype == w.dtype and w.dim() == 4 and at.get("group", 1) == 1 and 1 <= inp.shape[1] <= 4
            and w.shape[2] <= 8 and w.shape[3] <= 8 and at.get("__act", 0) in (0, 1)
            and list(at.get("dilations", [1, 1])) == [1, 1] and inp.numel() // inp.shape[1] * 4 * 2 < 2 ** 31)


def _stem_conv(rt, at, inp, w, b, res, act):
    from ..ops.conv import conv2d_nhwc

    B, C, H, W = inp.shape
    cache = rt.session.__dict__.setdefault("_stem_w", {})
    key = (w.data_ptr(), tuple(w.shape), w.dtype)
    wp = cache.get(key)
    if wp is None:  # packed once per weight: [Cout][8][8][4], zero taps / channels
        wp = torch.zeros((w.shape[0], 8, 8, 4), dtype=w.dtype, device=w.device)
        wp[:, :w.shape[2], :w.shape[3], :C] = w.permute(0, 2, 3, 1)
        cache[key] = wp
    x4 = torch.empty((B, 4, H, W), dtype=inp.dtype, device=inp.device, memory_format=torch.channels_last).zero_()
    x4[:, :C] = inp
    nd, strides, dil, pb, pe = conv_args(at, inp.shape, w.shape)
    # the 8-tap window is one row / column longer than the real one: one more (virtual) padding row and
    # column at the far side gives the real output size; the extra taps have zero weights
    pad = (pb[0], pb[1], pe[0] + 8 - w.shape[2], pe[1] + 8 - w.shape[3])
    dev = inp.device
    if res is not None:
        res = res.to(inp.dtype).contiguous(memory_format=torch.channels_last)
    return conv2d_nhwc(x4, wp, 8, 8, strides, pad, (1, 1), bias=None if b is None else b.to(dev, torch.float32).contiguous(),
                       relu=2 if act == 1 else 0, res=res, kernel=1)


def _general_conv_ok(rt, at, inp, w) -> bool:
    """2-D convs outside the tiled MFMA kernel's domain (any channel count, grouped / depthwise) that the
    GEMM-with-im2col or direct NHWC kernels run (ops.conv.conv2d_nhwc_general)."""
    return (rt.session._nn is not None and inp.is_cuda and inp.dim() == 4 and w.dim() == 4
            and inp.dtype in (torch.float32, torch.float16, torch.bfloat16) and inp.dtype == w.dtype
            and at.get("__act", 0) in (0, 1) and inp.numel() * inp.element_size() < 2 ** 31
            and inp.shape[1] % at.get("group", 1) == 0)


def _packed_weight(rt, w):
    """[Cout, Cg, R, S] -> contiguous [Cout, R, S, Cg], packed once per weight tensor."""
    cache = rt.session.__dict__.setdefault("_wpack", {})
    key = (w.data_ptr(), tuple(w.shape), w.dtype)
    wp = cache.get(key)
    if wp is None:
        wp = cache[key] = w.permute(0, 2, 3, 1).contiguous()
    return wp


def _fused_conv_fallback(rt, at, inp, w, b, res, pro, act):
    if pro is not None:  # prologue outside the kernel (fallback path)
        inp = _affine_act(rt, inp, pro[0], pro[1], None, 1 if at.get("__pro_relu", 1) else 0, 0.0)
    if _general_conv_ok(rt, at, inp, w):
        from ..ops.conv import conv2d_nhwc_general

        nd, strides, dil, pb, pe = conv_args(at, inp.shape, w.shape)
        return [conv2d_nhwc_general(inp, _packed_weight(rt, w), w.shape[2], w.shape[3], strides,
                                    (pb[0], pb[1], pe[0], pe[1]), dil, groups=at.get("group", 1), bias=b,
                                    relu=2 if act == 1 else 0, res=res)]
    nd, strides, dil, pb, pe = conv_args(at, inp.shape, w.shape)
    inp, pad = _sym_pad(inp, pb, pe)
    f = {1: torch.nn.functional.conv1d, 2: torch.nn.functional.conv2d, 3: torch.nn.functional.conv3d}[nd]
    if rt.session._nn is None:
        # host path: bias inside the conv, epilogue as torch ops
        y = f(inp, w, b.to(w.dtype) if b is not None else None, stride=strides, padding=pad, dilation=dil,
              groups=at.get("group", 1))
        if res is not None or act:
            y = _affine_act_torch(y, None, None, res.to(y.dtype) if res is not None else None, act,
                                  at.get("__alpha", 0.0))
        return [y]
    y = f(inp, w, None, stride=strides, padding=pad, dilation=dil, groups=at.get("group", 1))
    if b is None and res is None and not act:
        return [y]
    if res is not None and res.dtype != y.dtype:
        res = res.to(y.dtype)
    return [_affine_act(rt, y, None, b, res, act, at.get("__alpha", 0.0), out=y)]


def _fused_affine_act(rt, at, x):
    t = x[0]
    if not t.is_floating_point():
        t = t.float()
    return [_affine_act(rt, t, x[1], x[2], None, at.get("__act", 0), at.get("__alpha", 0.0))]


def _fused_add_affine_act(rt, at, x):
    a, b, scale, shift = x
    a, b = (a, b.to(a.dtype)) if a.dtype == b.dtype or not b.is_floating_point() else (a, b.to(a.dtype))
    act = at.get("__act", 0)
    nn = rt.session._nn
    if nn is not None and a.shape == b.shape and _kernel_ok(a, b):
        lay = _layout(a)
        if _layout(b) != lay:
            b = b.contiguous(memory_format=torch.channels_last) if lay == 1 else b.contiguous()
        if lay is not None:
            s = torch.empty_like(a)
            y = torch.empty_like(a)
            C = a.shape[1]
            HW = int(np.prod(a.shape[2:])) if a.dim() > 2 else 1
            sc = scale.to(a.device, torch.float32)
            sh = shift.to(a.device, torch.float32)
            nn.add_affine_act(a.data_ptr(), b.data_ptr(), a.numel(), C, HW, lay, sc.data_ptr(), sh.data_ptr(), act,
                              _dtype_code(a), s.data_ptr(), y.data_ptr(), _stream(a))
            return [s, y]
    s = a + b
    return [s, _affine_act_torch(s, scale, shift, None, act, 0.0)]


_FUSED = {"_FusedConv": _fused_conv, "_AffineAct": _fused_affine_act, "_AddAffineAct": _fused_add_affine_act}


def _numel(v) -> int:
    if isinstance(v, torch.Tensor):
        return v.numel()
    return int(np.asarray(v).size)


def _scalar(v):
    if v is None:
        return None
    return float(v.reshape(-1)[0]) if isinstance(v, torch.Tensor) else float(np.asarray(v).reshape(-1)[0])


class _Pending:
    """Outputs of ``run_async``: pinned host tensors filled by queued copies (or ready values)."""

    def __init__(self, outs, event):
        self._outs, self._event = outs, event

    def result(self) -> List[Any]:
        if self._event is None:
            return self._outs
        self._event.synchronize()
        # copy out of page-locked memory so the staging buffers go back to the pinned pool
        return [np.array(h.numpy()) for h in self._outs]


def _to_host(v):
    if isinstance(v, torch.Tensor):
        t = v.detach()
        if t.is_floating_point() and t.dtype != torch.float64:
            t = t.float()
        if t.dim() == 4 and not t.is_contiguous():
            t = t.contiguous()
        return t.cpu().numpy()
    return v
