"""ONNX graph IR: decoded ``ModelProto`` → nodes with Python attribute values,
initializers as numpy arrays, typed input/output infos; topological order,
slicing at intermediate outputs, and re-serialisation.

Slicing mirrors the reference's ``sliceModelAtOutputs`` (DFS from the
requested outputs back to the inputs, keeping only needed nodes and
initializers; ONNXUtils.scala:267-370)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Iterable, Any, Dict, List, Optional, Sequence

import numpy as np

from . import proto as P


@dataclass
class ValueInfo:
    name: str
    kind: str = "tensor"               # tensor | sequence | map
    elem_type: int = P.FLOAT32         # tensor element type (or map value elem type)
    shape: Optional[List[Any]] = None  # ints, strings (symbolic) or None
    key_type: int = 0                  # map key type / sequence(map) key type
    seq_of_maps: bool = False

    @property
    def np_dtype(self):
        return P.NP_OF.get(self.elem_type, np.float32)

    def describe(self) -> str:
        if self.kind == "tensor":
            return f"{self.name}: tensor({np.dtype(self.np_dtype).name if self.np_dtype is not object else 'string'})" \
                   f"{self.shape}"
        return f"{self.name}: {self.kind}"


@dataclass
class Node:
    op_type: str
    inputs: List[str]
    outputs: List[str]
    attrs: Dict[str, Any] = field(default_factory=dict)
    name: str = ""
    domain: str = ""


def _attr_value(a: P.Message):
    t = a.type
    if t == P.A_FLOAT:
        return float(a.f)
    if t == P.A_INT:
        return int(a.i)
    if t == P.A_STRING:
        return a.s.decode("utf-8", errors="replace")
    if t == P.A_TENSOR:
        return P.tensor_to_numpy(a.t)
    if t == P.A_GRAPH:
        return Graph.from_proto(a.g)
    if t == P.A_FLOATS:
        return [float(x) for x in a.floats]
    if t == P.A_INTS:
        return [int(x) for x in a.ints]
    if t == P.A_STRINGS:
        return [s.decode("utf-8", errors="replace") for s in a.strings]
    if t == P.A_TENSORS:
        return [P.tensor_to_numpy(x) for x in a.tensors]
    # untyped (old exporters): infer from the populated field
    if a.ints:
        return [int(x) for x in a.ints]
    if a.floats:
        return [float(x) for x in a.floats]
    if a.strings:
        return [s.decode("utf-8") for s in a.strings]
    if a.s:
        return a.s.decode("utf-8")
    if a.t is not None:
        return P.tensor_to_numpy(a.t)
    if a.f:
        return float(a.f)
    return int(a.i)


def _value_info(v: P.Message) -> ValueInfo:
    vi = ValueInfo(v.name)
    tp = v.type
    if tp is None:
        return vi
    if tp.tensor_type is not None:
        tt = tp.tensor_type
        vi.elem_type = tt.elem_type
        if tt.shape is not None:
            vi.shape = [d.dim_param if d.dim_param else (int(d.dim_value) if d.dim_value > 0 else None)
                        for d in tt.shape.dim]
    elif tp.sequence_type is not None:
        vi.kind = "sequence"
        et = tp.sequence_type.elem_type
        if et is not None and et.map_type is not None:
            vi.seq_of_maps = True
            vi.key_type = et.map_type.key_type
            vt = et.map_type.value_type
            vi.elem_type = vt.tensor_type.elem_type if vt is not None and vt.tensor_type is not None else P.FLOAT32
        elif et is not None and et.tensor_type is not None:
            vi.elem_type = et.tensor_type.elem_type
    elif tp.map_type is not None:
        vi.kind = "map"
        vi.key_type = tp.map_type.key_type
        vt = tp.map_type.value_type
        vi.elem_type = vt.tensor_type.elem_type if vt is not None and vt.tensor_type is not None else P.FLOAT32
    return vi


class Graph:
    def __init__(self):
        self.name = ""
        self.nodes: List[Node] = []
        self.initializers: Dict[str, np.ndarray] = {}
        self.inputs: List[ValueInfo] = []
        self.outputs: List[ValueInfo] = []
        self.value_info: Dict[str, ValueInfo] = {}
        self.opset: Dict[str, int] = {"": 13}
        self.ir_version = 7
        self.producer = ""

    # -------------------------------------------------------------- io
    @staticmethod
    def from_proto(g: P.Message) -> "Graph":
        gr = Graph()
        gr.name = g.name
        for t in g.initializer:
            gr.initializers[t.name] = P.tensor_to_numpy(t)
        for n in g.node:
            gr.nodes.append(Node(n.op_type, list(n.input), list(n.output),
                                 {a.name: _attr_value(a) for a in n.attribute}, n.name, n.domain))
        gr.inputs = [_value_info(v) for v in g.input if v.name not in gr.initializers]
        gr.outputs = [_value_info(v) for v in g.output]
        for v in g.value_info:
            gr.value_info[v.name] = _value_info(v)
        for v in list(gr.inputs) + list(gr.outputs):
            gr.value_info[v.name] = v
        return gr

    @staticmethod
    def from_bytes(data: bytes) -> "Graph":
        m = P.load_model(data)
        if m.graph is None:
            raise ValueError("ONNX model has no graph")
        g = Graph.from_proto(m.graph)
        g.opset = {o.domain: int(o.version) for o in m.opset_import} or {"": 13}
        g.ir_version = int(m.ir_version) or 7
        g.producer = m.producer_name
        return g

    def to_bytes(self) -> bytes:
        from .writer import make_graph, make_model

        gp = make_graph(self.nodes, self.name or "graph", self.inputs, self.outputs,
                        initializers=self.initializers, value_info=[v for k, v in self.value_info.items()
                                                                    if k not in {i.name for i in self.inputs}
                                                                    and k not in {o.name for o in self.outputs}])
        return P.encode(make_model(gp, opset=self.opset, ir_version=self.ir_version, producer=self.producer))

    # -------------------------------------------------------------- analysis
    def producers(self) -> Dict[str, int]:
        return {o: i for i, n in enumerate(self.nodes) for o in n.outputs if o}

    def consumers(self) -> Dict[str, List[int]]:
        out: Dict[str, List[int]] = {}
        for i, n in enumerate(self.nodes):
            for x in n.inputs:
                if x:
                    out.setdefault(x, []).append(i)
            for sub in _subgraphs(n):
                for x in sub.outer_refs():
                    out.setdefault(x, []).append(i)
        return out

    def outer_refs(self) -> List[str]:
        """Names a (sub)graph reads but does not define."""
        defined = set(self.initializers) | {i.name for i in self.inputs}
        refs = []
        for n in self.nodes:
            for x in n.inputs:
                if x and x not in defined:
                    refs.append(x)
            for sub in _subgraphs(n):
                refs += [r for r in sub.outer_refs() if r not in defined]
            defined.update(n.outputs)
        return refs

    def toposort(self, outer: Iterable[str] = ()) -> List[Node]:
        """nodes in dependency order; `outer`: names a subgraph may read from its enclosing scope"""
        avail = set(self.initializers) | {i.name for i in self.inputs} | {""} | set(outer)
        pending = list(self.nodes)
        order: List[Node] = []
        while pending:
            progressed = False
            rest = []
            for n in pending:
                needs = [x for x in n.inputs if x] + [r for s in _subgraphs(n) for r in s.outer_refs()]
                if all(x in avail for x in needs):
                    order.append(n)
                    avail.update(n.outputs)
                    progressed = True
                else:
                    rest.append(n)
            if not progressed:
                missing = sorted({x for n in rest for x in n.inputs if x and x not in avail})
                raise ValueError(f"graph has a cycle or undefined inputs: {missing[:10]}")
            pending = rest
        return order

    def slice_at(self, outputs: Sequence[str]) -> "Graph":
        """Sub-graph computing ``outputs`` (ONNXUtils.sliceModelAtOutputs)."""
        prod = self.producers()
        known = set(prod) | set(self.initializers) | {i.name for i in self.inputs}
        for o in outputs:
            if o not in known:
                raise ValueError(f"output {o} is not produced by the graph")
        keep_nodes = set()
        stack = list(outputs)
        seen = set()
        while stack:
            v = stack.pop()
            if v in seen or not v:
                continue
            seen.add(v)
            if v in prod:
                i = prod[v]
                if i not in keep_nodes:
                    keep_nodes.add(i)
                    n = self.nodes[i]
                    stack.extend(n.inputs)
                    for s in _subgraphs(n):
                        stack.extend(s.outer_refs())
        g = Graph()
        g.name = self.name
        g.opset = dict(self.opset)
        g.ir_version = self.ir_version
        g.producer = self.producer
        g.nodes = [n for i, n in enumerate(self.nodes) if i in keep_nodes]
        g.initializers = {k: v for k, v in self.initializers.items() if k in seen}
        g.inputs = [i for i in self.inputs if i.name in seen]
        g.outputs = [self.value_info.get(o) or ValueInfo(o) for o in outputs]
        g.value_info = {k: v for k, v in self.value_info.items() if k in seen}
        for o in g.outputs:
            g.value_info[o.name] = o
        return g


def _subgraphs(n: Node) -> List[Graph]:
    out = []
    for v in n.attrs.values():
        if isinstance(v, Graph):
            out.append(v)
        elif isinstance(v, list) and v and isinstance(v[0], Graph):
            out.extend(v)
    return out
