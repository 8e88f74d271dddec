"""Legacy ``CNTKModel`` (reference: deep-learning/src/main/python/synapse/ml/cntk/CNTKModel.py, a shim whose
CNTK runtime was removed from the reference). CNTK has no ROCm runtime; this class keeps the shim's API -
input / output node by index or name, input / output column, mini-batch size, model location, rebroadcast,
input shapes - and runs models exported to ONNX (CNTK's own ``save(format=ONNX)``) on the ONNX executor.
As in the shim, every node / column setter rewrites the feed / fetch dictionaries. Native CNTK v2 model
bytes are rejected with an explicit error naming the export route."""
from __future__ import annotations

from typing import List

from ..core.params import Param, TypeConverters as T
from ..onnx.model import ONNXModel


class CNTKModel(ONNXModel):
    inputNode = Param("index of the input node", 0, T.toInt)
    inputNodeName = Param("name of the input node (overrides inputNode)", None, T.toString)
    outputNodeIndex = Param("index of the output node", 0, T.toInt)
    outputNodeName = Param("name of the output node to fetch", None, T.toString)
    inputCol = Param("input column", "features", T.toString)
    outputCol = Param("output column", "output", T.toString)

    def setModelLocation(self, path: str):  # noqa: N802
        with open(path, "rb") as f:
            head = f.read(16)
        if head[:2] == b"\x08\x01" or head[:1] == b"\x08":
            super().setModelLocation(path)
            self._update_feed()
            self._update_fetch()
            return self
        raise NotImplementedError("native CNTK models cannot run on ROCm; export the model to ONNX "
                                  "(cntk.Function.save(path, format=C.ModelFormat.ONNX)) and load that file")

    # ---------------------------------------------------------- the shim's feed / fetch bookkeeping
    def _loaded(self) -> bool:
        try:
            return bool(self.getModelPayload())
        except Exception:  # noqa: BLE001 - no model set yet
            return False

    def _input_name(self) -> str:
        names = list(self.modelInput)
        if self.getInputNodeName():
            if self.getInputNodeName() not in names:
                raise ValueError(f"input node {self.getInputNodeName()!r} not in the model inputs {names}")
            return self.getInputNodeName()
        return names[self.getInputNode()]

    def _output_name(self) -> str:
        names = list(self.modelOutput)
        if self.getOutputNodeName():
            if self.getOutputNodeName() not in names:
                raise ValueError(f"output node {self.getOutputNodeName()!r} not in the model outputs {names}")
            return self.getOutputNodeName()
        return names[self.getOutputNodeIndex()]

    def _update_feed(self):
        if self._loaded():
            self.setFeedDict({self._input_name(): self.getInputCol()})

    def _update_fetch(self):
        if self._loaded():
            self.setFetchDict({self.getOutputCol(): self._output_name()})

    def setInputNodeIndex(self, n: int):  # noqa: N802
        self.set("inputNode", int(n))
        self.set("inputNodeName", None)
        self._update_feed()
        return self

    def getInputNodeIndex(self) -> int:  # noqa: N802
        return self.getInputNode()

    def setInputNode(self, n):  # noqa: N802
        """by index (int) or by node name (str), as the shim's overloads"""
        if isinstance(n, str):
            self.set("inputNodeName", n)
        else:
            self.set("inputNode", int(n))
            self.set("inputNodeName", None)
        self._update_feed()
        return self

    def setInputCol(self, c: str):  # noqa: N802
        self.set("inputCol", c)
        self._update_feed()
        return self

    def setOutputNodeIndex(self, n: int):  # noqa: N802
        self.set("outputNodeIndex", int(n))
        self.set("outputNodeName", None)
        self._update_fetch()
        return self

    def setOutputNode(self, n):  # noqa: N802
        if isinstance(n, str):
            self.set("outputNodeName", n)
        else:
            self.set("outputNodeIndex", int(n))
            self.set("outputNodeName", None)
        self._update_fetch()
        return self

    def getOutputNode(self):  # noqa: N802
        return self.getOutputNodeName() or self.getOutputNodeIndex()

    def setOutputCol(self, c: str):  # noqa: N802
        self.set("outputCol", c)
        self._update_fetch()
        return self

    def getInputShapes(self) -> List[List]:  # noqa: N802
        return [list(vi.shape or []) for vi in self.modelInput.values()]

    def setMiniBatchSize(self, n: int):  # noqa: N802
        self.set("miniBatchSize", int(n))
        return self

    def rebroadcastCNTKModel(self, sparkSession=None):  # noqa: N802, N803
        """the model bytes live in the stage itself (one device copy per executor process); nothing to
        re-broadcast - kept for API compatibility"""
        return self

    def _transform(self, df):
        if not self.getFeedDict():
            self._update_feed()
        if not self.getFetchDict():
            self._update_fetch()
        return super()._transform(df)


__all__ = ["CNTKModel"]
