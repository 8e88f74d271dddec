"""Legacy ``CNTKModel`` (reference: deep-learning/src/main/python/synapse/ml/cntk/CNTKModel.py, a shim over
the removed CNTK runtime). CNTK has no ROCm runtime; this class keeps the API and runs models that were
exported to ONNX (CNTK's own ``save(format=ONNX)``) through the ONNX executor. Native CNTK v2 model bytes are
rejected with an explicit error."""
from __future__ import annotations

from ..core.params import Param, TypeConverters as T
from ..onnx.model import ONNXModel


class CNTKModel(ONNXModel):
    inputNode = Param("index of the input node", 0, T.toInt)
    outputNodeName = Param("name of the output node to fetch", None, T.toString)
    inputCol = Param("input column", "features", T.toString)
    outputCol = Param("output column", "output", T.toString)

    def setModelLocation(self, path: str):  # noqa: N802
        with open(path, "rb") as f:
            head = f.read(16)
        if head[:2] == b"\x08\x01" or head[:1] == b"\x08":
            return super().setModelLocation(path)
        raise NotImplementedError("native CNTK models cannot run on ROCm; export the model to ONNX "
                                  "(cntk.Function.save(path, format=C.ModelFormat.ONNX)) and load that file")

    def _transform(self, df):
        names = self.modelInput()
        outs = self.modelOutput()
        if not self.getFeedDict():
            self.setFeedDict({list(names)[self.getInputNode()]: self.getInputCol()})
        if not self.getFetchDict():
            fetch = self.getOutputNodeName() or list(outs)[0]
            self.setFetchDict({self.getOutputCol(): fetch})
        return super()._transform(df)


__all__ = ["CNTKModel"]
