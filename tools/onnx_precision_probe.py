"""Relative error of the GPU ResNet-50 session (fp32 / fp16 / bf16) against the fp32 host graph: the
measurement behind the tolerances in tests/test_onnx.py."""
import os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from synapseml_amd.onnx import InferenceSession, writer
data = writer.resnet50_v2(seed=13)
x = np.random.default_rng(14).random((8, 3, 224, 224), dtype=np.float32)
cpu = InferenceSession(data, device="cpu").run(None, {"data": x})[0].astype(np.float64)
for prec in ["fp32", "fp16", "bf16"]:
    out = InferenceSession(data, device="cuda", precision=prec).run(None, {"data": x})[0].astype(np.float64)
    rel = np.linalg.norm(out - cpu) / np.linalg.norm(cpu)
    mx = np.abs(out - cpu).max() / np.abs(cpu).max()
    top1 = (out.argmax(1) == cpu.argmax(1)).mean()
    print(prec, "relL2", rel, "maxrel", mx, "top1", top1, flush=True)
data = writer.resnet50_v2(seed=7)
x = np.random.default_rng(8).random((2, 3, 224, 224), dtype=np.float32)
cpu = InferenceSession(data, device="cpu").run(None, {"data": x})[0]
out = InferenceSession(data, device="cuda").run(None, {"data": x})[0]
print("seed7 fp32 maxrel", np.abs(out - cpu).max() / np.abs(cpu).max())
