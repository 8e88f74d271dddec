"""onnx package."""
