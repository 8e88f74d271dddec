"""ONNXModel.transform on a DataFrame of 4096 synthetic 3x224x224 float tensors (tools/bench_onnx_dp.py's data),
fp32 and fp16 at mini-batch 256: img/s of a timed transform, then a cProfile of one more. One MI355X."""
import cProfile
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.onnx import ONNXModel, writer

    payload = writer.resnet50_v2(seed=0)
    imgs = np.random.default_rng(0).random((4096, 3, 224, 224), dtype=np.float32)
    df = DataFrame({"data": imgs})
    for prec in ("fp32", "fp16"):
        m = (ONNXModel().setModelPayload(payload).setDeviceType("GPU").setPrecision(prec)
             .setFeedDict({"data": "data"}).setFetchDict({"logits": "resnetv24_dense0_fwd"})
             .setArgMaxDict({"logits": "label"}).setMiniBatchSize(256))
        m.transform(df.limit(256))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.transform(df)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"precision": prec, "img_per_s": round(4096 / dt, 1), "s": round(dt, 3)}), flush=True)
        pr = cProfile.Profile()
        pr.enable()
        m.transform(df)
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
