#!/usr/bin/env python3
"""ResNet-50 (ONNX model-zoo v2 topology, random-init weights) inference
throughput on one GPU: (1) session only, device-resident input, per precision
and batch; (2) ImageFeaturizer end to end from ENCODED JPEG bytes (native
multi-threaded JPEG decode into pinned memory running ahead of the device -
or PIL with SML_NATIVE_JPEG=0 / --decoders pil - fused resize/crop/normalize
kernel, featurization) and, for reference, from pre-decoded image rows —
BASELINE.json config "ONNXModel ResNet-50, synthetic 224x224 images".
Precision is reported per line; fp32 is the reference's precision."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="32,128")
    ap.add_argument("--precisions", default="fp32,fp16,bf16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--images", type=int, default=512)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--decoders", default="native", help="comma list of native,pil for the JPEG e2e runs")
    a = ap.parse_args()
    import torch

    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.image import make_image_row
    from synapseml_amd.onnx import ImageFeaturizer, InferenceSession, writer

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    model = writer.resnet50_v2(seed=0)
    for prec in a.precisions.split(","):
        sess = InferenceSession(model, device=dev, precision=prec, use_graph=not a.no_graph)
        for bs in [int(b) for b in a.batches.split(",")]:
            x = torch.rand(bs, 3, 224, 224, device=dev)
            for _ in range(3):
                sess.run(None, {"data": x})
            if dev == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                if a.no_graph or dev == "cpu":
                    out = sess.run_values({"data": x})
                else:
                    out = sess._run_graph({"data": x}, [o.name for o in sess.outputs])
            if dev == "cuda":
                torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.iters
            print(json.dumps({"bench": "resnet50_session", "precision": prec, "batch": bs, "ms_per_batch": dt * 1e3,
                              "images_per_s": bs / dt, "hip_graph": not a.no_graph and dev == "cuda"}), flush=True)
    # end to end featurizer: JPEG bytes (decode included) and pre-decoded rows, fused preprocess, headless features
    if a.images <= 0:
        return
    import io as _io

    from PIL import Image

    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:256, 0:256]
    jpegs = np.empty(a.images, dtype=object)
    rows = np.empty(a.images, dtype=object)
    for i in range(a.images):
        # smooth colour fields + noise: JPEG sizes like photos (~20-40 KB at 256x256, quality 90)
        base = np.stack([(xx * (1 + i % 3) + yy) % 256, (yy * 2 + i) % 256, (xx + 2 * yy + 3 * i) % 256], -1)
        img = np.clip(base + rng.normal(0, 12, base.shape), 0, 255).astype(np.uint8)
        buf = _io.BytesIO()
        Image.fromarray(img).save(buf, format="JPEG", quality=90)
        jpegs[i] = buf.getvalue()
        rows[i] = make_image_row(img[:, :, ::-1].copy())
    avg_kb = float(np.mean([len(b) for b in jpegs])) / 1024
    runs = [("jpeg_bytes", jpegs, d) for d in a.decoders.split(",")] + [("decoded_rows", rows, None)]
    for src, col, decoder in runs:
        df = DataFrame({"image": col})
        if decoder is not None:
            os.environ["SML_NATIVE_JPEG"] = "1" if decoder == "native" else "0"
        for prec in ("fp32", "fp16"):
            f = ImageFeaturizer(inputCol="image", outputCol="features", featureTensorName="resnetv24_pool1_fwd",
                                imageTensorName="data").setModel(model)
            f.getOnnxModel().setPrecision(prec).setMiniBatchSize(128)
            f.transform(df.limit(128))  # warm-up / graph capture
            if dev == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = f.transform(df)
            dt = time.perf_counter() - t0
            assert out.count() == a.images
            print(json.dumps({"bench": "image_featurizer_e2e", "input": src, "decode_included": src == "jpeg_bytes",
                              "decoder": decoder,
                              "jpeg_kb_avg": round(avg_kb, 1) if src == "jpeg_bytes" else None,
                              "precision": prec, "images": a.images, "images_per_s": a.images / dt, "s": dt}),
                  flush=True)


if __name__ == "__main__":
    main()
