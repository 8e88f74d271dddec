#!/usr/bin/env python3
"""ImageTransformer throughput: resize(256, 256).centerCrop(224, 224) on a DataFrame of 512x512 BGR image rows
(the reference's OpenCV ImageTransformer stages, ImageTransformer.scala:68-283), device vs host, plus the same
list followed by toTensor (normalize). img/s of the whole transform call, DataFrame in / DataFrame out.

usage: python tools/bench_image.py [--images 1024] [--reps 3]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--size", type=int, default=512)
    args = ap.parse_args()
    from synapseml_amd.core import DataFrame
    from synapseml_amd.image import ImageTransformer
    from synapseml_amd.image.schema import make_image_row

    rng = np.random.default_rng(0)
    base = rng.integers(0, 256, (16, args.size, args.size, 3), dtype=np.uint8)
    rows = [make_image_row(base[i % 16], f"img{i}") for i in range(args.images)]
    df = DataFrame({"image": rows})
    out = {}
    for name, build in [
        ("resize256_centercrop224", lambda t: t.resize(height=256, width=256).centerCrop(224, 224)),
        ("resize256_centercrop224_blur5_flip", lambda t: t.resize(height=256, width=256).centerCrop(224, 224)
         .blur(5, 5).flip(1)),
        ("resize256_centercrop224_totensor", lambda t: t.resize(height=256, width=256).centerCrop(224, 224)
         .normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225], 1 / 255.0)),
    ]:
        for dev in ("gpu", "cpu"):
            t = build(ImageTransformer(inputCol="image", outputCol="o", deviceType=dev, batchSize=256))
            t.transform(df.slice(0, min(64, args.images)))  # warm-up (kernels, pinned pool)
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                t.transform(df)
                ts.append(time.perf_counter() - t0)
            out[f"{name}_{dev}_img_per_s"] = round(args.images / min(ts), 1)
            print(json.dumps({"stages": name, "device": dev, "img_per_s": out[f"{name}_{dev}_img_per_s"],
                              "best_s": round(min(ts), 4)}), flush=True)
    print(json.dumps({"metric": "ImageTransformer img/s (512x512 BGR rows)", **out}), flush=True)


if __name__ == "__main__":
    main()
