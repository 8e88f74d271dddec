"""Python-level profile of ImageTransformer.transform on the device path (tools/bench_image.py's data: 2048 x
512x512 BGR rows, resize(256) + centerCrop(224), and the same + normalize/toTensor), one MI355X."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np

    from synapseml_amd.core import DataFrame
    from synapseml_amd.image import ImageTransformer
    from synapseml_amd.image.schema import make_image_row

    rng = np.random.default_rng(0)
    base = rng.integers(0, 256, (16, 512, 512, 3), dtype=np.uint8)
    rows = [make_image_row(base[i % 16], f"img{i}") for i in range(2048)]
    df = DataFrame({"image": rows})
    for name, tensor in (("rows", False), ("totensor", True)):
        t = ImageTransformer(inputCol="image", outputCol="o", deviceType="gpu", batchSize=256).resize(
            height=256, width=256).centerCrop(224, 224)
        if tensor:
            t = t.normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225], 1 / 255.0)
        t.transform(df.slice(0, 64))
        t.transform(df)
        t0 = time.perf_counter()
        t.transform(df)
        dt = time.perf_counter() - t0
        pr = cProfile.Profile()
        pr.enable()
        t.transform(df)
        pr.disable()
        print(f"== {name}: {2048 / dt:.0f} img/s ({dt * 1e3:.1f} ms)", flush=True)
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
