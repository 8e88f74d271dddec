"""TreeSHAP throughput: HIP kernel (K10) vs the host recursion (OpenMP).
Higgs-shape 28 features, binary, 100 trees x 31 leaves."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from synapseml_amd.ops import native

    g = native.gbdt()
    rng = np.random.default_rng(0)
    n, f = 200_000, 28
    X = rng.standard_normal((n, f))
    y = ((X[:, 0] + X[:, 1] * X[:, 2] + np.sin(X[:, 3]) + 0.5 * rng.standard_normal(n)) > 0).astype(np.float32)
    params = "objective=binary num_leaves=31 learning_rate=0.1 device_type=gpu"
    ref = g.DatasetReference.from_sample(X[:50000], n, params, [f"f{i}" for i in range(f)])
    ds = g.Dataset(ref, n)
    ds.push_dense(X, 0)
    ds.set_label(y)
    b = g.Booster(ds, params, None)
    for _ in range(100):
        b.update()
    gp = g.GpuPredictor(b, 0, -1, -1)
    Xt = np.ascontiguousarray(X[:100_000])
    gp.predict_contrib(b, Xt[:1000])
    t = time.perf_counter()
    out = gp.predict_contrib(b, Xt)
    gpu_s = time.perf_counter() - t
    m = 10_000
    t = time.perf_counter()
    cpu = b.predict(Xt[:m], 3, 0, -1)
    cpu_s = (time.perf_counter() - t) * len(Xt) / m
    err = float(np.abs(out[:m] - cpu).max())
    print(json.dumps({"rows": len(Xt), "trees": 100, "gpu_rows_per_s": len(Xt) / gpu_s,
                      "cpu_rows_per_s": len(Xt) / cpu_s, "speedup": cpu_s / gpu_s, "max_abs_err": err,
                      "cpu_threads": os.environ.get("OMP_NUM_THREADS")}))


if __name__ == "__main__":
    main()
