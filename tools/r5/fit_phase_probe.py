#!/usr/bin/env python3
"""Host-side phases of a LightGBMClassifier fit on the bench matrix (11M x 28 float32), each timed alone and
together: the pinned upload (DeviceRows), the row sample, the bin boundaries (DatasetReference.from_sample)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import higgs_like  # noqa: E402


def main():
    import torch

    from synapseml_amd.ops import native

    torch.cuda.init()
    g = native.gbdt()
    X, y = higgs_like(11_000_000, 28, seed=1234)
    names = [f"f{i}" for i in range(28)]
    params = "objective=binary num_leaves=31 max_bin=255 min_data_in_leaf=20 bin_construct_sample_cnt=200000"
    for mode, thr in (("0", "8"), ("1", "8"), ("1", "12"), ("1", "16"), ("0", "8"), ("1", "8")):
        os.environ["SML_UPLOAD_PIPE"], os.environ["SML_UPLOAD_THREADS"] = mode, thr
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            up = g.DeviceRows(X)
            up.wait()
            ts.append(time.perf_counter() - t0)
            del up
        print(f"upload pipe={mode} threads={thr}: " + " ".join(f"{t * 1e3:.1f}" for t in ts) + " ms", flush=True)
    os.environ["SML_UPLOAD_PIPE"], os.environ["SML_UPLOAD_THREADS"] = "1", "8"
    for rep in range(3):
        t0 = time.perf_counter()
        up = g.DeviceRows(X)
        up.wait()
        t_up = time.perf_counter() - t0
        del up
        t0 = time.perf_counter()
        s = g.sample_dense_rows(X, 200000, 0)
        t_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        ref = g.DatasetReference.from_sample(s, len(X), params, names)
        t_b = time.perf_counter() - t0
        t0 = time.perf_counter()
        up = g.DeviceRows(X)
        s = g.sample_dense_rows(X, 200000, 0)
        ref = g.DatasetReference.from_sample(s, len(X), params, names)
        t_sb = time.perf_counter() - t0
        up.wait()
        t_all = time.perf_counter() - t0
        del up, ref
        print(f"rep {rep}: upload alone {t_up * 1e3:.1f} ms ({X.nbytes / t_up / 1e9:.1f} GB/s), sample {t_s * 1e3:.1f} ms, "
              f"bins {t_b * 1e3:.1f} ms; together: sample+bins {t_sb * 1e3:.1f} ms, upload done at {t_all * 1e3:.1f} ms",
              flush=True)


if __name__ == "__main__":
    main()
