"""Where the bench step's time goes outside the fit's own phases: per step, the fit call's wall time, the
estimator's total_ms (inside _train_batch), the model text, and the destruction of the previous model
(its native booster, dataset and device buffers). 11M x 28, 100 iterations, one MI355X."""
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    from bench import higgs_like
    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.lightgbm import LightGBMClassifier

    X, y = higgs_like(11_000_000, 28, seed=1234)
    df = DataFrame({"features": X, "label": y})
    est = LightGBMClassifier(numIterations=100, learningRate=0.1, numLeaves=31, maxBin=255, binSampleCount=200000,
                             minDataInLeaf=20, objective="binary", deviceType="gpu", metric="auc")
    model = est.fit(df)
    model.getNativeModel()
    torch.cuda.synchronize()
    for step in range(4):
        t0 = time.perf_counter()
        new = est.fit(df)
        t1 = time.perf_counter()
        new.getNativeModel()
        t2 = time.perf_counter()
        old, model = model, new
        del old  # refcount drop: the previous model, its native booster and datasets go here
        t3a = time.perf_counter()
        gc.collect()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        m = est.getPerformanceMeasures()[0]
        print(json.dumps({"step": step, "fit_ms": round((t1 - t0) * 1e3, 2), "total_ms": m.get("total_ms"),
                          "text_ms": round((t2 - t1) * 1e3, 2), "del_prev_ms": round((t3a - t2) * 1e3, 2),
                          "gc_ms": round((t3 - t3a) * 1e3, 2),
                          "sync_ms": round((t4 - t3) * 1e3, 2)}), flush=True)
    # the bench's loop (no explicit collection): time the interpreter's own cyclic collections inside each fit
    gcs = []
    t_start = [0.0]

    def cb(phase, info):
        if phase == "start":
            t_start[0] = time.perf_counter()
        else:
            gcs.append((info["generation"], (time.perf_counter() - t_start[0]) * 1e3))

    gc.callbacks.append(cb)
    for step in range(5):
        gcs.clear()
        t0 = time.perf_counter()
        model = est.fit(df)
        model.getNativeModel()
        t1 = time.perf_counter()
        m = est.getPerformanceMeasures()[0]
        print(json.dumps({"autogc_step": step, "step_ms": round((t1 - t0) * 1e3, 2), "total_ms": m.get("total_ms"),
                          "gc_gen2_ms": round(sum(t for g, t in gcs if g == 2), 2),
                          "gc_other_ms": round(sum(t for g, t in gcs if g < 2), 2), "n_gc": len(gcs)}), flush=True)
    gc.callbacks.remove(cb)


if __name__ == "__main__":
    main()
