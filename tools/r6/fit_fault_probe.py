"""Minor page faults (first touches of fresh host memory) per fit phase of the bench step, and the time between
the fit's total_ms mark and the end of the step. 11M x 28, 100 iterations, one MI355X."""
import json
import os
import resource
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from bench import higgs_like
    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.lightgbm import LightGBMClassifier
    from synapseml_amd.lightgbm import base as B

    marks = []
    orig = B.InstrumentationMeasures.mark

    def mark(self, name, value_ms):
        marks.append((name, time.perf_counter(), resource.getrusage(resource.RUSAGE_SELF).ru_minflt))
        orig(self, name, value_ms)

    B.InstrumentationMeasures.mark = mark
    orig_tb = B.LightGBMBase._train_batch if hasattr(B, "LightGBMBase") else None
    if orig_tb is not None:
        def train_batch(self, *a, **k):
            r = orig_tb(self, *a, **k)
            marks.append(("train_batch_return", time.perf_counter(), resource.getrusage(resource.RUSAGE_SELF).ru_minflt))
            return r

        B.LightGBMBase._train_batch = train_batch
    if "--ranker" in sys.argv:  # tools/bench_ranker.py's data and estimator
        import numpy as np

        from synapseml_amd.lightgbm import LightGBMRanker
        from tools.bench_ranker import ranking_data

        X, y, sizes = ranking_data(12_500_000, 28, seed=77)
        qid = np.repeat(np.arange(len(sizes), dtype=np.int64), sizes)
        df = DataFrame({"features": X, "label": y, "query": qid})
        est = LightGBMRanker(numIterations=100, learningRate=0.1, numLeaves=31, maxBin=255, minDataInLeaf=20,
                             groupCol="query", evalAt=[10], deviceType="gpu")
    else:
        X, y = higgs_like(11_000_000, 28, seed=1234)
        df = DataFrame({"features": X, "label": y})
        est = LightGBMClassifier(numIterations=100, learningRate=0.1, numLeaves=31, maxBin=255,
                                 binSampleCount=200000, minDataInLeaf=20, objective="binary", deviceType="gpu",
                                 metric="auc")
    model = est.fit(df)
    model.getNativeModel()
    torch.cuda.synchronize()
    for step in range(5):
        marks.clear()
        f0 = resource.getrusage(resource.RUSAGE_SELF).ru_minflt
        t0 = time.perf_counter()
        model = est.fit(df)
        tf = time.perf_counter()
        model.getNativeModel()
        t1 = time.perf_counter()
        f1 = resource.getrusage(resource.RUSAGE_SELF).ru_minflt
        out = {"step": step, "step_ms": round((t1 - t0) * 1e3, 2), "faults": f1 - f0}
        prev_t, prev_f = t0, f0
        for name, t, f in marks:
            if name in ("prepare_ms", "sampling_ms", "dataset_creation_ms", "booster_init_ms", "training_iterations_ms",
                        "total_ms", "train_batch_return"):
                out[name] = [round((t - prev_t) * 1e3, 2), f - prev_f]
                prev_t, prev_f = t, f
        out["after_total"] = [round((t1 - prev_t) * 1e3, 2), f1 - prev_f]
        out["text_ms"] = round((t1 - tf) * 1e3, 2)
        pm = est.getPerformanceMeasures()[0]
        out["finalize_ms"] = {k: round(pm[k], 2) for k in ("stats_sync_ms", "release_ms", "dataset_free_ms")}
        print(json.dumps(out), flush=True)
    # page size / THP, for reading the counts
    try:
        with open("/sys/kernel/mm/transparent_hugepage/enabled") as fh:
            print("thp:", fh.read().strip())
    except OSError:
        pass


if __name__ == "__main__":
    main()
