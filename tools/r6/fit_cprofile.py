"""Python-level profile of the bench step (LightGBMClassifier.fit + model text, 11M x 28, 100 iterations) on one
MI355X: which host calls outside the fit's own phases (total_ms) take the step's remaining milliseconds."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from bench import higgs_like
    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.lightgbm import LightGBMClassifier

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
    pr = cProfile.Profile()
    steps = 4
    t0 = time.perf_counter()
    pr.enable()
    tot = 0.0
    for _ in range(steps):
        model = est.fit(df)
        model.getNativeModel()
        tot += est.getPerformanceMeasures()[0]["total_ms"]
    pr.disable()
    torch.cuda.synchronize()
    print(f"step_ms {(time.perf_counter() - t0) * 1e3 / steps:.2f} total_ms {tot / steps:.2f}", flush=True)
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
