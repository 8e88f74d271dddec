"""Is the VW learn kernel bound by hot-slot contention? One resident pass of 2M examples x ~64 features at
2^30 through GpuSgd.learn, with the bench's Zipf-like ids and with uniformly random ids (same counts, values,
labels). One MI355X."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    from synapseml_amd.ops import native
    from tools.bench_vw import make_pass

    vw = native.load("_vw")
    ip, idx, val, y = make_pass(2_000_000, 64, seed=0)
    rng = np.random.default_rng(1)
    uni = rng.integers(0, 1 << 32, size=len(idx), dtype=np.uint64).astype(np.uint32)
    torch.cuda.init()
    for name, ids in (("zipf", idx), ("uniform", uni), ("zipf", idx), ("uniform", uni)):
        cfg = vw.GpuSgdConfig()
        cfg.bits = 30
        cfg.loss = 1
        sgd = vw.GpuSgd(cfg, 0)
        sgd.stage(ip, ids, val, y, None)  # resident pass: the timed part is the learning only
        sgd.learn_staged(0, 1000, 16384)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sgd.learn_staged(1000, len(y), 16384)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"ids": name, "learn_ms": round(dt * 1e3, 2), "ex_per_s": round(len(y) / dt)}), flush=True)
        del sgd


if __name__ == "__main__":
    main()
