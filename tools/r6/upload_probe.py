"""Host -> HBM upload of the bench matrix (11M x 28 float32, 1.23 GB, pageable numpy) through DeviceRows, alone
and with the fit's sampling running beside it; SML_UPLOAD_THREADS sweeps the copy threads. One MI355X."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    from bench import higgs_like
    from synapseml_amd.ops import native

    g = native.gbdt()
    X, _ = higgs_like(11_000_000, 28, seed=1234)
    torch.cuda.init()
    for rep in range(3):
        t0 = time.perf_counter()
        up = g.DeviceRows(X)
        up.wait()
        t1 = time.perf_counter()
        up2 = g.DeviceRows(X)
        s = g.sample_dense_rows(X, 200000, 7)
        t2 = time.perf_counter()
        up2.wait()
        t3 = time.perf_counter()
        del up, up2, s
        print(json.dumps({"rep": rep, "threads": os.environ.get("SML_UPLOAD_THREADS", "8"),
                          "upload_ms": round((t1 - t0) * 1e3, 2), "GBps": round(X.nbytes / (t1 - t0) / 1e9, 1),
                          "with_sampling_ms": round((t3 - t1) * 1e3, 2), "sample_ms": round((t2 - t1) * 1e3, 2)}),
              flush=True)
    # the device's own copy rate from pinned memory (the floor for any staging scheme)
    h = torch.empty(X.nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(X.nbytes, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    print(json.dumps({"pinned_h2d_GBps": round(X.nbytes / (t1 - t0) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
