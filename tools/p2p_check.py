"""Two+ ranks (torchrun, gloo control plane) exercise the one-shot P2P
allreduce (csrc/gbdt/comm_p2p.hip) on the device(s) they see, and data-parallel
GBDT training over it vs the plain host communicator.

On a one-GPU box every rank shares cuda:0 (IPC between processes on the same
device); on a node each rank takes LOCAL_RANK. Prints one JSON line per rank.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    from synapseml_amd.ops import native
    from synapseml_amd.parallel import distributed as D

    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    ndev = torch.cuda.device_count()
    dev = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev)
    torch.cuda.set_device(dev)
    g = native.gbdt()
    host = g.host_comm(r, w, lambda a: D.allreduce_numpy(a))
    c, ok, why = g.p2p_comm(host, dev, 1 << 20, 20000.0)
    out = {"rank": r, "world": w, "device": dev, "p2p_active": bool(ok), "reason": why}
    if ok:
        n = 14282  # 2E+2 doubles for 28 features x 255 bins
        x = [float((r + 1) * 10 + (i % 101)) for i in range(n)]
        got = np.asarray(g.comm_device_allreduce(c, x, 4))
        exp = np.asarray([w * (w + 1) / 2 * 10 + w * (i % 101) for i in range(n)], dtype=np.float64)
        out["allreduce_exact"] = bool(np.array_equal(got, exp))
        out["us_per_allreduce_114KB"] = g.comm_device_allreduce_us(c, n, 200)
        out["us_per_allreduce_8KB"] = g.comm_device_allreduce_us(c, 1024, 200)
        # data-parallel training over P2P vs host comm: identical models
        rng = np.random.default_rng(7 + r)
        X = rng.standard_normal((40000, 8))
        y = (X[:, 0] + X[:, 1] * X[:, 2] + 0.3 * rng.standard_normal(40000) > 0).astype(np.float32)
        params = "objective=binary num_leaves=15 learning_rate=0.1 device_type=gpu"
        S = np.random.default_rng(99).standard_normal((5000, 8))  # same bin mappers on every rank
        ref = g.DatasetReference.from_sample(S, 40000 * w, params, [f"f{i}" for i in range(8)])
        models = []
        for comm in (c, host):
            ds = g.Dataset(ref, len(X))
            ds.push_dense(X, 0)
            ds.set_label(y)
            b = g.Booster(ds, params, comm)
            for _ in range(5):
                b.update()
            models.append(b.save_model_string())
        out["train_models_equal"] = models[0] == models[1]
        allm = D.all_gather_object(models[0])
        out["ranks_agree"] = all(m == allm[0] for m in allm)
    print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
