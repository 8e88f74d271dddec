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
        # one round of the batched tree growth: 8 expansions x (histogram + count) = 8 x 114 KB
        out["us_per_allreduce_917KB"] = g.comm_device_allreduce_us(c, 8 * (28 * 256 + 1) * 2, 100)
        # the default batched round: 4 expansions x (E + 1) int64 (g, h) pairs, E = 28 x 256 -> 459 KB
        out["us_per_allreduce_459KB_round"] = g.comm_device_allreduce_us(c, 4 * (28 * 256 + 1) * 2, 100)
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
        # PV-Tree voting (topK=1: 2 of the 8 features reduced per leaf) on the device over P2P vs the host
        # backend's voting over the host comm: same split structure; and it differs from data-parallel
        # somewhere (the vote really restricted the search)
        vp = params + " tree_learner=voting top_k=1"
        vm = []
        for dev_type, comm in (("gpu", c), ("cpu", host)):
            ds = g.Dataset(ref, len(X))
            ds.push_dense(X, 0)
            ds.set_label(y)
            b = g.Booster(ds, vp.replace("device_type=gpu", "device_type=" + dev_type), comm)
            for _ in range(5):
                b.update()
            vm.append(b.save_model_string())
        keys = ("split_feature=", "threshold=", "leaf_count=")
        struct = lambda m: [l for l in m.splitlines() if l.startswith(keys)]
        # first tree (as test_gpu_trees_match_cpu: later trees inherit fp64-summation differences of the scores)
        tree0 = lambda m: [l for l in m.split("Tree=0")[1].split("Tree=1")[0].splitlines()
                           if l.startswith(("split_feature=", "threshold="))]
        out["voting_gpu_eq_cpu"] = tree0(vm[0]) == tree0(vm[1])
        out["voting_differs_from_data_parallel"] = struct(vm[0]) != struct(models[0])
        allv = D.all_gather_object(vm[0])
        out["voting_ranks_agree"] = all(m == allv[0] for m in allv)
    print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
