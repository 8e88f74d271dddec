"""ai.onnx.ml TreeEnsembleRegressor / TreeEnsembleClassifier (the form in
which LightGBM/sklearn tree models are exported to ONNX). Every (row, tree)
pair walks its tree in lock-step — one gather per level over flattened node
arrays — so a whole batch is a handful of device-wide tensor ops."""
from __future__ import annotations

import numpy as np
import torch

_MODES = {"BRANCH_LEQ": 0, "BRANCH_LT": 1, "BRANCH_GTE": 2, "BRANCH_GT": 3, "BRANCH_EQ": 4, "BRANCH_NEQ": 5,
          "LEAF": 6}


def _compile(at, classifier: bool):
    tids = np.asarray(at["nodes_treeids"], np.int64)
    nids = np.asarray(at["nodes_nodeids"], np.int64)
    key = {(int(t), int(n)): i for i, (t, n) in enumerate(zip(tids, nids))}
    m = len(tids)
    feat = np.asarray(at.get("nodes_featureids", [0] * m), np.int64)
    vals = np.asarray(at.get("nodes_values", [0.0] * m), np.float32)
    modes = np.asarray([_MODES[s] for s in at.get("nodes_modes", ["LEAF"] * m)], np.int64)
    tn = np.asarray(at.get("nodes_truenodeids", [0] * m), np.int64)
    fn = np.asarray(at.get("nodes_falsenodeids", [0] * m), np.int64)
    miss = np.asarray(at.get("nodes_missing_value_tracks_true", [0] * m), np.int64)
    true_idx = np.array([key.get((int(t), int(x)), i) for i, (t, x) in enumerate(zip(tids, tn))], np.int64)
    false_idx = np.array([key.get((int(t), int(x)), i) for i, (t, x) in enumerate(zip(tids, fn))], np.int64)
    true_idx[modes == 6] = np.nonzero(modes == 6)[0]
    false_idx[modes == 6] = np.nonzero(modes == 6)[0]
    trees = sorted(set(tids.tolist()))
    roots = np.array([key[(t, 0)] if (t, 0) in key else int(np.nonzero(tids == t)[0][0]) for t in trees], np.int64)
    pfx = "class_" if classifier else "target_"
    ct = np.asarray(at.get(pfx + "treeids", []), np.int64)
    cn = np.asarray(at.get(pfx + "nodeids", []), np.int64)
    cid = np.asarray(at.get(pfx + "ids", []), np.int64)
    cw = np.asarray(at.get(pfx + "weights", []), np.float32)
    if classifier:
        labels = at.get("classlabels_int64s") or at.get("classlabels_strings")
        nk = max(int(cid.max()) + 1 if len(cid) else 1, 1)
    else:
        labels = None
        nk = int(at.get("n_targets", 1))
    leafw = np.zeros((m, nk), np.float32)
    for t, n, k, w in zip(ct, cn, cid, cw):
        leafw[key[(int(t), int(n))], int(k)] += w
    return dict(feat=feat, vals=vals, modes=modes, tidx=true_idx, fidx=false_idx, miss=miss, roots=roots,
                leafw=leafw, nk=nk, labels=labels, max_depth=_max_depth(true_idx, false_idx, modes, roots))


def _max_depth(ti, fi, modes, roots):
    best = 0
    stack = [(int(r), 0) for r in roots]
    while stack:
        n, d = stack.pop()
        best = max(best, d)
        if modes[n] != 6 and d < len(modes):
            stack.append((int(ti[n]), d + 1))
            stack.append((int(fi[n]), d + 1))
    return best


def run_tree_ensemble(rt, at, x):
    classifier = rt.op_type == "TreeEnsembleClassifier"
    cache = at.setdefault("__compiled__", {})
    X = x[0]
    dev = X.device if isinstance(X, torch.Tensor) else torch.device("cpu")
    if dev not in cache:
        c = _compile(at, classifier)
        cache[dev] = {k: (torch.as_tensor(v, device=dev) if isinstance(v, np.ndarray) else v) for k, v in c.items()}
    c = cache[dev]
    X = torch.as_tensor(X, device=dev).to(torch.float32)
    if X.dim() == 1:
        X = X.unsqueeze(0)
    n = X.shape[0]
    T = c["roots"].shape[0]
    cur = c["roots"].unsqueeze(0).expand(n, T).clone()
    rows = torch.arange(n, device=dev).unsqueeze(1).expand(n, T)
    for _ in range(c["max_depth"]):
        f = c["feat"][cur]
        v = X[rows, f]
        thr = c["vals"][cur]
        md = c["modes"][cur]
        go = torch.where(md == 0, v <= thr, torch.where(md == 1, v < thr, torch.where(
            md == 2, v >= thr, torch.where(md == 3, v > thr, torch.where(md == 4, v == thr, v != thr)))))
        go = torch.where(torch.isnan(v), c["miss"][cur].bool(), go)
        nxt = torch.where(go, c["tidx"][cur], c["fidx"][cur])
        cur = torch.where(md == 6, cur, nxt)
    scores = c["leafw"][cur].sum(dim=1)  # [n, K]
    agg = at.get("aggregate_function", "SUM")
    if agg == "AVERAGE":
        scores = scores / T
    base = at.get("base_values")
    if base:
        if "base" not in c:
            c["base"] = torch.tensor(base, dtype=torch.float32, device=dev)
        scores = scores + c["base"]
    post = at.get("post_transform", "NONE")
    if not classifier:
        if post == "LOGISTIC":
            scores = torch.sigmoid(scores)
        return [scores]
    labels = c["labels"]
    if len(labels) == 2 and scores.shape[1] == 1:
        s1 = scores[:, 0:1]
        if post == "LOGISTIC":
            p = torch.sigmoid(s1)
            probs = torch.cat([1 - p, p], 1)
        else:
            probs = torch.cat([-s1, s1], 1)
        idx = (s1[:, 0] > 0.0).long()
    else:
        if post == "SOFTMAX":
            probs = torch.softmax(scores, dim=1)
        elif post == "LOGISTIC":
            probs = torch.sigmoid(scores)
        else:
            probs = scores
        idx = torch.argmax(scores, dim=1)
    if isinstance(labels[0], str):
        return [np.asarray(labels)[idx.cpu().numpy()].astype(object), probs]
    if "labels_t" not in c:
        c["labels_t"] = torch.tensor([int(v) for v in labels], dtype=torch.int64, device=dev)
    return [c["labels_t"][idx], probs]
