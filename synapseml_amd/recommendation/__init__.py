"""Recommendation (reference: core/.../recommendation/{SAR, SARModel,
RankingAdapter, RankingEvaluator, RankingTrainValidationSplit,
RecommendationIndexer}.scala, Python RankingTrainValidationSplit.py).

SAR's item-item similarity is a co-occurrence GEMM (Bᵀ·B over the binary
user×item matrix) and scoring is affinity × similarity — both run as dense
device GEMMs through torch (hipBLASLt on the MI355X) when a GPU is visible.
An explicit/implicit ALS is included for the RankingAdapter workflows the
reference runs with SparkML's ALS."""
from __future__ import annotations

import datetime as _dt
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..core.contracts import HasLabelCol, HasPredictionCol, HasSeed
from ..core.dataframe import DataFrame
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Estimator, Evaluator, Model


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


def _torch_dev():
    import torch

    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class RecommendationParams(Params):
    userCol = Param("Column of users", "user", T.toString)
    itemCol = Param("Column of items", "item", T.toString)
    ratingCol = Param("Column of ratings", "rating", T.toString)


class HasK(Params):
    k = Param("number of items", 10, T.toInt)


# ---------------------------------------------------------------------- SAR
def _java_to_py(fmt: str) -> str:
    out = fmt
    for a, b in (("yyyy", "%Y"), ("EEE", "%a"), ("MMM", "%b"), ("MM", "%m"), ("dd", "%d"), ("HH", "%H"),
                 ("mm", "%M"), ("ss", "%S"), ("'T'", "T"), ("Z", "%z")):
        out = out.replace(a, b)
    out = out.replace("h:", "%H:")
    return out


class SARModel(Model, RecommendationParams):
    userDataFrame = Param("user affinity rows: user, flatList", None, complex=True)
    itemDataFrame = Param("item similarity rows: item, itemAffinities", None, complex=True)
    supportThreshold = Param("Minimum number of ratings per item", 4, T.toInt)
    rank = Param("rank (unused by SAR, kept for API parity)", 10, T.toInt)

    def _mats(self):
        u = self.getUserDataFrame()
        it = self.getItemDataFrame()
        A = np.stack([np.asarray(v, np.float32) for v in u["flatList"].tolist()])
        S = np.stack([np.asarray(v, np.float32) for v in it["itemAffinities"].tolist()])
        return np.asarray(u[self.getUserCol()]), A, np.asarray(it[self.getItemCol()]), S

    def _scores(self, A, S, item_ids):
        import torch

        dev = _torch_dev()
        # S rows are items ordered by item id; expand to a dense item x item matrix
        n = A.shape[1]
        Sd = np.zeros((n, n), np.float32)
        for row, iid in zip(S, item_ids.astype(int)):
            Sd[iid, : len(row)] = row[:n]
        At = torch.as_tensor(A, device=dev)
        St = torch.as_tensor(Sd, device=dev)
        return (At @ St).cpu().numpy()

    def _topk(self, users, scores, k):
        recs = []
        for r in range(scores.shape[0]):
            idx = np.argsort(-scores[r], kind="stable")[:k]
            recs.append([{self.getItemCol(): int(i), "rating": float(scores[r, i])} for i in idx])
        return DataFrame({self.getUserCol(): users, "recommendations": _obj(recs)})

    def recommendForAllUsers(self, numItems: int) -> DataFrame:  # noqa: N802
        users, A, items, S = self._mats()
        return self._topk(users, self._scores(A, S, items), numItems)

    def recommendForUserSubset(self, dataset: DataFrame, numItems: int) -> DataFrame:  # noqa: N802
        users, A, items, S = self._mats()
        want = set(dataset[self.getUserCol()].tolist())
        keep = np.asarray([u in want for u in users.tolist()])
        return self._topk(users[keep], self._scores(A[keep], S, items), numItems)

    def recommendForAllItems(self, numItems: int) -> DataFrame:  # noqa: N802
        users, A, items, S = self._mats()
        sc = self._scores(A, S, items).T
        recs = []
        for r in range(sc.shape[0]):
            idx = np.argsort(-sc[r], kind="stable")[:numItems]
            recs.append([{self.getUserCol(): users[i].item() if hasattr(users[i], "item") else users[i],
                          "rating": float(sc[r, i])} for i in idx])
        return DataFrame({self.getItemCol(): np.arange(sc.shape[0]), "recommendations": _obj(recs)})

    def _transform(self, df):
        users, A, items, S = self._mats()
        sc = self._scores(A, S, items)
        upos = {u: i for i, u in enumerate(users.tolist())}
        pred = []
        for u, it in zip(df[self.getUserCol()].tolist(), df[self.getItemCol()].tolist()):
            r = upos.get(u)
            pred.append(float(sc[r, int(it)]) if r is not None and 0 <= int(it) < sc.shape[1] else np.nan)
        return df.withColumn("prediction", np.asarray(pred))


class SAR(Estimator, RecommendationParams):
    similarityFunction = Param("Defines the similarity function to be used by the model: jaccard, lift, "
                               "cooccurrence", "jaccard", T.toString)
    timeCol = Param("Time of activity", "time", T.toString)
    supportThreshold = Param("Minimum number of ratings per item", 4, T.toInt)
    startTime = Param("Set time custom now time if using historical data", None, T.toString)
    activityTimeFormat = Param("Time format for events", "yyyy/MM/dd'T'h:mm:ss", T.toString)
    timeDecayCoeff = Param("Use to scale time decay coeff to different half life dur", 30, T.toInt)
    startTimeFormat = Param("Format for start time", "EEE MMM dd HH:mm:ss Z yyyy", T.toString)

    def _affinity(self, df) -> np.ndarray:
        n = df.count()
        has_t = self.getTimeCol() in df
        has_r = self.getRatingCol() in df
        r = np.asarray(df[self.getRatingCol()], np.float64) if has_r else np.ones(n)
        if not has_t:
            return r
        ref = _dt.datetime.strptime(self.getStartTime(), _java_to_py(self.getStartTimeFormat())) \
            if self.getStartTime() else _dt.datetime.now()
        fmt = _java_to_py(self.getActivityTimeFormat())
        decay = []
        for t in df[self.getTimeCol()].tolist():
            at = t if isinstance(t, _dt.datetime) else _dt.datetime.strptime(str(t), fmt)
            if ref.tzinfo is not None and at.tzinfo is None:
                at = at.replace(tzinfo=ref.tzinfo)
            minutes = (ref - at).total_seconds() // 60
            decay.append(2.0 ** (-minutes / (self.getTimeDecayCoeff() * 24 * 60)))
        return np.asarray(decay) * r

    def _fit(self, df):
        import torch

        u = np.asarray(df[self.getUserCol()], np.float64).astype(np.int64)
        it = np.asarray(df[self.getItemCol()], np.float64).astype(np.int64)
        aff = self._affinity(df)
        users = np.unique(u)
        nU, nI = int(u.max()) + 1, int(it.max()) + 1
        A = np.zeros((nU, nI + 1), np.float32)
        np.add.at(A, (u, it), aff)
        dev = _torch_dev()
        B = torch.zeros((nU, nI), device=dev)
        B[torch.as_tensor(u, device=dev), torch.as_tensor(it, device=dev)] = 1.0
        C = (B.T @ B).cpu().numpy().astype(np.float64)  # item co-occurrence (users in common)
        cnt = np.diag(C).copy()
        f = self.getSimilarityFunction()
        with np.errstate(divide="ignore", invalid="ignore"):
            if f == "jaccard":
                sim = C / (cnt[:, None] + cnt[None, :] - C)
            elif f == "lift":
                sim = C / (cnt[:, None] * cnt[None, :])
            else:
                sim = C
        sim = np.where(C < self.getSupportThreshold(), 0.0, np.nan_to_num(sim)).astype(np.float32)
        items = np.unique(it)
        user_df = DataFrame({self.getUserCol(): users.astype(np.float64),
                             "flatList": _obj([A[x].astype(np.float32) for x in users])})
        item_df = DataFrame({self.getItemCol(): items.astype(np.float64),
                             "itemAffinities": _obj([sim[i] for i in items])})
        m = SARModel(userCol=self.getUserCol(), itemCol=self.getItemCol(), ratingCol=self.getRatingCol(),
                     supportThreshold=self.getSupportThreshold())
        m.set("userDataFrame", user_df)
        m.set("itemDataFrame", item_df)
        return m


# ---------------------------------------------------------------------- ALS
class ALSModel(Model, RecommendationParams, HasPredictionCol):
    userFactors = Param("user factors", None, complex=True)
    itemFactors = Param("item factors", None, complex=True)
    coldStartStrategy = Param("nan | drop", "nan", T.toString)

    def _transform(self, df):
        U, V = np.asarray(self.getUserFactors()), np.asarray(self.getItemFactors())
        u = np.asarray(df[self.getUserCol()], np.float64).astype(np.int64)
        i = np.asarray(df[self.getItemCol()], np.float64).astype(np.int64)
        ok = (u >= 0) & (u < len(U)) & (i >= 0) & (i < len(V))
        pred = np.full(len(u), np.nan)
        pred[ok] = np.einsum("ij,ij->i", U[u[ok]], V[i[ok]])
        out = df.withColumn(self.getPredictionCol(), pred)
        return out.filter(~np.isnan(pred)) if self.getColdStartStrategy() == "drop" else out

    def _recommend(self, src, dst, src_name, dst_name, k, ids=None):
        sc = src @ dst.T
        recs = []
        rows = range(len(src)) if ids is None else ids
        for r in rows:
            idx = np.argsort(-sc[r], kind="stable")[:k]
            recs.append([{dst_name: int(j), "rating": float(sc[r, j])} for j in idx])
        return DataFrame({src_name: np.asarray(list(rows)), "recommendations": _obj(recs)})

    def recommendForAllUsers(self, numItems: int) -> DataFrame:  # noqa: N802
        return self._recommend(np.asarray(self.getUserFactors()), np.asarray(self.getItemFactors()),
                               self.getUserCol(), self.getItemCol(), numItems)

    def recommendForAllItems(self, numUsers: int) -> DataFrame:  # noqa: N802
        return self._recommend(np.asarray(self.getItemFactors()), np.asarray(self.getUserFactors()),
                               self.getItemCol(), self.getUserCol(), numUsers)

    def recommendForUserSubset(self, dataset: DataFrame, numItems: int) -> DataFrame:  # noqa: N802
        ids = sorted(set(int(x) for x in dataset[self.getUserCol()].tolist()))
        return self._recommend(np.asarray(self.getUserFactors()), np.asarray(self.getItemFactors()),
                               self.getUserCol(), self.getItemCol(), numItems, ids)


class ALS(Estimator, RecommendationParams, HasPredictionCol, HasSeed):
    rank = Param("rank of the factorization", 10, T.toInt)
    maxIter = Param("max number of iterations", 10, T.toInt)
    regParam = Param("regularization parameter", 0.1, T.toFloat)
    implicitPrefs = Param("whether to use implicit preference", False, T.toBoolean)
    alpha = Param("alpha for implicit preference", 1.0, T.toFloat)
    nonnegative = Param("whether to use nonnegative constraint for least squares", False, T.toBoolean)
    coldStartStrategy = Param("nan | drop", "nan", T.toString)

    def _fit(self, df):
        import torch

        dev = _torch_dev()
        u = np.asarray(df[self.getUserCol()], np.float64).astype(np.int64)
        i = np.asarray(df[self.getItemCol()], np.float64).astype(np.int64)
        r = np.asarray(df[self.getRatingCol()], np.float64) if self.getRatingCol() in df else np.ones(len(u))
        nU, nI, k = int(u.max()) + 1, int(i.max()) + 1, self.getRank()
        g = torch.Generator().manual_seed(self.getSeed())
        U = (torch.rand(nU, k, generator=g, dtype=torch.float64) * 0.1).to(dev)
        V = (torch.rand(nI, k, generator=g, dtype=torch.float64) * 0.1).to(dev)
        R = torch.zeros(nU, nI, dtype=torch.float64, device=dev)
        M = torch.zeros(nU, nI, dtype=torch.float64, device=dev)
        R[torch.as_tensor(u, device=dev), torch.as_tensor(i, device=dev)] = torch.as_tensor(r, device=dev)
        M[torch.as_tensor(u, device=dev), torch.as_tensor(i, device=dev)] = 1.0
        lam = self.getRegParam()
        eye = torch.eye(k, dtype=torch.float64, device=dev)
        implicit = self.getImplicitPrefs()
        if implicit:
            P = (R > 0).double()
            Cw = self.getAlpha() * R * M  # confidence - 1 on observed entries
        nonneg = self.getNonnegative()
        # Every half-sweep is batched: all normal-equation matrices come from one GEMM against the Y (x) Y
        # outer products ([n, k*k]) and all k x k systems are solved in one batched call.
        for _ in range(self.getMaxIter()):
            for side in (0, 1):
                X, Y = (U, V) if side == 0 else (V, U)
                Mm, Rm = (M, R) if side == 0 else (M.T, R.T)
                YY = (Y[:, :, None] * Y[:, None, :]).reshape(Y.shape[0], k * k)
                if implicit:
                    Cm, Pm = (Cw, P) if side == 0 else (Cw.T, P.T)
                    A = (Y.T @ Y)[None] + (Cm @ YY).reshape(-1, k, k) + lam * eye
                    bvec = ((1.0 + Cm) * Pm) @ Y
                else:
                    n_a = Mm.sum(1)
                    A = (Mm @ YY).reshape(-1, k, k) + (lam * n_a.clamp(min=1.0))[:, None, None] * eye
                    bvec = (Mm * Rm) @ Y
                sol = torch.linalg.solve(A, bvec.unsqueeze(-1)).squeeze(-1)
                if not implicit:
                    sol = torch.where((Mm.sum(1) > 0)[:, None], sol, X)
                X.copy_(sol.clamp(min=0) if nonneg else sol)
        model = ALSModel(userCol=self.getUserCol(), itemCol=self.getItemCol(), ratingCol=self.getRatingCol(),
                         predictionCol=self.getPredictionCol(), coldStartStrategy=self.getColdStartStrategy())
        model.set("userFactors", U.cpu().numpy())
        model.set("itemFactors", V.cpu().numpy())
        return model


# ---------------------------------------------------------------------- ranking metrics
class AdvancedRankingMetrics:
    """Spark RankingMetrics + the reference's extras (RankingEvaluator.scala:16-98)."""

    def __init__(self, pairs: Sequence, k: int, n_items: int):
        self.pairs = [(list(p), list(l)) for p, l in pairs]
        self.k = k
        self.n_items = n_items

    def ndcg(self) -> float:
        vals = []
        for pred, lab in self.pairs:
            ls = set(lab)
            if not ls:
                vals.append(0.0)
                continue
            n = min(max(len(pred), len(ls)), self.k)
            dcg = sum(1.0 / np.log2(i + 2) for i in range(min(n, len(pred))) if pred[i] in ls)
            idcg = sum(1.0 / np.log2(i + 2) for i in range(min(len(ls), self.k)))
            vals.append(dcg / idcg if idcg else 0.0)
        return float(np.mean(vals)) if vals else 0.0

    def map(self) -> float:
        vals = []
        for pred, lab in self.pairs:
            ls = set(lab)
            if not ls:
                vals.append(0.0)
                continue
            hits, s = 0, 0.0
            for i, p in enumerate(pred):
                if p in ls:
                    hits += 1
                    s += hits / (i + 1.0)
            vals.append(s / len(ls))
        return float(np.mean(vals)) if vals else 0.0

    def precision_at_k(self) -> float:
        vals = [sum(1 for p in pred[: self.k] if p in set(lab)) / self.k for pred, lab in self.pairs]
        return float(np.mean(vals)) if vals else 0.0

    def recall_at_k(self) -> float:
        vals = [len(set(pred) & set(lab)) / len(pred) if pred else 0.0 for pred, lab in self.pairs]
        return float(np.mean(vals)) if vals else 0.0

    def diversity_at_k(self) -> float:
        uniq = set()
        for pred, _ in self.pairs:
            uniq |= set(pred)
        return len(uniq) / self.n_items

    def max_diversity(self) -> float:
        uniq = set()
        for pred, lab in self.pairs:
            uniq |= set(pred) | set(lab)
        return len(uniq) / self.n_items

    def mrr(self) -> float:
        vals = []
        for pred, lab in self.pairs:
            ls = set(lab)
            rr = 0.0
            for i, p in enumerate(pred):
                if p in ls:
                    rr = 1.0 / (i + 1)
                    break
            vals.append(rr)
        return float(np.mean(vals)) if vals else 0.0

    def fcp(self) -> float:
        vals = []
        for pred, lab in self.pairs:
            nc = nd = 0.0
            for i, p in enumerate(pred):
                if len(lab) > i:
                    if p == lab[i]:
                        nc += 1
                    else:
                        nd += 1
            vals.append(nc / (nc + nd) if nc + nd else np.nan)
        return float(np.nanmean(vals)) if vals else 0.0

    def get(self, name: str) -> float:
        return {"map": self.map, "ndcgAt": self.ndcg, "precisionAtk": self.precision_at_k,
                "recallAtK": self.recall_at_k, "diversityAtK": self.diversity_at_k,
                "maxDiversity": self.max_diversity, "mrr": self.mrr, "fcp": self.fcp}[name]()

    def all(self) -> Dict[str, float]:
        return {n: self.get(n) for n in ("map", "ndcgAt", "precisionAtk", "recallAtK", "diversityAtK",
                                         "maxDiversity", "mrr", "fcp")}


class RankingEvaluator(Evaluator, HasK, HasLabelCol, HasPredictionCol):
    nItems = Param("number of items", -1, T.toInt)
    metricName = Param("ndcgAt | map | mapk | recallAtK | diversityAtK | maxDiversity | mrr | fcp", "ndcgAt",
                       T.toString)

    def getMetrics(self, df: DataFrame) -> AdvancedRankingMetrics:  # noqa: N802
        pairs = list(zip(df[self.getPredictionCol()].tolist(), df[self.getLabelCol()].tolist()))
        n = self.getNItems()
        if n <= 0:
            items = set()
            for p, l in pairs:
                items |= set(p) | set(l)
            n = max(1, len(items))
        return AdvancedRankingMetrics(pairs, self.getK(), n)

    def getMetricsMap(self, df: DataFrame) -> Dict[str, float]:  # noqa: N802
        return self.getMetrics(df).all()

    def _evaluate(self, df):
        name = "map" if self.getMetricName() == "mapk" else self.getMetricName()
        return self.getMetrics(df).get(name)

    def isLargerBetter(self):  # noqa: N802
        return True


# ---------------------------------------------------------------------- adapter & split
class RankingAdapterModel(Model, RecommendationParams, HasK, HasLabelCol):
    recommenderModel = Param("recommenderModel", None, complex=True)
    mode = Param("recommendation mode", "allUsers", T.toString)

    def _transform(self, df):
        m = self.getRecommenderModel()
        recs = m.recommendForAllUsers(self.getK()) if self.getMode() == "allUsers" else \
            m.recommendForUserSubset(df, self.getK())
        rec_map = {}
        for u, r in zip(recs[self.getUserCol()].tolist(), recs["recommendations"].tolist()):
            rec_map[float(u)] = [float(x[self.getItemCol()]) for x in r]
        truth: Dict[float, list] = {}
        rating = self.getRatingCol() if self.getRatingCol() in df else None
        rows = list(zip(df[self.getUserCol()].tolist(), df[self.getItemCol()].tolist(),
                        df[rating].tolist() if rating else [1.0] * df.count()))
        rows.sort(key=lambda t: -t[2])
        for u, it, _ in rows:
            truth.setdefault(float(u), []).append(float(it))
        users = sorted(truth)
        return DataFrame({self.getUserCol(): np.asarray(users),
                          "prediction": _obj([rec_map.get(u, []) for u in users]),
                          self.getLabelCol(): _obj([truth[u] for u in users])})


class RankingAdapter(Estimator, RecommendationParams, HasK, HasLabelCol):
    recommender = Param("estimator for selection", None, complex=True)
    mode = Param("recommendation mode", "allUsers", T.toString)
    minRatingsPerUser = Param("min ratings for users > 0", 1, T.toInt)
    minRatingsPerItem = Param("min ratings for items > 0", 1, T.toInt)

    def _fit(self, df):
        rec = self.getRecommender()
        for p in ("userCol", "itemCol", "ratingCol"):
            if rec.hasParam(p) and not rec.isSet(p):
                rec.set(p, self.getOrDefault(p))
        m = RankingAdapterModel(userCol=self.getUserCol(), itemCol=self.getItemCol(), ratingCol=self.getRatingCol(),
                                k=self.getK(), labelCol=self.getLabelCol(), mode=self.getMode())
        return m.set("recommenderModel", rec.fit(df))


def split_per_user(df: DataFrame, user_col: str, ratio: float, seed: int):
    """Stratified split: each user's ratings are split ratio : 1 - ratio."""
    rng = np.random.default_rng(seed)
    users = df[user_col].tolist()
    by: Dict = {}
    for i, u in enumerate(users):
        by.setdefault(u, []).append(i)
    train = np.zeros(len(users), bool)
    for u, idx in by.items():
        idx = np.asarray(idx)
        rng.shuffle(idx)
        ntr = max(1, int(round(len(idx) * ratio))) if len(idx) > 1 else 1
        train[idx[:ntr]] = True
    return df.filter(train), df.filter(~train)


class RankingTrainValidationSplitModel(Model, RecommendationParams):
    bestModel = Param("best model", None, complex=True)
    validationMetrics = Param("validation metrics", [], T.identity)

    def _transform(self, df):
        return self.getBestModel().transform(df)

    def recommendForAllUsers(self, numItems: int) -> DataFrame:  # noqa: N802
        return self.getBestModel().recommendForAllUsers(numItems)

    def recommendForAllItems(self, numItems: int) -> DataFrame:  # noqa: N802
        return self.getBestModel().recommendForAllItems(numItems)


class RankingTrainValidationSplit(Estimator, RecommendationParams, HasSeed):
    estimator = Param("estimator for selection", None, complex=True)
    estimatorParamMaps = Param("param maps for the estimator", [{}], T.identity)
    evaluator = Param("evaluator used to select hyper-parameters", None, complex=True)
    trainRatio = Param("ratio between training set and validation set (>= 0 && <= 1)", 0.75, T.toFloat)
    minRatingsU = Param("min ratings for users > 0", 1, T.toInt)
    minRatingsI = Param("min ratings for items > 0", 1, T.toInt)

    def _fit(self, df):
        ev = self.getEvaluator() or RankingEvaluator()
        tr, va = split_per_user(df, self.getUserCol(), self.getTrainRatio(), self.getSeed())
        metrics = []
        for pm in self.getEstimatorParamMaps() or [{}]:
            est = self.getEstimator().copy(pm)
            adapter = RankingAdapter(userCol=self.getUserCol(), itemCol=self.getItemCol(),
                                     ratingCol=self.getRatingCol(), k=ev.getK()).set("recommender", est)
            am = adapter.fit(tr)
            metrics.append(ev.evaluate(am.transform(va)))
        best = int(np.argmax(metrics) if ev.isLargerBetter() else np.argmin(metrics))
        bm = self.getEstimator().copy((self.getEstimatorParamMaps() or [{}])[best]).fit(df)
        out = RankingTrainValidationSplitModel(userCol=self.getUserCol(), itemCol=self.getItemCol(),
                                               ratingCol=self.getRatingCol(), validationMetrics=metrics)
        return out.set("bestModel", bm)


# ---------------------------------------------------------------------- indexer
class RecommendationIndexerModel(Model):
    userInputCol = Param("User Input Col", None, T.toString)
    userOutputCol = Param("User Output Col", None, T.toString)
    itemInputCol = Param("Item Input Col", None, T.toString)
    itemOutputCol = Param("Item Output Col", None, T.toString)
    ratingCol = Param("Rating Col", None, T.toString)
    userIndexModel = Param("userIndexModel", None, complex=True)
    itemIndexModel = Param("itemIndexModel", None, complex=True)

    def _transform(self, df):
        out = self.getUserIndexModel().transform(df)
        return self.getItemIndexModel().transform(out)

    def getUserIndex(self) -> Dict[int, str]:  # noqa: N802
        return {i: l for i, l in enumerate(self.getUserIndexModel().getLabels())}

    def getItemIndex(self) -> Dict[int, str]:  # noqa: N802
        return {i: l for i, l in enumerate(self.getItemIndexModel().getLabels())}

    def recoverUser(self, idx: int) -> str:  # noqa: N802
        return self.getUserIndex().get(int(idx), "-1")

    def recoverItem(self, idx: int) -> str:  # noqa: N802
        return self.getItemIndex().get(int(idx), "-1")


class RecommendationIndexer(Estimator):
    userInputCol = Param("User Input Col", None, T.toString)
    userOutputCol = Param("User Output Col", None, T.toString)
    itemInputCol = Param("Item Input Col", None, T.toString)
    itemOutputCol = Param("Item Output Col", None, T.toString)
    ratingCol = Param("Rating Col", None, T.toString)

    def _fit(self, df):
        from ..featurize.ml import StringIndexer

        um = StringIndexer(inputCol=self.getUserInputCol(), outputCol=self.getUserOutputCol(),
                           handleInvalid="skip").fit(df)
        im = StringIndexer(inputCol=self.getItemInputCol(), outputCol=self.getItemOutputCol(),
                           handleInvalid="skip").fit(df)
        m = RecommendationIndexerModel(userInputCol=self.getUserInputCol(), userOutputCol=self.getUserOutputCol(),
                                       itemInputCol=self.getItemInputCol(), itemOutputCol=self.getItemOutputCol(),
                                       ratingCol=self.getRatingCol())
        m.set("userIndexModel", um)
        m.set("itemIndexModel", im)
        return m


__all__ = ["SAR", "SARModel", "ALS", "ALSModel", "RankingEvaluator", "AdvancedRankingMetrics", "RankingAdapter",
           "RankingAdapterModel", "RankingTrainValidationSplit", "RankingTrainValidationSplitModel",
           "RecommendationIndexer", "RecommendationIndexerModel", "split_per_user"]
