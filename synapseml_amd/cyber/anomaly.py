"""Access anomaly detection by collaborative filtering (reference:
core/src/main/python/synapse/ml/cyber/anomaly/{collaborative_filtering,
complement_access}.py).

Fit: index users/resources per tenant, scale the access likelihoods to
[lowValue, highValue] per tenant, optionally add sampled complement
(never-seen) accesses with ``negScore`` (explicit mode), factorise with ALS
(implicit by default; batched GEMM normal equations on the device), then
normalise so that the training accesses score mean 0 / std 1 per tenant:
anomaly_score(u, r) = -(u·r - mean_t) / std_t. Users and resources in
different access-graph connected components score +inf; pairs seen in
``historyAccessDf`` score 0."""
from __future__ import annotations

import random
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..core.dataframe import DataFrame
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model, Transformer
from ..recommendation import ALS
from .feature import IdIndexer, LinearScalarScaler, MultiIndexer


class AccessAnomalyConfig:
    default_tenant_col = "tenant"
    default_user_col = "user"
    default_res_col = "res"
    default_likelihood_col = "likelihood"
    default_output_col = "anomaly_score"
    default_rank = 10
    default_max_iter = 25
    default_reg_param = 1.0
    default_num_blocks = None
    default_separate_tenants = False
    default_low_value = 5.0
    default_high_value = 10.0
    default_apply_implicit_cf = True
    default_alpha = 1.0
    default_complementset_factor = 2
    default_neg_score = 1.0


class ComplementAccessTransformer(Transformer):
    """Sample ``complementsetFactor`` random index tuples per input row, within each partition's index ranges,
    keeping only tuples that never occur in the input (a sample of the complement set)."""

    partitionKey = Param("The name of the partition_key field name", None, T.toString)
    indexedColNamesArr = Param("The name of the fields to use to generate the complement set from", None,
                               T.toListString)
    complementsetFactor = Param("The estimated average size of the complement set to generate", 2, T.toInt)
    seed = Param("random seed", 42, T.toInt)

    def __init__(self, partition_key=None, indexed_col_names_arr=None, complementset_factor=2, **kw):
        super().__init__(**kw)
        self.setParams(partitionKey=partition_key, indexedColNamesArr=indexed_col_names_arr,
                       complementsetFactor=complementset_factor)

    def _transform(self, df):
        cols = self.getIndexedColNamesArr()
        pk = self.getPartitionKey()
        factor = self.getComplementsetFactor()
        if factor == 0 or df.count() == 0:
            return DataFrame({c: np.empty(0, dtype=np.int64) for c in ([pk] if pk else []) + cols})
        keys = df[pk].tolist() if pk else [0] * df.count()
        data = [np.asarray(df[c], dtype=np.int64) for c in cols]
        seen = set()
        lim: Dict = {}
        for i, k in enumerate(keys):
            t = tuple(int(d[i]) for d in data)
            seen.add((k, t))
            lo, hi = lim.get(k, ([None] * len(cols), [None] * len(cols)))
            lim[k] = ([t[j] if lo[j] is None else min(lo[j], t[j]) for j in range(len(cols))],
                      [t[j] if hi[j] is None else max(hi[j], t[j]) for j in range(len(cols))])
        rng = random.Random(self.getSeed())
        out = set()
        for k in keys:
            lo, hi = lim[k]
            for _ in range(factor):
                t = tuple(rng.randint(lo[j], hi[j]) for j in range(len(cols)))
                if (k, t) not in seen:
                    out.add((k, t))
        out = sorted(out, key=lambda kt: (str(kt[0]), kt[1]))
        res = {c: np.asarray([t[j] for _, t in out], dtype=np.int64) for j, c in enumerate(cols)}
        if pk:
            kc = np.empty(len(out), dtype=object)
            for i, (k, _) in enumerate(out):
                kc[i] = k
            res = {pk: kc, **res}
        return DataFrame(res)


class ConnectedComponents:
    """Per-tenant connected components of the bipartite user-resource access graph (union-find)."""

    def __init__(self, tenantCol: str, userCol: str, res_col: str, componentColName: str = "component"):  # noqa: N803
        self.tenant_col, self.user_col, self.res_col = tenantCol, userCol, res_col
        self.component_col_name = componentColName

    def components(self, df: DataFrame) -> Tuple[Dict, Dict]:
        parent: Dict = {}

        def find(x):
            while parent.setdefault(x, x) != x:
                parent[x] = parent[parent[x]]
                x = parent[x]
            return x

        for t, u, r in zip(df[self.tenant_col].tolist(), df[self.user_col].tolist(), df[self.res_col].tolist()):
            a, b = find(("u", t, u)), find(("r", t, r))
            if a != b:
                parent[max(a, b, key=str)] = min(a, b, key=str)
        users = {(k[1], k[2]): find(k) for k in list(parent) if k[0] == "u"}
        res = {(k[1], k[2]): find(k) for k in list(parent) if k[0] == "r"}
        return users, res

    def transform(self, df: DataFrame) -> Tuple[DataFrame, DataFrame]:
        users, res = self.components(df)
        ids: Dict = {}
        for c in sorted({str(c) for c in list(users.values()) + list(res.values())}):
            ids[c] = len(ids)

        def frame(m, col):
            items = sorted(m.items(), key=lambda kv: (str(kv[0][0]), str(kv[0][1])))
            t = np.empty(len(items), dtype=object)
            v = np.empty(len(items), dtype=object)
            for i, ((tt, vv), _) in enumerate(items):
                t[i], v[i] = tt, vv
            return DataFrame({self.tenant_col: t, col: v,
                              self.component_col_name: np.asarray([ids[str(c)] for _, c in items], dtype=np.int64)})

        return frame(users, self.user_col), frame(res, self.res_col)


class AccessAnomalyModel(Model):
    outputCol = Param("The name of the output column representing the calculated anomaly score", "anomaly_score",
                      T.toString)
    tenantCol = Param("tenant column", "tenant", T.toString)
    userCol = Param("user column", "user", T.toString)
    resCol = Param("resource column", "res", T.toString)
    preserveHistory = Param("score pairs seen in the history access frame as 0", True, T.toBoolean)
    userVectors = Param("(tenant, user) -> normalised vector", None, complex=True)
    resVectors = Param("(tenant, res) -> normalised vector", None, complex=True)
    userComponents = Param("(tenant, user) -> component", None, complex=True)
    resComponents = Param("(tenant, res) -> component", None, complex=True)
    history = Param("set of seen (tenant, user, res)", None, complex=True)

    # reference collaborative_filtering.py AccessAnomalyModel properties
    @property
    def tenant_col(self) -> str:
        return self.getTenantCol()

    @property
    def user_col(self) -> str:
        return self.getUserCol()

    @property
    def res_col(self) -> str:
        return self.getResCol()

    @property
    def user_vec_col(self) -> str:
        return self.getUserCol() + "_vector"

    @property
    def res_vec_col(self) -> str:
        return self.getResCol() + "_vector"

    def _mapping_df(self, vecs, col: str, vec_col: str) -> DataFrame:
        keys = sorted(vecs or {}, key=lambda k: (str(k[0]), str(k[1])))
        obj = lambda xs: np.array(xs + [None], dtype=object)[:-1]  # noqa: E731  (1-D object column)
        return DataFrame({self.getTenantCol(): obj([k[0] for k in keys]), col: obj([k[1] for k in keys]),
                          vec_col: obj([np.asarray(vecs[k], np.float64) for k in keys])})

    @property
    def user_mapping_df(self) -> DataFrame:
        """(tenant, user, user_vector) rows of the fitted model"""
        return self._mapping_df(self.getUserVectors(), self.getUserCol(), self.user_vec_col)

    @property
    def res_mapping_df(self) -> DataFrame:
        return self._mapping_df(self.getResVectors(), self.getResCol(), self.res_vec_col)

    def _transform(self, df):
        tc, uc, rc = self.getTenantCol(), self.getUserCol(), self.getResCol()
        T_ = df[tc].tolist() if tc in df else [0] * df.count()  # fit uses tenant 0 when the column is absent
        U, R = df[uc].tolist(), df[rc].tolist()
        uv, rv = self.getUserVectors(), self.getResVectors()
        ucmp, rcmp = self.getUserComponents() or {}, self.getResComponents() or {}
        hist = self.getHistory() if self.getPreserveHistory() else None
        out = np.empty(len(U), dtype=np.float64)
        for i, (t, u, r) in enumerate(zip(T_, U, R)):
            if hist is not None and (t, u, r) in hist:
                out[i] = 0.0
                continue
            a, b = uv.get((t, u)), rv.get((t, r))
            if a is None or b is None:
                out[i] = np.nan
            elif ucmp and ucmp.get((t, u)) != rcmp.get((t, r)):
                out[i] = np.inf
            else:
                out[i] = float(np.dot(a, b))
        return df.withColumn(self.getOutputCol(), out)


class AccessAnomaly(Estimator):
    tenantCol = Param("The name of the tenant column.", AccessAnomalyConfig.default_tenant_col, T.toString)
    userCol = Param("The name of the user column.", AccessAnomalyConfig.default_user_col, T.toString)
    resCol = Param("The name of the resource column.", AccessAnomalyConfig.default_res_col, T.toString)
    likelihoodCol = Param("The name of the column with the likelihood estimate for user, res access",
                          AccessAnomalyConfig.default_likelihood_col, T.toString)
    outputCol = Param("The name of the output column representing the calculated anomaly score",
                      AccessAnomalyConfig.default_output_col, T.toString)
    rankParam = Param("rankParam is the number of latent factors in the model", AccessAnomalyConfig.default_rank,
                      T.toInt)
    maxIter = Param("maxIter is the maximum number of iterations to run", AccessAnomalyConfig.default_max_iter,
                    T.toInt)
    regParam = Param("regParam specifies the regularization parameter in ALS",
                     AccessAnomalyConfig.default_reg_param, T.toFloat)
    numBlocks = Param("numBlocks (kept for API parity; factorisation is one batched device solve)", None,
                      T.identity)
    separateTenants = Param("separateTenants applies the algorithm per tenant in isolation",
                            AccessAnomalyConfig.default_separate_tenants, T.toBoolean)
    lowValue = Param("lowValue is used to scale the values of likelihood_col to be in the range "
                     "[lowValue, highValue]", AccessAnomalyConfig.default_low_value, T.identity)
    highValue = Param("highValue is used to scale the values of likelihood_col to be in the range "
                      "[lowValue, highValue]", AccessAnomalyConfig.default_high_value, T.identity)
    applyImplicitCf = Param("specifies whether to use the implicit/explicit feedback ALS for the data",
                            AccessAnomalyConfig.default_apply_implicit_cf, T.toBoolean)
    alphaParam = Param("alphaParam is a parameter applicable to the implicit feedback variant of ALS",
                       AccessAnomalyConfig.default_alpha, T.identity)
    complementsetFactor = Param("complementsetFactor (explicit mode): average number of complement accesses "
                                "sampled per access", AccessAnomalyConfig.default_complementset_factor, T.identity)
    negScore = Param("negScore is used to assign a value to the complement-set accesses",
                     AccessAnomalyConfig.default_neg_score, T.identity)
    historyAccessDf = Param("historyAccessDf: seen accesses (score 0) and the connected-component graph", None,
                            complex=True)
    seed = Param("random seed", 0, T.toInt)


    # reference collaborative_filtering.py AccessAnomaly column-name properties
    @property
    def indexed_user_col(self) -> str:
        return self.getUserCol() + "_index"

    @property
    def user_vec_col(self) -> str:
        return self.getUserCol() + "_vector"

    @property
    def indexed_res_col(self) -> str:
        return self.getResCol() + "_index"

    @property
    def res_vec_col(self) -> str:
        return self.getResCol() + "_vector"

    @property
    def scaled_likelihood_col(self) -> str:
        return self.getLikelihoodCol() + "_scaled"

    def create_spark_model_vectors_df(self, df: DataFrame):
        """fit and return the (tenant, user, vector) / (tenant, res, vector) mappings and the access history
        (reference _UserResourceFeatureVectorMapping fields)"""
        from types import SimpleNamespace

        m = self.fit(df)
        return SimpleNamespace(tenant_col=self.getTenantCol(), user_col=self.getUserCol(),
                               user_vec_col=self.user_vec_col, res_col=self.getResCol(), res_vec_col=self.res_vec_col,
                               history_access_df=df, user_feature_vector_mapping_df=m.user_mapping_df,
                               res_feature_vector_mapping_df=m.res_mapping_df)

    def _fit(self, df):
        tc, uc, rc, lc = self.getTenantCol(), self.getUserCol(), self.getResCol(), self.getLikelihoodCol()
        if tc not in df:
            df = df.withColumn(tc, np.zeros(df.count(), dtype=np.int64))
        iu, ir, sl = "__" + uc + "_index__", "__" + rc + "_index__", "__scaled_" + lc + "__"
        sep = self.getSeparateTenants()
        indexer = MultiIndexer([IdIndexer(uc, tc, iu, sep), IdIndexer(rc, tc, ir, sep)]).fit(df)
        idx = indexer.transform(df)
        lo, hi = self.getLowValue(), self.getHighValue()
        if lo is not None and hi is not None:
            idx = LinearScalarScaler(lc, tc, sl, lo, hi).fit(idx).transform(idx)
        else:
            idx = idx.withColumn(sl, np.asarray(idx[lc], dtype=np.float64))
        train = DataFrame({tc: idx[tc], iu: idx[iu], ir: idx[ir], sl: idx[sl]})
        if not self.getApplyImplicitCf():
            comp = ComplementAccessTransformer(tc, [iu, ir], self.getComplementsetFactor()).transform(train)
            if comp.count():
                comp = comp.withColumn(sl, np.full(comp.count(), float(self.getNegScore())))
                train = DataFrame.union_all([train, comp.select(tc, iu, ir, sl)])
        tenants = sorted(set(train[tc].tolist()), key=str)
        groups = [[t] for t in tenants] if sep else [tenants]
        uvec: Dict = {}
        rvec: Dict = {}
        k = self.getRankParam()
        for grp in groups:
            gset = set(grp)
            mask = np.asarray([t in gset for t in train[tc].tolist()])
            part = train.filter(mask)
            # global (tenant, index) -> dense ids for this factorisation
            upairs = sorted(set(zip(part[tc].tolist(), part[iu].tolist())), key=lambda p: (str(p[0]), p[1]))
            rpairs = sorted(set(zip(part[tc].tolist(), part[ir].tolist())), key=lambda p: (str(p[0]), p[1]))
            uid = {p: i for i, p in enumerate(upairs)}
            rid = {p: i for i, p in enumerate(rpairs)}
            als_df = DataFrame({"u": np.asarray([uid[p] for p in zip(part[tc].tolist(), part[iu].tolist())]),
                                "i": np.asarray([rid[p] for p in zip(part[tc].tolist(), part[ir].tolist())]),
                                "r": np.asarray(part[sl], dtype=np.float64)})
            als = ALS(userCol="u", itemCol="i", ratingCol="r", rank=k, maxIter=self.getMaxIter(),
                      regParam=self.getRegParam(), implicitPrefs=self.getApplyImplicitCf(),
                      alpha=float(self.getAlphaParam() or 1.0), nonnegative=True, seed=self.getSeed())
            m = als.fit(als_df)
            Uf, Vf = np.asarray(m.getUserFactors()), np.asarray(m.getItemFactors())
            for p, i in uid.items():
                uvec[p] = Uf[i]
            for p, i in rid.items():
                rvec[p] = Vf[i]
        # back to names
        um, rm = indexer.get_model_by_input_col(uc), indexer.get_model_by_input_col(rc)
        uinv = {(t, i): v for (t, v), i in um.getVocab().items()}
        rinv = {(t, i): v for (t, v), i in rm.getVocab().items()}
        uvec = {(t, uinv[(t, i)]): v for (t, i), v in uvec.items() if (t, i) in uinv}
        rvec = {(t, rinv[(t, i)]): v for (t, i), v in rvec.items() if (t, i) in rinv}
        # normalisation so that the training accesses score mean 0 / std 1 per tenant
        hist_df = self.getHistoryAccessDf()
        access = hist_df if hist_df is not None else df
        acc_t = access[tc].tolist() if tc in access else [0] * access.count()
        acc = list(zip(acc_t, access[uc].tolist(), access[rc].tolist()))
        dots: Dict = {}
        for t, u, r in acc:
            if (t, u) in uvec and (t, r) in rvec:
                dots.setdefault(t, []).append(float(np.dot(uvec[(t, u)], rvec[(t, r)])))
        stats = {t: (float(np.mean(v)), float(np.std(v))) for t, v in dots.items()}
        nu, nr = {}, {}
        for (t, u), v in uvec.items():
            mean, std = stats.get(t, (0.0, 1.0))
            coeff = -1.0 / (std if std != 0 else 1.0)
            nu[(t, u)] = coeff * np.concatenate([v, [-mean, 1.0]])
        for (t, r), v in rvec.items():
            nr[(t, r)] = np.concatenate([v, [1.0, 0.0]])
        cc = ConnectedComponents(tc, uc, rc)
        ucmp, rcmp = cc.components(DataFrame({tc: np.asarray(acc_t, dtype=object), uc: access[uc], rc: access[rc]}))
        model = AccessAnomalyModel(outputCol=self.getOutputCol(), tenantCol=tc, userCol=uc, resCol=rc)
        model.set("userVectors", nu).set("resVectors", nr).set("userComponents", ucmp).set("resComponents", rcmp)
        model.set("history", set(acc) if hist_df is not None else None)
        return model


__all__ = ["AccessAnomaly", "AccessAnomalyModel", "AccessAnomalyConfig", "ComplementAccessTransformer",
           "ConnectedComponents"]
