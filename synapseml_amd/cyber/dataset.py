"""Synthetic access datasets for the access-anomaly model (reference:
core/src/main/python/synapse/ml/cyber/dataset.py DataFactory): three
departments (HR, finance, engineering) whose users mostly access their own
department's resources; optional shared resource joining the components;
intra-department (normal) and cross-department (anomalous) test sets."""
from __future__ import annotations

import random
from typing import List, Optional, Set, Tuple

import numpy as np

from ..core.dataframe import DataFrame
from .anomaly import AccessAnomalyConfig


class DataFactory:
    def __init__(self, num_hr_users: int = 7, num_hr_resources: int = 30, num_fin_users: int = 5,
                 num_fin_resources: int = 25, num_eng_users: int = 10, num_eng_resources: int = 50,
                 single_component: bool = True):
        self.hr_users = ["hr_user_" + str(i) for i in range(num_hr_users)]
        self.hr_resources = ["hr_res_" + str(i) for i in range(num_hr_resources)]
        self.fin_users = ["fin_user_" + str(i) for i in range(num_fin_users)]
        self.fin_resources = ["fin_res_" + str(i) for i in range(num_fin_resources)]
        self.eng_users = ["eng_user_" + str(i) for i in range(num_eng_users)]
        self.eng_resources = ["eng_res_" + str(i) for i in range(num_eng_resources)]
        self.join_resources = ["ffa"] if single_component else []
        self.rand = random.Random(42)

    @staticmethod
    def to_df(tups: List[Tuple[str, str, float]]) -> DataFrame:
        u = np.empty(len(tups), dtype=object)
        r = np.empty(len(tups), dtype=object)
        for i, t in enumerate(tups):
            u[i], r[i] = t[0], t[1]
        return DataFrame({AccessAnomalyConfig.default_user_col: u, AccessAnomalyConfig.default_res_col: r,
                          AccessAnomalyConfig.default_likelihood_col: np.asarray([t[2] for t in tups], float)})

    def to_pdf(self, users: List, resources: List, likelihoods: List[float]) -> DataFrame:
        """(user, res, likelihood) columns as strings / floats (reference dataset.py DataFactory.to_pdf; a
        pandas frame there, this framework's DataFrame here)"""
        return self.to_df([(str(u), str(r), float(s)) for u, r, s in zip(users, resources, likelihoods)])

    def tups2pdf(self, tup_arr: List[Tuple[str, str, float]]) -> DataFrame:
        return self.to_pdf([t[0] for t in tup_arr], [t[1] for t in tup_arr], [t[2] for t in tup_arr])

    def create_fixed_training_data(self) -> DataFrame:
        """a small fixed access log: 25 (user, res, likelihood) rows over users 1..11 and resources 1..8, 14 of
        them at likelihood 1 and the rest heavier (same shape as the reference fixture; generated from a fixed
        seed rather than listed)"""
        rng = random.Random(7)
        users = [rng.randint(1, 11) for _ in range(25)]
        resources = [rng.randint(1, 8) for _ in range(25)]
        likelihoods = [1.0] * 14 + [round(rng.uniform(10.0, 47.0), 6) for _ in range(11)]
        return self.to_pdf(users, resources, likelihoods)

    def edges_between(self, users: List[str], resources: List[str], ratio: float, full_node_coverage: bool,
                      not_set: Optional[Set[Tuple[str, str]]] = None) -> List[Tuple[str, str, float]]:
        if not users or not resources:
            return []
        need = int(len(users) * len(resources) * ratio)
        seen: Set[Tuple[str, str]] = set()
        out = []
        if full_node_coverage:
            for i in range(max(len(users), len(resources))):
                u, r = users[i % len(users)], resources[i % len(resources)]
                if (u, r) not in seen and (not_set is None or (u, r) not in not_set):
                    seen.add((u, r))
                    out.append((u, r, float(self.rand.randint(500, 1000))))
        tries = 0
        while len(out) < need and tries < 50 * need + 100:
            tries += 1
            u, r = self.rand.choice(users), self.rand.choice(resources)
            if (u, r) in seen or (not_set is not None and (u, r) in not_set):
                continue
            seen.add((u, r))
            out.append((u, r, float(self.rand.randint(500, 1000))))
        return out

    def create_clustered_training_data(self, ratio: float = 0.25) -> DataFrame:
        tups = (self.edges_between(self.hr_users, self.hr_resources, ratio, True)
                + self.edges_between(self.fin_users, self.fin_resources, ratio, True)
                + self.edges_between(self.eng_users, self.eng_resources, ratio, True)
                + self.edges_between(self.hr_users + self.fin_users + self.eng_users, self.join_resources, 1.0,
                                     True))
        return self.to_df(tups)

    def create_clustered_intra_test_data(self, train: Optional[DataFrame] = None) -> DataFrame:
        seen = set(zip(train["user"].tolist(), train["res"].tolist())) if train is not None else None
        tups = (self.edges_between(self.hr_users, self.hr_resources, 0.025, False, seen)
                + self.edges_between(self.fin_users, self.fin_resources, 0.025, False, seen)
                + self.edges_between(self.eng_users, self.eng_resources, 0.025, False, seen))
        return self.to_df(tups)

    def create_clustered_inter_test_data(self) -> DataFrame:
        tups = (self.edges_between(self.hr_users, self.fin_resources, 0.025, False)
                + self.edges_between(self.hr_users, self.eng_resources, 0.025, False)
                + self.edges_between(self.fin_users, self.hr_resources, 0.025, False)
                + self.edges_between(self.fin_users, self.eng_resources, 0.025, False)
                + self.edges_between(self.eng_users, self.fin_resources, 0.025, False)
                + self.edges_between(self.eng_users, self.hr_resources, 0.025, False))
        return self.to_df(tups)


__all__ = ["DataFactory"]
