"""Estimator / Transformer / Model / Pipeline (SparkML pipeline semantics)."""
from __future__ import annotations

from typing import List, Optional

from .dataframe import DataFrame
from .logging import log_verb
from .params import Param, Params
from . import serialize


class _Writer:
    def __init__(self, stage):
        self.stage = stage
        self._overwrite = False

    def overwrite(self):
        self._overwrite = True
        return self

    def save(self, path: str):
        serialize.save_stage(self.stage, path, overwrite=self._overwrite)


class PipelineStage(Params):
    def __init__(self, uid: Optional[str] = None, **kwargs):
        super().__init__(uid=uid, **kwargs)
        self._init_state()

    def _init_state(self) -> None:
        """Non-param state; also called when loading a saved stage."""

    # persistence -----------------------------------------------------
    def save(self, path: str, overwrite: bool = False) -> None:
        serialize.save_stage(self, path, overwrite=overwrite)

    def write(self) -> _Writer:
        return _Writer(self)

    @classmethod
    def load(cls, path: str):
        obj = serialize.load_stage(path)
        if cls is not PipelineStage and not isinstance(obj, cls):
            raise TypeError(f"{path} holds a {type(obj).__name__}, not a {cls.__name__}")
        return obj

    @classmethod
    def read(cls):
        class _R:
            @staticmethod
            def load(path):
                return cls.load(path)

        return _R()

    def _save_extra(self, path: str) -> None:
        """Hook for stages with state beyond params."""

    def _load_extra(self, path: str) -> None:
        """Hook for stages with state beyond params."""

    def transformSchema(self, schema):  # noqa: N802
        return schema


class Transformer(PipelineStage):
    def transform(self, df: DataFrame, params: Optional[dict] = None) -> DataFrame:
        stage = self.copy(params) if params else self
        return log_verb(stage, "transform", lambda: stage._transform(df), df)

    def _transform(self, df: DataFrame) -> DataFrame:
        raise NotImplementedError


class Estimator(PipelineStage):
    def fit(self, df: DataFrame, params=None):
        if isinstance(params, (list, tuple)):
            return [self.fit(df, p) for p in params]
        stage = self.copy(params) if params else self
        return log_verb(stage, "fit", lambda: stage._fit(df), df)

    def _fit(self, df: DataFrame):
        raise NotImplementedError


class Model(Transformer):
    parent = None


class Evaluator(Params):
    def evaluate(self, df: DataFrame, params: Optional[dict] = None) -> float:
        stage = self.copy(params) if params else self
        return stage._evaluate(df)

    def _evaluate(self, df: DataFrame) -> float:
        raise NotImplementedError

    def isLargerBetter(self) -> bool:  # noqa: N802
        return True


class Pipeline(Estimator):
    stages = Param("pipeline stages", None, complex=True)

    def __init__(self, stages: Optional[List[PipelineStage]] = None, **kw):
        super().__init__(**kw)
        if stages is not None:
            self.setStages(stages)

    def getStages(self) -> List[PipelineStage]:  # noqa: N802
        return list(self.getOrDefault("stages") or [])

    def _fit(self, df: DataFrame) -> "PipelineModel":
        fitted = []
        cur = df
        stages = self.getStages()
        last_est = max((i for i, s in enumerate(stages) if isinstance(s, Estimator)), default=-1)
        for i, s in enumerate(stages):
            if isinstance(s, Estimator):
                m = s.fit(cur)
                fitted.append(m)
                if i < last_est:
                    cur = m.transform(cur)
            elif isinstance(s, Transformer):
                fitted.append(s)
                if i < last_est:
                    cur = s.transform(cur)
            else:
                raise TypeError(f"{s} is not a pipeline stage")
        return PipelineModel(stages=fitted)


class PipelineModel(Model):
    stages = Param("fitted pipeline stages", None, complex=True)

    def __init__(self, stages: Optional[List[Transformer]] = None, **kw):
        super().__init__(**kw)
        if stages is not None:
            self.set("stages", stages)

    def getStages(self) -> List[Transformer]:  # noqa: N802
        return list(self.getOrDefault("stages") or [])

    def _transform(self, df: DataFrame) -> DataFrame:
        for s in self.getStages():
            df = s.transform(df)
        return df
