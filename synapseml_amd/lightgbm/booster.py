"""Python handle of a trained ensemble (reference:
lightgbm/.../booster/LightGBMBooster.scala). The model is persisted as the
LightGBM v3 text model; the native handle is created lazily from it (the
reference's @transient boosterHandler), and whole batches are scored in one
call - on the MI355X through the K9 kernel when a GPU is present."""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

from ..ops import native

_GPU_BATCH_MIN_ROWS = 4096


class LightGBMBooster:
    def __init__(self, model_str: Optional[str] = None, native_booster=None, best_iteration: int = -1):
        if model_str is None and native_booster is None:
            raise ValueError("need a model string or a native booster")
        self._model_str = model_str
        self._native = native_booster
        self._gpu_predictors = {}
        self.bestIteration = best_iteration
        self.startIteration = 0
        self.numIterations = -1

    # ------------------------------------------------------------- native handle
    @property
    def native(self):
        if self._native is None:
            self._native = native.gbdt().Booster.from_model_string(self._model_str)
        return self._native

    @property
    def modelStr(self) -> str:  # noqa: N802
        if self._model_str is None:
            self._model_str = self._native.save_model_string(0, -1, 0)
        return self._model_str

    def __getstate__(self):
        return {"model_str": self.modelStr, "best": self.bestIteration}

    def __setstate__(self, st):
        self.__init__(st["model_str"], best_iteration=st.get("best", -1))

    # persistence protocol used by core.serialize for complex params
    def _sml_save(self, d: str) -> None:
        with open(os.path.join(d, "model.txt"), "w") as f:
            f.write(self.modelStr)
        with open(os.path.join(d, "best_iteration"), "w") as f:
            f.write(str(self.bestIteration))

    @classmethod
    def _sml_load(cls, d: str) -> "LightGBMBooster":
        with open(os.path.join(d, "model.txt")) as f:
            s = f.read()
        best = -1
        p = os.path.join(d, "best_iteration")
        if os.path.exists(p):
            with open(p) as f:
                best = int(f.read().strip() or -1)
        return cls(s, best_iteration=best)

    # ------------------------------------------------------------- properties
    @property
    def numClasses(self) -> int:  # noqa: N802
        return self.native.num_classes

    @property
    def numFeatures(self) -> int:  # noqa: N802
        return self.native.num_features

    @property
    def numTotalModel(self) -> int:  # noqa: N802
        return self.native.num_total_model

    @property
    def numModelPerIteration(self) -> int:  # noqa: N802
        return self.native.num_model_per_iteration

    @property
    def numTotalIterations(self) -> int:  # noqa: N802
        return self.native.current_iteration

    def setStartIteration(self, v: int):  # noqa: N802
        self.startIteration = int(v)

    def setNumIterations(self, v: int):  # noqa: N802
        self.numIterations = int(v)

    # ------------------------------------------------------------- scoring
    def _shape(self, X: np.ndarray, disable_shape_check: bool, keep_f32: bool = False) -> np.ndarray:
        """float64 rows (float32 kept as is when the device path scores them: no host conversion copy)"""
        X = np.asarray(X)
        X = np.ascontiguousarray(X) if (keep_f32 and X.dtype == np.float32) else np.ascontiguousarray(X, dtype=np.float64)
        if X.ndim == 1:
            X = X[None, :]
        nf = self.numFeatures
        if X.shape[1] != nf:
            if not disable_shape_check:
                raise ValueError(
                    f"The number of features in data ({X.shape[1]}) is not the same as it was in training data "
                    f"({nf}). You can set ``predictDisableShapeCheck=true`` to discard this error")
            if X.shape[1] < nf:
                X = np.concatenate([X, np.zeros((X.shape[0], nf - X.shape[1]), dtype=X.dtype)], axis=1)
        return X

    def _gpu(self, device: str):
        if device != "gpu" or not native.gpu_available():
            return None
        key = (self.startIteration, self.numIterations)
        p = self._gpu_predictors.get(key)
        if p is None:
            p = native.gbdt().GpuPredictor(self.native, self.startIteration, self.numIterations, -1)
            self._gpu_predictors[key] = p
        return p

    def _gpu_for(self, X, device: str):
        n = np.shape(X)[0] if np.ndim(X) == 2 else 1
        return self._gpu(device) if n >= _GPU_BATCH_MIN_ROWS else None

    def predict_raw(self, X, disable_shape_check=False, device="gpu") -> np.ndarray:
        gp = self._gpu_for(X, device)
        if gp is not None:  # one device pass over the rows in their own dtype (float32 stays float32)
            return gp.predict_raw(self._shape(X, disable_shape_check, keep_f32=True))
        return self.native.predict(self._shape(X, disable_shape_check), 0, self.startIteration, self.numIterations)

    def predict_normal(self, X, disable_shape_check=False, device="gpu") -> np.ndarray:
        gp = self._gpu_for(X, device)
        if gp is not None:
            return self.native.convert_outputs(gp.predict_raw(self._shape(X, disable_shape_check, keep_f32=True)))
        return self.native.predict(self._shape(X, disable_shape_check), 1, self.startIteration, self.numIterations)

    def predict_raw_and_normal(self, X, disable_shape_check=False, device="gpu"):
        """(raw, transformed) outputs from ONE ensemble pass: the device (or host) computes the raw scores
        and the objective's transform is applied to them (LightGBMBooster.scala:394-405 scores twice)."""
        raw = self.predict_raw(X, disable_shape_check, device)
        return raw, self.native.convert_outputs(np.ascontiguousarray(raw))

    def score(self, X, raw: bool, classification: bool, disable_shape_check: bool = False,
              device: str = "gpu") -> np.ndarray:
        """Batch version of LightGBMBooster.score (Scala :394-405, :559-575):
        binary classification expands to two columns, [-r, r] or [1-p, p]."""
        out = self.predict_raw(X, disable_shape_check, device) if raw else self.predict_normal(X, disable_shape_check, device)
        return self._expand(out, raw, classification)

    @staticmethod
    def _expand(out, raw: bool, classification: bool):
        if classification and out.shape[1] == 1:
            if raw:
                return np.concatenate([-out, out], axis=1)
            return np.concatenate([1.0 - out, out], axis=1)
        return out

    def score_both(self, X, classification: bool, disable_shape_check: bool = False, device: str = "gpu"):
        """(rawPrediction, probability) of a batch from a single ensemble pass"""
        r, p = self.predict_raw_and_normal(X, disable_shape_check, device)
        return self._expand(r, True, classification), self._expand(p, False, classification)

    def predictLeaf(self, X, disable_shape_check=False, device="gpu") -> np.ndarray:  # noqa: N802
        X = self._shape(X, disable_shape_check)
        gp = self._gpu(device) if X.shape[0] >= _GPU_BATCH_MIN_ROWS else None
        if gp is not None:
            return gp.predict_leaf(X).astype(np.float64)
        return self.native.predict(X, 2, self.startIteration, self.numIterations)

    def featuresShap(self, X, disable_shape_check=False, device="gpu") -> np.ndarray:  # noqa: N802
        """TreeSHAP contributions, (numFeatures + 1) * numClasses per row (last
        column of each class block is the expected value). Batches go to the
        HIP TreeSHAP kernel (K10, ``csrc/gbdt/predict_gpu.hip``)."""
        X = self._shape(X, disable_shape_check)
        gp = self._gpu(device) if X.shape[0] >= _GPU_BATCH_MIN_ROWS else None
        if gp is not None:
            out = gp.predict_contrib(self.native, X)
            if out is not None:
                return out
        return self.native.predict(X, 3, self.startIteration, self.numIterations)

    def getFeatureImportances(self, importance_type: str = "split") -> np.ndarray:  # noqa: N802
        t = 0 if importance_type == "split" else 1
        return np.asarray(self.native.feature_importance(-1, t))

    def saveNativeModel(self, filename: str, overwrite: bool = True) -> None:  # noqa: N802
        if os.path.exists(filename) and not overwrite:
            raise FileExistsError(filename)
        with open(filename, "w") as f:
            f.write(self.modelStr)

    def dumpModel(self) -> str:  # noqa: N802
        return self.native.dump_model(0, -1)

    def getNativeModel(self) -> str:  # noqa: N802
        return self.modelStr
