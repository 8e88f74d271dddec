"""LangchainTransformer: run an LLM chain over a text column (reference:
cognitive/src/main/python/synapse/ml/services/langchain/LangchainTransform.py:114-288).

The ``langchain`` package is not installed in this image, so the stage is
duck-typed: ``chain`` is any object exposing ``invoke(x)`` (LCEL runnables),
``run(x)`` (legacy chains) or a plain callable. Behavior mirrors the
reference:
  * rows are evaluated independently; an exception from the chain is caught
    and its message goes to ``errorCol`` (the output is None for that row),
    like the reference's per-row ``error_message`` struct (LangchainTransform.py:234-275);
  * ``subscriptionKey`` / ``url`` / ``apiVersion`` are exported as the
    OpenAI environment variables the chain's LLM reads, for the duration of
    the transform only;
  * rows are evaluated on a small thread pool (``concurrency``), since chain
    calls are network-bound.
The chain persists as a complex param (our serializer's cloudpickle slot) —
the reference serializes it through langchain's own config loader instead.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from ..core.contracts import HasInputCol, HasOutputCol
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Transformer


def _call_chain(chain, x):
    if hasattr(chain, "invoke"):
        r = chain.invoke(x)
    elif hasattr(chain, "run"):
        r = chain.run(x)
    elif callable(chain):
        r = chain(x)
    else:
        raise TypeError(f"chain of type {type(chain).__name__} has no invoke/run and is not callable")
    if isinstance(r, dict) and len(r) == 1:  # chains return {output_key: text}
        r = next(iter(r.values()))
    return getattr(r, "content", r)  # chat messages carry their text in .content


class LangchainTransformer(Transformer, HasInputCol, HasOutputCol):
    chain = Param("Langchain chain (any object with invoke/run, or a callable)", None, complex=True)
    subscriptionKey = Param("openai api key", None, T.toString)
    url = Param("openai api base", None, T.toString)
    apiVersion = Param("openai api version", None, T.toString)
    errorCol = Param("column for error", "errorCol", T.toString)
    concurrency = Param("rows evaluated concurrently", 1, T.toInt)

    def _env(self):
        env = {}
        if self.getSubscriptionKey():
            env["OPENAI_API_KEY"] = self.getSubscriptionKey()
        if self.getUrl():
            env["OPENAI_API_BASE"] = self.getUrl()
            env["AZURE_OPENAI_ENDPOINT"] = self.getUrl()
        if self.getApiVersion():
            env["OPENAI_API_VERSION"] = self.getApiVersion()
        if env:
            env["OPENAI_API_TYPE"] = "azure"
        return env

    def _transform(self, df):
        chain = self.getChain()
        if chain is None:
            raise ValueError("LangchainTransformer: chain is not set")
        xs = df[self.getInputCol()].tolist()
        n = len(xs)
        out = np.empty(n, dtype=object)
        err = np.empty(n, dtype=object)

        def one(i):
            try:
                out[i], err[i] = _call_chain(chain, xs[i]), None
            except Exception as e:  # per-row failure -> errorCol, like the reference's error struct
                out[i], err[i] = None, f"{type(e).__name__}: {e}"

        env = self._env()
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            workers = max(1, int(self.getConcurrency()))
            if workers == 1 or n < 2:
                for i in range(n):
                    one(i)
            else:
                with ThreadPoolExecutor(min(workers, n)) as ex:
                    list(ex.map(one, range(n)))
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        return df.withColumn(self.getOutputCol(), out).withColumn(self.getErrorCol(), err)
