"""Azure OpenAI transformers (reference: cognitive/.../services/openai/
{OpenAI, OpenAICompletion, OpenAIChatCompletion, OpenAIEmbedding,
OpenAIPrompt}.scala).

URL: ``{url}openai/deployments/{deploymentName}/{completions|chat/completions|
embeddings}?api-version=...``; the key goes in the ``api-key`` header.
Optional generation params are sent snake_cased (``maxTokens`` → max_tokens,
``logProbs`` → logprobs)."""
from __future__ import annotations

import csv
import io
import json
import re
from typing import Any, Dict

import numpy as np

from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Transformer
from .base import CognitiveServicesBase, HasAPIVersion, ServiceParam

_DEFAULTS: Dict[str, Any] = {}


class OpenAIDefaults:
    """Process-wide defaults applied to new OpenAI transformers (reference: OpenAIDefaults.scala)."""

    @staticmethod
    def set(name: str, value) -> None:
        _DEFAULTS[name] = value

    @staticmethod
    def get(name: str):
        return _DEFAULTS.get(name)

    @staticmethod
    def reset(name: str = None) -> None:
        if name is None:
            _DEFAULTS.clear()
        else:
            _DEFAULTS.pop(name, None)

    # reference-style accessors
    setDeploymentName = staticmethod(lambda v: OpenAIDefaults.set("deploymentName", v))  # noqa: N815
    setSubscriptionKey = staticmethod(lambda v: OpenAIDefaults.set("subscriptionKey", v))  # noqa: N815
    setTemperature = staticmethod(lambda v: OpenAIDefaults.set("temperature", v))  # noqa: N815
    setURL = staticmethod(lambda v: OpenAIDefaults.set("url", v))  # noqa: N815


def _snake(name: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


class _OpenAIBase(CognitiveServicesBase, HasAPIVersion):
    subscription_key_header = "api-key"
    endpoint_suffix = "completions"
    deploymentName = ServiceParam("The name of the deployment", required=True)
    user = ServiceParam("The ID of the end-user, for use in tracking and rate-limiting.")

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(apiVersion={"kind": "value", "value": "2024-02-01"}, timeout=360.0)
        for k, v in _DEFAULTS.items():
            if k == "url":
                self._setDefault(url=v)
            elif self.hasParam(k):
                self._setDefault(**{k: {"kind": "value", "value": v}})

    def setCustomServiceName(self, name: str):  # noqa: N802
        return self.setUrl(f"https://{name}.openai.azure.com/")

    def _base_url(self, vals):
        u = self.getUrl()
        if not u:
            raise ValueError(f"{type(self).__name__}: url is not set")
        return f"{u.rstrip('/')}/openai/deployments/{vals['deploymentName']}/{self.endpoint_suffix}"


class _TextParams(_OpenAIBase):
    maxTokens = ServiceParam("The maximum number of tokens to generate. Has minimum of 0.")
    temperature = ServiceParam("What sampling temperature to use.")
    stop = ServiceParam("A sequence which indicates the end of the current document.")
    topP = ServiceParam("An alternative to sampling with temperature, called nucleus sampling")
    n = ServiceParam("How many snippets to generate for each prompt. Minimum of 1 and maximum of 128 allowed.")
    logProbs = ServiceParam("Include the log probabilities on the logprobs most likely tokens")
    echo = ServiceParam("Echo back the prompt in addition to the completion")
    cacheLevel = ServiceParam("can be used to disable any server-side caching, 0=no cache, 1=prompt prefix "
                              "enabled, 2=full cache")
    presencePenalty = ServiceParam("How much to penalize new tokens based on their existing frequency")
    frequencyPenalty = ServiceParam("How much to penalize new tokens based on whether they appear in the text")
    bestOf = ServiceParam("How many generations to create server side, and display only the best.")

    _optional = ("maxTokens", "temperature", "topP", "user", "n", "echo", "stop", "cacheLevel", "presencePenalty",
                 "frequencyPenalty", "bestOf")

    def _optional_params(self, vals):
        out = {_snake(k): vals[k] for k in self._optional if k in vals}
        if "logProbs" in vals:
            out["logprobs"] = vals["logProbs"]
        return out


class OpenAICompletion(_TextParams):
    prompt = ServiceParam("The text to complete")
    batchPrompt = ServiceParam("Sequence of prompts to complete")

    def _should_skip(self, vals):
        return "deploymentName" not in vals or ("prompt" not in vals and "batchPrompt" not in vals)

    def _entity(self, vals):
        body = self._optional_params(vals)
        body["prompt"] = vals["prompt"] if "prompt" in vals else list(vals["batchPrompt"])
        return json.dumps(body).encode("utf-8"), "application/json"


class OpenAIChatCompletion(_TextParams):
    endpoint_suffix = "chat/completions"
    messages = ServiceParam("list of {role, content, name} chat messages", required=True)

    def _entity(self, vals):
        msgs = [{k: m[k] for k in ("role", "content", "name") if m.get(k) is not None} for m in vals["messages"]]
        body = self._optional_params(vals)
        body["messages"] = msgs
        return json.dumps(body).encode("utf-8"), "application/json"


class OpenAIEmbedding(_OpenAIBase):
    endpoint_suffix = "embeddings"
    text = ServiceParam("Input text to get embeddings for.", required=True)
    dimensions = ServiceParam("Number of dimensions for output embeddings.")

    def _entity(self, vals):
        body = {"input": vals["text"]}
        for k in ("user", "dimensions"):
            if k in vals:
                body[k] = vals[k]
        return json.dumps(body).encode("utf-8"), "application/json"

    def _postprocess(self, parsed, vals):
        """The embedding vector (float32) of the first (only) input."""
        try:
            return np.asarray(parsed["data"][0]["embedding"], dtype=np.float32)
        except (KeyError, IndexError, TypeError):
            return None


class OpenAIPrompt(Transformer):
    """Fill ``promptTemplate`` ({col} placeholders) per row, complete it, post-process the first choice's text
    (csv → list, json → parsed object, regex → group, '' → text)."""

    promptTemplate = Param("The prompt. supports string interpolation {col1}: {col2}.", None, T.toString)
    postProcessing = Param("Post processing options for output: csv, json, regex or ''", "", T.toString)
    postProcessingOptions = Param("Options (default): delimiter=',', jsonSchema, regex, regexGroup=0", {},
                                  T.identity)
    dropPrompt = Param("whether to drop the column of prompts after templating", True, T.toBoolean)
    outputCol = Param("The name of the output column", None, T.toString)
    completion = Param("configured OpenAICompletion (or chat completion) used for the calls", None, complex=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol=self.uid + "_output")

    def _template(self, row: Dict[str, Any]) -> str:
        return re.sub(r"\{(\w+)\}", lambda m: str(row.get(m.group(1), m.group(0))), self.getPromptTemplate())

    def _parse(self, text):
        if text is None:
            return None
        kind = (self.getPostProcessing() or "").lower()
        opts = self.getPostProcessingOptions() or {}
        if kind == "csv":
            return next(csv.reader(io.StringIO(text.strip()), delimiter=opts.get("delimiter", ",")), [])
        if kind == "json":
            try:
                return json.loads(text)
            except ValueError:
                return None
        if kind == "regex":
            m = re.search(opts["regex"], text)
            return m.group(int(opts.get("regexGroup", 0))) if m else ""
        if kind == "":
            return text
        raise ValueError(f"Unsupported postProcessing type: '{self.getPostProcessing()}'")

    def _transform(self, df):
        comp = self.getCompletion()
        if comp is None:
            raise ValueError("OpenAIPrompt: set completion (a configured OpenAICompletion / OpenAIChatCompletion)")
        cols = df.columns
        data = {c: df[c].tolist() for c in cols}
        prompts = [self._template({c: data[c][i] for c in cols}) for i in range(df.count())]
        pcol = "_prompt_" + self.uid[-6:]
        arr = np.empty(len(prompts), dtype=object)
        for i, p in enumerate(prompts):
            arr[i] = p if not isinstance(comp, OpenAIChatCompletion) else [{"role": "user", "content": p}]
        comp = comp.copy()
        if isinstance(comp, OpenAIChatCompletion):
            comp.setMessagesCol(pcol)
        else:
            comp.setPromptCol(pcol)
        out = comp.transform(df.withColumn(pcol, arr))
        texts = []
        for r in out[comp.getOutputCol()].tolist():
            try:
                ch = r["choices"][0]
                texts.append(ch["message"]["content"] if "message" in ch else ch["text"])
            except (KeyError, IndexError, TypeError):
                texts.append(None)
        parsed = np.empty(len(texts), dtype=object)
        for i, t in enumerate(texts):
            parsed[i] = self._parse(t)
        out = out.withColumn(self.getOutputCol(), parsed).drop(comp.getOutputCol())
        return out.drop(pcol) if self.getDropPrompt() else out.withColumnRenamed(pcol, "prompt")


__all__ = ["OpenAICompletion", "OpenAIChatCompletion", "OpenAIEmbedding", "OpenAIPrompt", "OpenAIDefaults"]
