"""Text Analytics v3.1, Language (analyze-text) and Translator transformers
(reference: cognitive/.../services/text/TextAnalytics.scala:28-703,
language/AnalyzeText.scala, translate/TextTranslator.scala:22-577,
translate/DocumentTranslator.scala).

Text Analytics: ``text`` may be a string (one document per row; the output
is that document's result, or its error object) or a list of strings (the
output is the list of per-document results, in input order)."""
from __future__ import annotations

import json
from typing import Any, Dict, List

from ..core.params import Param, TypeConverters as T
from .base import CognitiveServicesBase, HasAPIVersion, HasAsyncReply, ServiceParam


def _docs(vals: Dict[str, Any]) -> List[dict]:
    text = vals["text"]
    texts = [text] if isinstance(text, str) else list(text)
    lang = vals.get("language")
    if lang is None:
        langs = [None] * len(texts)
    elif isinstance(lang, str):
        langs = [lang] * len(texts)
    else:
        langs = list(lang) if len(lang) == len(texts) else [lang[0]] * len(texts)
    out = []
    for i, (t, l) in enumerate(zip(texts, langs)):
        d = {"id": str(i), "text": t}
        if l:
            d["language"] = l
        out.append(d)
    return out


def _unpack(resp: dict, vals: Dict[str, Any]):
    """Per-document results in input order (errors in place of failed documents)."""
    if not isinstance(resp, dict):
        return resp
    by_id = {d.get("id"): d for d in resp.get("documents", [])}
    by_id.update({e.get("id"): {"id": e.get("id"), "error": e.get("error")} for e in resp.get("errors", [])})
    n = 1 if isinstance(vals["text"], str) else len(vals["text"])
    docs = [by_id.get(str(i)) for i in range(n)]
    return docs[0] if isinstance(vals["text"], str) else docs


class TextAnalyticsBase(CognitiveServicesBase):
    text = ServiceParam("the text in the request body", required=True)
    language = ServiceParam("the language code of the text (optional for some services)")
    modelVersion = ServiceParam("Version of the model", url_param=True, payload_name="model-version")
    showStats = ServiceParam("Whether to include detailed statistics in the response", url_param=True)
    disableServiceLogs = ServiceParam("disables service logging of the input text", url_param=True,
                                      payload_name="loggingOptOut")

    def _entity(self, vals):
        return json.dumps({"documents": _docs(vals)}).encode("utf-8"), "application/json"

    def _postprocess(self, parsed, vals):
        return _unpack(parsed, vals)


class TextSentiment(TextAnalyticsBase):
    url_path = "/text/analytics/v3.1/sentiment"
    opinionMining = ServiceParam("if set to true, response will contain input and document level sentiment",
                                 url_param=True)
    stringIndexType = ServiceParam("Specifies the method used to interpret string offsets", url_param=True)


class KeyPhraseExtractor(TextAnalyticsBase):
    url_path = "/text/analytics/v3.1/keyPhrases"


class NER(TextAnalyticsBase):
    url_path = "/text/analytics/v3.1/entities/recognition/general"
    stringIndexType = ServiceParam("Specifies the method used to interpret string offsets", url_param=True)


class PII(TextAnalyticsBase):
    url_path = "/text/analytics/v3.1/entities/recognition/pii"
    domain = ServiceParam("if specified, will set the PII domain to include only a subset of the entity "
                          "categories ('phi', 'none')", url_param=True)
    piiCategories = ServiceParam("describes the PII categories to return", url_param=True)
    stringIndexType = ServiceParam("Specifies the method used to interpret string offsets", url_param=True)


class LanguageDetector(TextAnalyticsBase):
    url_path = "/text/analytics/v3.1/languages"

    def _entity(self, vals):
        docs = [{"id": d["id"], "text": d["text"]} for d in _docs(vals)]
        return json.dumps({"documents": docs}).encode("utf-8"), "application/json"


class EntityDetector(TextAnalyticsBase):
    url_path = "/text/analytics/v3.1/entities/linking"
    stringIndexType = ServiceParam("Specifies the method used to interpret string offsets", url_param=True)


class AnalyzeHealthText(TextAnalyticsBase, HasAsyncReply):
    url_path = "/text/analytics/v3.1/entities/health/jobs"

    def _postprocess(self, parsed, vals):
        return _unpack(parsed.get("results", parsed) if isinstance(parsed, dict) else parsed, vals)


_ANALYZE_TASKS = (  # (include param, params param, request task list, output field)
    ("includeEntityRecognition", "entityRecognitionParams", "entityRecognitionTasks", "entityRecognition"),
    ("includeEntityLinking", "entityLinkingParams", "entityLinkingTasks", "entityLinking"),
    ("includePii", "piiParams", "entityRecognitionPiiTasks", "pii"),
    ("includeKeyPhraseExtraction", "keyPhraseExtractionParams", "keyPhraseExtractionTasks", "keyPhraseExtraction"),
    ("includeSentimentAnalysis", "sentimentAnalysisParams", "sentimentAnalysisTasks", "sentimentAnalysis"),
)


class TextAnalyze(TextAnalyticsBase, HasAsyncReply):
    """Several Text Analytics tasks over the same documents in one asynchronous ``/analyze`` job
    (reference: TextAnalytics.scala:488-703). The output holds, per document, one record with
    ``entityRecognition``, ``entityLinking``, ``pii``, ``keyPhraseExtraction`` and
    ``sentimentAnalysis`` (null for tasks that were not included), each that task's per-document
    result (the reference's UnpackedTextAnalyzeResponse)."""

    url_path = "/text/analytics/v3.1/analyze"
    includeEntityRecognition = Param("Whether to perform entity recognition", True, T.toBoolean)
    entityRecognitionParams = Param("the parameters to pass to the entity recognition model",
                                    {"model-version": "latest"}, T.toDictStrStr)
    includePii = Param("Whether to perform PII Detection", True, T.toBoolean)
    piiParams = Param("the parameters to pass to the PII model", {"model-version": "latest"}, T.toDictStrStr)
    includeEntityLinking = Param("Whether to perform EntityLinking", True, T.toBoolean)
    entityLinkingParams = Param("the parameters to pass to the entityLinking model",
                                {"model-version": "latest"}, T.toDictStrStr)
    includeKeyPhraseExtraction = Param("Whether to perform KeyPhraseExtraction", True, T.toBoolean)
    keyPhraseExtractionParams = Param("the parameters to pass to the keyPhraseExtraction model",
                                      {"model-version": "latest"}, T.toDictStrStr)
    includeSentimentAnalysis = Param("Whether to perform SentimentAnalysis", True, T.toBoolean)
    sentimentAnalysisParams = Param("the parameters to pass to the sentimentAnalysis model",
                                    {"model-version": "latest"}, T.toDictStrStr)

    def _entity(self, vals):
        tasks = {}
        for inc, prm, key, _ in _ANALYZE_TASKS:
            tasks[key] = [{"parameters": dict(self.getOrDefault(prm))}] if self.getOrDefault(inc) else []
        body = {"displayName": "SynapseML", "analysisInput": {"documents": _docs(vals)}, "tasks": tasks}
        return json.dumps(body).encode("utf-8"), "application/json"

    def _modify_polling_url(self, url: str) -> str:
        # the job pages 20 documents by default; the API takes the first $top it sees
        base, _, query = url.partition("?")
        return base + "?$top=25" + ("&" + query if query else "")

    def _postprocess(self, parsed, vals):
        if not isinstance(parsed, dict) or "tasks" not in parsed:
            return parsed
        tasks = parsed["tasks"]
        per_task = {}
        for _, _, key, field in _ANALYZE_TASKS:
            lst = tasks.get(key) or []
            per_task[field] = _unpack(lst[0].get("results", {}), dict(vals, text=vals["text"])) if lst else None
        single = isinstance(vals["text"], str)
        n = 1 if single else len(vals["text"])
        docs = []
        for i in range(n):
            docs.append({f: (None if r is None else (r if single else r[i])) for f, r in per_task.items()})
        return docs[0] if single else docs


class AnalyzeText(CognitiveServicesBase, HasAPIVersion):
    """Language service ``:analyze-text`` (kind = SentimentAnalysis, KeyPhraseExtraction, EntityRecognition,
    PiiEntityRecognition, LanguageDetection, EntityLinking)."""

    url_path = "/language/:analyze-text"
    text = ServiceParam("the text in the request body", required=True)
    language = ServiceParam("the language code of the text")
    kind = ServiceParam("Enumeration of supported Text Analysis tasks", required=True)
    modelVersion = ServiceParam("Version of the model")
    loggingOptOut = ServiceParam("loggingOptOut for task")
    stringIndexType = ServiceParam("Specifies the method used to interpret string offsets.")
    opinionMining = ServiceParam("opinionMining option for SentimentAnalysisTask")
    domain = ServiceParam("domain option for PiiEntityRecognitionTask")
    piiCategories = ServiceParam("piiCategories option for PiiEntityRecognitionTask")
    showStats = ServiceParam("Whether to include detailed statistics in the response", url_param=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(apiVersion={"kind": "value", "value": "2022-05-01"})

    def _entity(self, vals):
        docs = _docs(vals)
        if vals["kind"] == "LanguageDetection":
            docs = [{"id": d["id"], "text": d["text"]} for d in docs]
        params = {k: vals[k] for k in ("modelVersion", "loggingOptOut", "stringIndexType", "opinionMining",
                                      "domain", "piiCategories") if k in vals}
        body = {"kind": vals["kind"], "analysisInput": {"documents": docs}, "parameters": params}
        return json.dumps(body).encode("utf-8"), "application/json"

    def _postprocess(self, parsed, vals):
        if isinstance(parsed, dict) and "results" in parsed:
            return _unpack(parsed["results"], vals)
        return parsed


# ---------------------------------------------------------------------- Translator
class _TranslatorBase(CognitiveServicesBase, HasAPIVersion):
    host_template = "https://api.cognitive.microsofttranslator.com/"
    subscriptionRegion = ServiceParam("the API region to use")
    text = ServiceParam("the string to translate", required=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(apiVersion={"kind": "value", "value": "3.0"})

    def setLocation(self, location: str):  # noqa: N802 - translator is global; location = region header
        self.setSubscriptionRegion(location)
        return self.setUrl(self.host_template + self.url_path.lstrip("/"))

    def _headers(self, vals, content_type):
        h = super()._headers(vals, content_type)
        if vals.get("subscriptionRegion"):
            h["Ocp-Apim-Subscription-Region"] = vals["subscriptionRegion"]
        return h

    def _texts(self, vals):
        t = vals["text"]
        return [t] if isinstance(t, str) else list(t)

    def _entity(self, vals):
        return json.dumps([{"Text": t} for t in self._texts(vals)]).encode("utf-8"), "application/json"


class Translate(_TranslatorBase):
    url_path = "/translate"
    toLanguage = ServiceParam("Specifies the language of the output text", required=True, url_param=True,
                              payload_name="to")
    fromLanguage = ServiceParam("Specifies the language of the input text", url_param=True, payload_name="from")
    textType = ServiceParam("Defines whether the text being translated is plain text or HTML text", url_param=True)
    category = ServiceParam("A string specifying the category (domain) of the translation", url_param=True)
    profanityAction = ServiceParam("Specifies how profanities should be treated", url_param=True)
    profanityMarker = ServiceParam("Specifies how profanities should be marked", url_param=True)
    includeAlignment = ServiceParam("Specifies whether to include alignment projection", url_param=True)
    includeSentenceLength = ServiceParam("Specifies whether to include sentence boundaries", url_param=True)
    suggestedFrom = ServiceParam("Specifies a fallback language", url_param=True)
    fromScript = ServiceParam("Specifies the script of the input text", url_param=True)
    toScript = ServiceParam("Specifies the script of the translated text", url_param=True)
    allowFallback = ServiceParam("Specifies that the service is allowed to fall back to a general system",
                                 url_param=True)


class Transliterate(_TranslatorBase):
    url_path = "/transliterate"
    language = ServiceParam("Language tag of the text", required=True, url_param=True)
    fromScript = ServiceParam("Specifies the script used by the input text", required=True, url_param=True)
    toScript = ServiceParam("Specifies the output script", required=True, url_param=True)


class Detect(_TranslatorBase):
    url_path = "/detect"


class BreakSentence(_TranslatorBase):
    url_path = "/breaksentence"
    language = ServiceParam("Language tag identifying the language of the input text", url_param=True)
    script = ServiceParam("Script tag identifying the script used by the input text", url_param=True)


class DictionaryLookup(_TranslatorBase):
    url_path = "/dictionary/lookup"
    fromLanguage = ServiceParam("Specifies the language of the input text", required=True, url_param=True,
                                payload_name="from")
    toLanguage = ServiceParam("Specifies the language of the output text", required=True, url_param=True,
                              payload_name="to")


class DictionaryExamples(_TranslatorBase):
    url_path = "/dictionary/examples"
    fromLanguage = ServiceParam("Specifies the language of the input text", required=True, url_param=True,
                                payload_name="from")
    toLanguage = ServiceParam("Specifies the language of the output text", required=True, url_param=True,
                              payload_name="to")
    textAndTranslation = ServiceParam("list of (text, translation) pairs", required=True)
    text = ServiceParam("unused for examples", required=False)

    def _entity(self, vals):
        pairs = vals["textAndTranslation"]
        if isinstance(pairs, dict) or (len(pairs) == 2 and isinstance(pairs[0], str)):
            pairs = [pairs]
        body = [{"Text": p["text"], "Translation": p["translation"]} if isinstance(p, dict)
                else {"Text": p[0], "Translation": p[1]} for p in pairs]
        return json.dumps(body).encode("utf-8"), "application/json"


class DocumentTranslator(CognitiveServicesBase, HasAsyncReply):
    """Batch document translation: POST translator/text/batch/v1.0/batches, then poll the operation."""

    url_path = "/translator/text/batch/v1.0/batches"
    serviceName = ServiceParam("the name of the translator resource")
    sourceUrl = ServiceParam("Location of the folder / container or single file with your documents",
                             required=True)
    sourceLanguage = ServiceParam("Language code of the source documents")
    targets = ServiceParam("Destination(s) for the finished translated documents: list of "
                           "{targetUrl, language, category, glossaries}", required=True)
    storageType = ServiceParam("Storage type of the input documents source string (Folder|File)")
    filterPrefix = ServiceParam("A case-sensitive prefix string to filter documents")
    filterSuffix = ServiceParam("A case-sensitive suffix string to filter documents")

    def setServiceName(self, name: str):  # noqa: N802
        self.set("serviceName", {"kind": "value", "value": name})
        return self.setUrl(f"https://{name}.cognitiveservices.azure.com/" + self.url_path.lstrip("/"))

    def _entity(self, vals):
        src = {"sourceUrl": vals["sourceUrl"]}
        if "sourceLanguage" in vals:
            src["language"] = vals["sourceLanguage"]
        flt = {k: vals[f"filter{k.capitalize()}"] for k in ("prefix", "suffix") if f"filter{k.capitalize()}" in vals}
        if flt:
            src["filter"] = flt
        inp = {"source": src, "targets": vals["targets"]}
        if "storageType" in vals:
            inp["storageType"] = vals["storageType"]
        return json.dumps({"inputs": [inp]}).encode("utf-8"), "application/json"


__all__ = ["TextSentiment", "KeyPhraseExtractor", "NER", "PII", "LanguageDetector", "EntityDetector",
           "AnalyzeHealthText", "AnalyzeText", "Translate", "Transliterate", "Detect", "BreakSentence",
           "DictionaryLookup", "DictionaryExamples", "DocumentTranslator"]
