"""Form Recognizer v2.1 / Document Intelligence v3 transformers and the form
ontology learner (reference: cognitive/.../services/form/FormRecognizer.scala,
FormRecognizerV3.scala, FormOntologyLearner.scala).

All analyze calls are asynchronous: POST returns 202 + Operation-Location,
polled until the status is terminal."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np

from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model
from .base import CognitiveServicesBase, HasAPIVersion, HasAsyncReply, ServiceParam
from .vision import _ImageInput


class _FormBase(_ImageInput, HasAsyncReply):
    """imageUrl / imageBytes from the vision base: same {"url"} / octet-stream entity."""

    def _entity(self, vals):
        import json

        if vals.get("imageBytes") is not None:
            return bytes(vals["imageBytes"]), "application/octet-stream"
        key = "urlSource" if isinstance(self, AnalyzeDocument) else "source"
        return json.dumps({key: vals["imageUrl"]}).encode("utf-8"), "application/json"


class AnalyzeLayout(_FormBase):
    url_path = "/formrecognizer/v2.1/layout/analyze"
    language = ServiceParam("The BCP-47 language code of the text in the document.", url_param=True)
    pages = ServiceParam("The page selection only leveraged for multi-page PDF and TIFF documents.",
                         url_param=True)
    readingOrder = ServiceParam("Optional parameter to specify which reading order algorithm should be applied",
                                url_param=True)


class _Prebuilt(_FormBase):
    includeTextDetails = ServiceParam("Include text lines and element references in the result.", url_param=True)
    locale = ServiceParam("Locale of the receipt. Supported locales: en-AU, en-CA, en-GB, en-IN, en-US.",
                          url_param=True)
    pages = ServiceParam("The page selection only leveraged for multi-page PDF and TIFF documents.",
                         url_param=True)


class AnalyzeReceipts(_Prebuilt):
    url_path = "/formrecognizer/v2.1/prebuilt/receipt/analyze"


class AnalyzeBusinessCards(_Prebuilt):
    url_path = "/formrecognizer/v2.1/prebuilt/businessCard/analyze"


class AnalyzeInvoices(_Prebuilt):
    url_path = "/formrecognizer/v2.1/prebuilt/invoice/analyze"


class AnalyzeIDDocuments(_FormBase):
    url_path = "/formrecognizer/v2.1/prebuilt/idDocument/analyze"
    includeTextDetails = ServiceParam("Include text lines and element references in the result.", url_param=True)
    pages = ServiceParam("The page selection only leveraged for multi-page PDF and TIFF documents.",
                         url_param=True)


class AnalyzeCustomModel(_FormBase):
    url_path = "/formrecognizer/v2.1/custom/models/"
    modelId = ServiceParam("Model identifier.", required=True)
    includeTextDetails = ServiceParam("Include text lines and element references in the result.", url_param=True)

    def _base_url(self, vals):
        return self.getUrl().rstrip("/") + "/" + vals["modelId"] + "/analyze"


class GetCustomModel(CognitiveServicesBase):
    url_path = "/formrecognizer/v2.1/custom/models/"
    method = "GET"
    modelId = ServiceParam("Model identifier.", required=True)
    includeKeys = ServiceParam("Include list of extracted keys in model information.", url_param=True)

    def _base_url(self, vals):
        return self.getUrl().rstrip("/") + "/" + vals["modelId"]


class ListCustomModels(CognitiveServicesBase):
    url_path = "/formrecognizer/v2.1/custom/models"
    method = "GET"
    op = ServiceParam("Specify whether to return summary or full list of models.", url_param=True)


class AnalyzeDocument(_FormBase, HasAPIVersion):
    url_path = "/formrecognizer/documentModels/"
    prebuiltModelId = ServiceParam("Prebuilt model identifier for Form Recognizer V3.0, e.g. prebuilt-layout, "
                                   "prebuilt-invoice, prebuilt-read", required=True)
    pages = ServiceParam("The page selection only leveraged for multi-page PDF and TIFF documents.",
                         url_param=True)
    locale = ServiceParam("Locale hint for text recognition and document analysis.", url_param=True)
    stringIndexType = ServiceParam("Method used to compute string offset and length.", url_param=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(apiVersion={"kind": "value", "value": "2022-08-31"})

    def _base_url(self, vals):
        return self.getUrl().rstrip("/") + "/" + vals["prebuiltModelId"] + ":analyze"


# ---------------------------------------------------------------------- ontology
def _field_value(f: Dict[str, Any]):
    if not isinstance(f, dict):
        return f
    t = f.get("type") or f.get("valueType")
    for k in ("valueString", "valueNumber", "valueInteger", "valueDate", "valueTime", "valuePhoneNumber",
              "valueCountryRegion", "valueSelectionMark", "content", "text"):
        if k in f:
            return f[k]
    if t == "array" or "valueArray" in f:
        return [_field_value(x) for x in f.get("valueArray", [])]
    if t == "object" or "valueObject" in f:
        return {k: _field_value(v) for k, v in f.get("valueObject", {}).items()}
    return None


def _fields_of(resp) -> Dict[str, Any]:
    if not isinstance(resp, dict):
        return {}
    ar = resp.get("analyzeResult", resp)
    docs = ar.get("documents") or ar.get("documentResults") or []
    out: Dict[str, Any] = {}
    for d in docs:
        for k, v in (d.get("fields") or {}).items():
            out[k] = _field_value(v)
    return out


def _merge_schema(a, b):
    if isinstance(a, dict) and isinstance(b, dict):
        out = dict(a)
        for k, v in b.items():
            out[k] = _merge_schema(out.get(k), v)
        return out
    if isinstance(a, list) and isinstance(b, list):
        inner = None
        for x in a + b:
            inner = _merge_schema(inner, x)
        return [inner]
    return b if a is None else a if b is None else (type(a).__name__ if not isinstance(a, str) else a)


def _schema_of(v):
    if isinstance(v, dict):
        return {k: _schema_of(x) for k, x in v.items()}
    if isinstance(v, list):
        inner = None
        for x in v:
            inner = _merge_schema(inner, _schema_of(x))
        return [inner]
    if v is None:
        return None
    return "double" if isinstance(v, (int, float)) and not isinstance(v, bool) else "string"


def _conform(v, schema):
    if isinstance(schema, dict):
        v = v if isinstance(v, dict) else {}
        return {k: _conform(v.get(k), s) for k, s in schema.items()}
    if isinstance(schema, list):
        return None if v is None else [_conform(x, schema[0]) for x in v]
    if v is None:
        return None
    if schema == "double":
        try:
            return float(v)
        except (TypeError, ValueError):
            return None
    return str(v)


class FormOntologyTransformer(Model):
    inputCol = Param("The name of the input column", None, T.toString)
    outputCol = Param("The name of the output column", None, T.toString)
    ontology = Param("The ontology to cast values to", None, T.identity)

    def _transform(self, df):
        sch = self.getOntology()
        vals = [_conform(_fields_of(r), sch) for r in df[self.getInputCol()].tolist()]
        col = np.empty(len(vals), dtype=object)
        for i, v in enumerate(vals):
            col[i] = v
        return df.withColumn(self.getOutputCol(), col)


class FormOntologyLearner(Estimator):
    """Learns the union of the extracted fields' schema across analyze results; the model conforms every
    row's fields to it (missing fields null)."""

    inputCol = Param("The name of the input column", None, T.toString)
    outputCol = Param("The name of the output column", None, T.toString)

    def _fit(self, df):
        sch: Dict[str, Any] = {}
        for r in df[self.getInputCol()].tolist():
            sch = _merge_schema(sch, _schema_of(_fields_of(r)))
        return FormOntologyTransformer(inputCol=self.getInputCol(), outputCol=self.getOutputCol(), ontology=sch)


__all__ = ["AnalyzeLayout", "AnalyzeReceipts", "AnalyzeBusinessCards", "AnalyzeInvoices", "AnalyzeIDDocuments",
           "AnalyzeCustomModel", "GetCustomModel", "ListCustomModels", "AnalyzeDocument", "FormOntologyLearner",
           "FormOntologyTransformer"]
