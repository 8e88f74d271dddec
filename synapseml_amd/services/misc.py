"""Speech (REST), Bing image search, Azure AI Search writer and Azure Maps
transformers (reference: cognitive/.../services/speech/{SpeechToText,
TextToSpeech, SpeakerEmotionInference}.scala, bing/BingImageSearch.scala,
search/AzureSearch.scala, geospatial/{Geocoders,CheckPointInPolygon}.scala)."""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional
from xml.sax.saxutils import escape

import numpy as np

from ..core.dataframe import DataFrame
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Transformer
from ..io.http import error_of
from .base import CognitiveServicesBase, HasAPIVersion, HasAsyncReply, ServiceParam, _obj


# ---------------------------------------------------------------------- speech
class SpeechToText(CognitiveServicesBase):
    """Short-audio REST recognition: POST WAV/OGG bytes, query language / format / profanity."""

    url_path = "/speech/recognition/conversation/cognitiveservices/v1"
    host_template = "https://{location}.stt.speech.microsoft.{domain}/"
    audioData = ServiceParam("The data sent to the service must be a .wav files", required=True)
    language = ServiceParam("Identifies the spoken language that is being recognized.", url_param=True)
    format = ServiceParam("Specifies the result format. Accepted values are simple and detailed.",
                          url_param=True)
    profanity = ServiceParam("Specifies how to handle profanity in recognition results.", url_param=True)

    def _entity(self, vals):
        return bytes(vals["audioData"]), "audio/wav; codecs=audio/pcm; samplerate=16000"


def wav_chunks(data: bytes, max_seconds: float) -> List[tuple]:
    """Split a PCM WAV file into (offset_seconds, wav_bytes) pieces of at most ``max_seconds`` (the reference
    streams a WavStream into the SDK; the short-audio REST endpoint takes <= 60 s per request)."""
    import io
    import wave

    with wave.open(io.BytesIO(bytes(data)), "rb") as w:
        params = w.getparams()
        rate = w.getframerate()
        frames = w.readframes(w.getnframes())
    step = max(1, int(max_seconds * rate))
    fbytes = params.sampwidth * params.nchannels
    out = []
    for f0 in range(0, max(1, len(frames) // fbytes), step):
        buf = io.BytesIO()
        with wave.open(buf, "wb") as o:
            o.setparams(params)
            o.writeframes(frames[f0 * fbytes:(f0 + step) * fbytes])
        out.append((f0 / rate, buf.getvalue()))
    return out


_AUDIO_TYPES = {"wav": "audio/wav; codecs=audio/pcm; samplerate=16000", "ogg": "audio/ogg; codecs=opus"}


class SpeechToTextSDK(SpeechToText):
    """Continuous recognition of arbitrarily long audio (reference: SpeechToTextSDK.scala:44-510). The
    reference streams the audio through the native Speech SDK; that SDK does not exist for this platform,
    so WAV audio is cut into pieces the short-audio REST endpoint accepts (``chunkSeconds``) and each
    piece is recognised in turn: the output is the list of per-piece results (``Offset`` shifted to the
    position in the whole file, in 100-ns ticks as the SDK reports it), or, with
    ``streamIntermediateResults``, one output row per result (the reference's flatMap of the stream).
    OGG/OPUS is sent whole; other compressed formats (the SDK's CompressedStream: mp3, flac, ...) need a
    decoder and are rejected with a clear error."""

    fileType = ServiceParam("The file type of the sound files, supported types: wav, ogg, mp3", default="wav")
    streamIntermediateResults = Param("Whether or not to immediately return itermediate results, or group in "
                                      "a sequence", True, T.toBoolean)
    wordLevelTimestamps = ServiceParam("Whether to request timestamps foe each indivdual word", default=False)
    endpointId = ServiceParam("endpoint for custom speech models", url_param=True, payload_name="cid")
    chunkSeconds = Param("longest audio piece sent in one request (the REST limit is 60 s)", 55.0, T.toFloat)

    def _query(self, vals):
        q = super()._query(vals)
        if vals.get("wordLevelTimestamps"):
            q.append(("wordLevelTimestamps", "true"))
        return q

    def _pieces(self, vals) -> List[tuple]:
        ftype = str(vals.get("fileType", "wav")).lower()
        if ftype not in _AUDIO_TYPES:
            raise ValueError(f"{type(self).__name__}: fileType {ftype!r} needs an audio decoder that is not "
                             f"available; supported: {sorted(_AUDIO_TYPES)}")
        data = bytes(vals["audioData"])
        return wav_chunks(data, self.getChunkSeconds()) if ftype == "wav" else [(0.0, data)]

    def _transform(self, df):
        import requests

        reqs, allvals = self._requests_for(df)
        session = requests.Session()
        results, errs = [], []
        for req, vals in zip(reqs, allvals):
            if req is None:
                results.append(None)
                errs.append(None)
                continue
            method, url, headers, _ = req
            pieces = self._pieces(vals)
            h = dict(headers, **{"Content-Type": _AUDIO_TYPES[str(vals.get("fileType", "wav")).lower()]})
            row_res, row_err = [], None
            for off, piece in pieces:
                resp = self._send(session, (method, url, h, piece))
                err = error_of(resp)
                if err is not None:
                    row_err = err
                    break
                r = self._parse(resp)
                if isinstance(r, dict):
                    r = self._decorate(dict(r), vals)
                    if "Offset" in r:
                        r["Offset"] = int(r["Offset"]) + int(round(off * 1e7))
                row_res.append(r)
            results.append(row_res if row_err is None else None)
            errs.append(row_err)
        if not self.getStreamIntermediateResults():
            return df.withColumn(self.getOutputCol(), _obj(results)).withColumn(self.getErrorCol(), _obj(errs))
        idx, outs, oerr = [], [], []
        for i, (rs, e) in enumerate(zip(results, errs)):
            for r in (rs or [None]):
                idx.append(i)
                outs.append(r)
                oerr.append(e)
        out = df._take_rows(np.asarray(idx, dtype=np.int64))
        return out.withColumn(self.getOutputCol(), _obj(outs)).withColumn(self.getErrorCol(), _obj(oerr))

    def _decorate(self, r: dict, vals) -> dict:
        return r


class ConversationTranscription(SpeechToTextSDK):
    """Multi-speaker transcription (reference: SpeechToTextSDK.scala:511-600, ConversationTranscriber). The
    REST endpoint does not separate speakers, so every result carries ``SpeakerId = "Unidentified"`` (the
    value the SDK itself reports for voices it cannot match); ``participantsJson`` is validated and kept
    for API parity."""

    participantsJson = ServiceParam("a json representation of a list of conversation participants (email, "
                                    "language, user)")

    def _decorate(self, r: dict, vals) -> dict:
        if vals.get("participantsJson"):
            json.loads(vals["participantsJson"])  # malformed participant lists fail like the SDK call would
        r.setdefault("SpeakerId", "Unidentified")
        r.setdefault("Type", "ConversationTranscription")
        return r


class TextToSpeech(CognitiveServicesBase):
    """SSML synthesis; the output column holds the audio bytes."""

    url_path = "/cognitiveservices/v1"
    host_template = "https://{location}.tts.speech.microsoft.{domain}/"
    text = ServiceParam("The text to synthesize", required=True)
    language = ServiceParam("The name of the language used for synthesis", default="en-US")
    voiceName = ServiceParam("The name of the voice used for synthesis", default="en-US-JennyNeural")
    outputFormat = ServiceParam("The format for the output audio", default="riff-24khz-16bit-mono-pcm")
    useSSML = ServiceParam("whether to interpret the provided text input as SSML", default=False)

    def _headers(self, vals, content_type):
        h = super()._headers(vals, content_type)
        h["X-Microsoft-OutputFormat"] = vals.get("outputFormat", "riff-24khz-16bit-mono-pcm")
        h["User-Agent"] = "synapseml-amd"
        return h

    def _entity(self, vals):
        if vals.get("useSSML"):
            ssml = vals["text"]
        else:
            ssml = (f"<speak version='1.0' xml:lang='{vals.get('language', 'en-US')}'>"
                    f"<voice name='{vals.get('voiceName', 'en-US-JennyNeural')}'>{escape(vals['text'])}</voice></speak>")
        return ssml.encode("utf-8"), "application/ssml+xml"

    def _parse(self, resp):
        return resp["entity"]["content"] if resp.get("entity") else None


class SpeakerEmotionInference(CognitiveServicesBase):
    """Annotates quoted speech in a passage with speaker/emotion SSML (reference: SpeakerEmotionInference.scala)."""

    url_path = "/cognitiveservices/v1"
    host_template = "https://{location}.customvoice.api.speech.microsoft.{domain}/api/texttospeech/v3.0-beta1/" \
                    "voicegeneration/"
    text = ServiceParam("The text to annotate with inferred emotion", required=True)
    locale = ServiceParam("The locale of the input text", default="en-US")
    voiceName = ServiceParam("The name of the voice used for synthesis", default="en-US-JennyNeural")

    def _entity(self, vals):
        return json.dumps({"text": vals["text"], "locale": vals.get("locale", "en-US"),
                           "voices": {"male": vals.get("voiceName"), "female": vals.get("voiceName"),
                                      "narrator": vals.get("voiceName")}}).encode("utf-8"), "application/json"


# ---------------------------------------------------------------------- Bing
class BingImageSearch(CognitiveServicesBase):
    url_path = "/v7.0/images/search"
    method = "GET"
    host_template = "https://api.bing.microsoft.com/"
    q = ServiceParam("The user's search query string", required=True, url_param=True)
    count = ServiceParam("The number of image results to return in the response.", url_param=True)
    offset = ServiceParam("The zero-based offset that indicates the number of image results to skip",
                          url_param=True)
    mkt = ServiceParam("The market where the results come from.", url_param=True)
    imageType = ServiceParam("Filter images by the following image types", url_param=True)
    aspect = ServiceParam("Filter images by the following aspect ratios", url_param=True)
    color = ServiceParam("Filter images by the following color options", url_param=True)
    freshness = ServiceParam("Filter images by the following discovery options", url_param=True)
    height = ServiceParam("Filter images that have the specified height, in pixels", url_param=True)
    width = ServiceParam("Filter images that have the specified width, in pixels", url_param=True)
    license = ServiceParam("Filter images by the following license types", url_param=True)
    safeSearch = ServiceParam("Filter images for adult content", url_param=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(url="https://api.bing.microsoft.com/v7.0/images/search")

    # reference BingImageSearch.py aliases of the q / mkt service params
    def setQuery(self, value):  # noqa: N802
        return self.setQ(value)

    def setQueryCol(self, value):  # noqa: N802
        return self.setQCol(value)

    def setMarket(self, value):  # noqa: N802
        return self.setMkt(value)

    def setMarketCol(self, value):  # noqa: N802
        return self.setMktCol(value)

    @staticmethod
    def getUrlTransformer(imageCol: str, urlCol: str) -> Transformer:  # noqa: N802,N803
        """Explode the search responses' ``value[].contentUrl`` into one row per image URL."""
        def fn(df):
            rows = []
            for r in df.collect():
                for img in ((r.get(imageCol) or {}).get("value") or []):
                    d = dict(r)
                    d[urlCol] = img.get("contentUrl")
                    rows.append(d)
            return DataFrame.fromRows(rows) if rows else DataFrame({urlCol: np.empty(0, dtype=object)})

        return _Fn(fn)

    @staticmethod
    def downloadFromUrls(pathCol: str, bytesCol: str, concurrency: int, timeout: int) -> Transformer:  # noqa: N802
        """Fetch each URL's bytes (failures -> null), like the reference's download pipeline."""

        def fn(df):
            import requests
            from concurrent.futures import ThreadPoolExecutor

            def get(u):
                try:
                    r = requests.get(u, timeout=timeout)
                    return r.content if r.status_code == 200 else None
                except Exception:  # noqa: BLE001 - unreachable urls become nulls
                    return None

            urls = df[pathCol].tolist()
            with ThreadPoolExecutor(max_workers=max(1, concurrency)) as ex:
                blobs = list(ex.map(get, urls))
            col = np.empty(len(blobs), dtype=object)
            for i, b in enumerate(blobs):
                col[i] = b
            return df.withColumn(bytesCol, col)

        return _Fn(fn)


class _Fn(Transformer):
    def __init__(self, fn=None, **kw):
        super().__init__(**kw)
        self._fn = fn

    def _transform(self, df):
        return self._fn(df)


# ---------------------------------------------------------------------- Azure AI Search
class AzureSearchWriter:
    """Create (if missing) an index and upload rows as documents in batches (reference: AzureSearch.scala).

    ``options``: subscriptionKey, serviceName or url, indexName, indexJson (optional: created when the index
    does not exist), actionCol (default "@search.action", default action "upload"), batchSize (100),
    apiVersion ("2019-05-06")."""

    @staticmethod
    def write(df: DataFrame, options: Dict[str, Any]) -> List[dict]:
        import requests

        key = options["subscriptionKey"]
        base = options.get("url") or f"https://{options['serviceName']}.search.windows.net"
        ver = options.get("apiVersion", "2019-05-06")
        index = options.get("indexName") or json.loads(options["indexJson"])["name"]
        hdr = {"api-key": key, "Content-Type": "application/json"}
        s = requests.Session()
        if options.get("indexJson"):
            r = s.get(f"{base}/indexes/{index}?api-version={ver}", headers=hdr, timeout=60)
            if r.status_code == 404:
                r = s.post(f"{base}/indexes?api-version={ver}", headers=hdr, data=options["indexJson"], timeout=60)
                if r.status_code not in (200, 201):
                    raise RuntimeError(f"index creation failed: {r.status_code} {r.text}")
        action_col = options.get("actionCol", "@search.action")
        bs = int(options.get("batchSize", 100))
        rows = df.collect()
        results = []
        for i in range(0, len(rows), bs):
            docs = []
            for r in rows[i:i + bs]:
                d = {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in dict(r).items()}
                d["@search.action"] = d.pop(action_col, None) or "upload"
                docs.append(d)
            r = s.post(f"{base}/indexes/{index}/docs/index?api-version={ver}", headers=hdr,
                       data=json.dumps({"value": docs}, default=str), timeout=60)
            if r.status_code not in (200, 201, 207):
                raise RuntimeError(f"document upload failed: {r.status_code} {r.text}")
            results.append(r.json())
        return results


class AddDocuments(CognitiveServicesBase):
    """Row-wise batch upload transformer used by the writer (body: {"value": [docs]})."""

    method = "POST"
    subscription_key_header = "api-key"
    actionCol = Param("You can combine actions, such as an upload and a delete, in the same batch", "@search.action",
                      T.toString)
    serviceName = Param("The name of the search service", None, T.toString)
    indexName = Param("The name of the index", None, T.toString)
    documents = ServiceParam("list of documents to index", required=True)

    def _base_url(self, vals):
        return self.getUrl() or (f"https://{self.getServiceName()}.search.windows.net/indexes/"
                                 f"{self.getIndexName()}/docs/index?api-version=2019-05-06")

    def _entity(self, vals):
        docs = []
        for d in vals["documents"]:
            d = dict(d)
            d["@search.action"] = d.pop(self.getActionCol(), None) or "upload"
            docs.append(d)
        return json.dumps({"value": docs}, default=str).encode("utf-8"), "application/json"


# ---------------------------------------------------------------------- Azure Maps
class _MapsBase(CognitiveServicesBase, HasAsyncReply):
    subscription_key_header = "subscription-key"

    def _query(self, vals):
        q = [("api-version", "1.0")]
        if vals.get("subscriptionKey"):
            q.append(("subscription-key", vals["subscriptionKey"]))
        return q + super()._query(vals)

    def _headers(self, vals, content_type):
        return {"Content-Type": content_type} if content_type else {}

    def _postprocess(self, parsed, vals):
        return parsed.get("batchItems", parsed) if isinstance(parsed, dict) else parsed


class AddressGeocoder(_MapsBase):
    address = ServiceParam("the address to geocode (string or list of strings)", required=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(url="https://atlas.microsoft.com/search/address/batch/json")

    def _entity(self, vals):
        a = vals["address"]
        items = [a] if isinstance(a, str) else list(a)
        body = {"batchItems": [{"query": "?query=" + x + "&limit=1"} for x in items]}
        return json.dumps(body).encode("utf-8"), "application/json"


class ReverseAddressGeocoder(_MapsBase):
    latitude = ServiceParam("the latitude(s) of the location", required=True)
    longitude = ServiceParam("the longitude(s) of the location", required=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(url="https://atlas.microsoft.com/search/address/reverse/batch/json")

    def _entity(self, vals):
        lat, lon = vals["latitude"], vals["longitude"]
        lats = [lat] if not isinstance(lat, (list, tuple, np.ndarray)) else list(lat)
        lons = [lon] if not isinstance(lon, (list, tuple, np.ndarray)) else list(lon)
        body = {"batchItems": [{"query": f"?query={a},{b}&limit=1"} for a, b in zip(lats, lons)]}
        return json.dumps(body).encode("utf-8"), "application/json"


class CheckPointInPolygon(_MapsBase):
    method = "GET"
    url_path = "spatial/pointInPolygon/json"
    host_template = "https://{location}.atlas.microsoft.com/"
    userDataIdentifier = ServiceParam("the identifier for the user uploaded data", required=True,
                                      url_param=True, payload_name="udid")
    latitude = ServiceParam("the latitude of the point", required=True, url_param=True, payload_name="lat")
    longitude = ServiceParam("the longitude of the point", required=True, url_param=True, payload_name="lon")

    def _postprocess(self, parsed, vals):
        return parsed


__all__ = ["SpeechToText", "SpeechToTextSDK", "ConversationTranscription", "wav_chunks", "TextToSpeech", "SpeakerEmotionInference", "BingImageSearch",
           "AzureSearchWriter", "AddDocuments", "AddressGeocoder", "ReverseAddressGeocoder", "CheckPointInPolygon"]
