"""Cognitive-service transformers against a local 127.0.0.1 mock service
(no network): request shape (URL, query, auth headers, entity), response
parsing, error column, skip-on-null, async polling, batching helpers
(reference tests: cognitive/src/test/scala/.../services/**; those call live
endpoints, so here the service side is mocked)."""
import json
from urllib.parse import parse_qs, urlparse

import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.io.serving import ServingServer, make_response
from synapseml_amd import services as S


def _obj(v):
    a = np.empty(len(v), dtype=object)
    for i, x in enumerate(v):
        a[i] = x
    return a


class Mock:
    """Records requests; ``routes`` maps a path suffix to fn(path, query, headers, body) -> response dict."""

    def __init__(self, routes):
        self.routes = routes
        self.log = []
        self.srv = ServingServer(self._fn, max_batch_size=1).start()

    @property
    def base(self):
        return f"http://127.0.0.1:{self.srv.port}"

    def _fn(self, df):
        reps = []
        for req in df["request"].tolist():
            u = urlparse(req["requestLine"]["uri"])
            hdr = {h["name"].lower(): h["value"] for h in req["headers"]}
            body = (req.get("entity") or {}).get("content")
            self.log.append((req["requestLine"]["method"], u.path, parse_qs(u.query), hdr, body))
            for suffix, fn in self.routes.items():
                if u.path.endswith(suffix):
                    reps.append(fn(u.path, parse_qs(u.query), hdr, body))
                    break
            else:
                reps.append(make_response({"error": "no route"}, 404, "Not Found"))
        return df.withColumn("reply", _obj(reps))

    def stop(self):
        self.srv.stop()


@pytest.fixture
def mock():
    m = []

    def make(routes):
        m.append(Mock(routes))
        return m[-1]

    yield make
    for x in m:
        x.stop()


def test_text_sentiment_request_and_unpack(mock):
    def sent(path, q, h, body):
        docs = json.loads(body)["documents"]
        return make_response({"documents": [{"id": d["id"], "sentiment": "positive" if "good" in d["text"] else
                                             "negative"} for d in docs], "errors": [], "modelVersion": "x"})

    m = mock({"/sentiment": sent})
    df = DataFrame({"text": _obj(["good day", "bad day", None]), "lang": _obj(["en", "en", "en"])})
    t = S.TextSentiment().setUrl(m.base + "/text/analytics/v3.1/sentiment").setSubscriptionKey("k123") \
        .setTextCol("text").setLanguageCol("lang").setOutputCol("out").setShowStats(True)
    out = t.transform(df)
    res = out["out"].tolist()
    assert res[0]["sentiment"] == "positive" and res[1]["sentiment"] == "negative"
    assert res[2] is None and out[t.getErrorCol()].tolist()[2] is None  # null text -> skipped
    meth, path, q, h, body = m.log[0]
    assert meth == "POST" and h["ocp-apim-subscription-key"] == "k123"
    assert q["showStats"] == ["true"]
    assert json.loads(body) == {"documents": [{"id": "0", "text": "good day", "language": "en"}]}
    assert len(m.log) == 2


def test_batched_text_list_and_doc_errors(mock):
    def kp(path, q, h, body):
        docs = json.loads(body)["documents"]
        return make_response({"documents": [{"id": d["id"], "keyPhrases": d["text"].split()} for d in docs
                                            if d["text"]],
                              "errors": [{"id": d["id"], "error": {"code": "EmptyText"}} for d in docs
                                         if not d["text"]]})

    m = mock({"/keyPhrases": kp})
    df = DataFrame({"t": _obj([["a b", "", "c"]])})
    out = S.KeyPhraseExtractor(url=m.base + "/keyPhrases", outputCol="o").setTextCol("t").transform(df)
    r = out["o"].tolist()[0]
    assert r[0]["keyPhrases"] == ["a", "b"] and r[1]["error"]["code"] == "EmptyText" and r[2]["keyPhrases"] == ["c"]


def test_auth_precedence_and_location():
    t = S.TextSentiment().setLocation("eastus")
    assert t.getUrl() == "https://eastus.api.cognitive.microsoft.com/text/analytics/v3.1/sentiment"
    assert S.TextSentiment().setLocation("usgovarizona").getUrl().startswith("https://usgovarizona.api.cognitive.microsoft.us/")
    assert S.TextSentiment().setEndpoint("https://x.cognitiveservices.azure.com/").getUrl() == \
        "https://x.cognitiveservices.azure.com/text/analytics/v3.1/sentiment"
    h = t._headers({"AADToken": "tok"}, "application/json")
    assert h["Authorization"] == "Bearer tok" and "x-ms-workload-resource-moniker" in h
    h = t._headers({"subscriptionKey": "k", "AADToken": "tok"}, None)
    assert h == {"Ocp-Apim-Subscription-Key": "k"}
    assert t._headers({"CustomAuthHeader": "Custom x"}, None)["Authorization"] == "Custom x"


def test_missing_required_and_dynamic_cols():
    with pytest.raises(ValueError, match="Missing required"):
        S.TextSentiment(url="http://127.0.0.1:1/").transform(DataFrame({"x": np.arange(2)}))
    with pytest.raises(ValueError, match="dynamic columns"):
        S.TextSentiment(url="http://127.0.0.1:1/").setTextCol("nope").transform(DataFrame({"x": np.arange(2)}))


def test_translate_query_and_region(mock):
    def tr(path, q, h, body):
        items = json.loads(body)
        return make_response([{"translations": [{"text": it["Text"].upper(), "to": t} for t in q["to"]]}
                              for it in items])

    m = mock({"/translate": tr})
    t = S.Translate(url=m.base + "/translate", outputCol="o").setSubscriptionKey("k").setSubscriptionRegion("eastus") \
        .setToLanguage(["de", "fr"]).setTextCol("s")
    out = t.transform(DataFrame({"s": _obj(["hi"])}))
    assert out["o"].tolist()[0][0]["translations"][1] == {"text": "HI", "to": "fr"}
    _, _, q, h, _ = m.log[0]
    assert q["api-version"] == ["3.0"] and q["to"] == ["de", "fr"]
    assert h["ocp-apim-subscription-region"] == "eastus"


def test_error_column_on_4xx(mock):
    m = mock({"/analyze": lambda p, q, h, b: make_response({"error": {"code": "InvalidImageUrl"}}, 400, "Bad")})
    t = S.AnalyzeImage(url=m.base + "/vision/v3.2/analyze", outputCol="o", errorCol="e").setImageUrlCol("u") \
        .setVisualFeatures(["Categories", "Tags"])
    out = t.transform(DataFrame({"u": _obj(["http://x/img.png"])}))
    assert out["o"].tolist()[0] is None
    assert out["e"].tolist()[0]["status"]["statusCode"] == 400
    _, _, q, _, body = m.log[0]
    assert q["visualFeatures"] == ["Categories,Tags"] and json.loads(body) == {"url": "http://x/img.png"}


def test_image_bytes_and_thumbnail_binary(mock):
    seen = {}

    def thumb(p, q, h, body):
        seen["ct"] = h["content-type"]
        seen["body"] = body
        return make_response(b"\x89PNGthumb")

    m = mock({"/generateThumbnail": thumb})
    t = S.GenerateThumbnails(url=m.base + "/generateThumbnail", outputCol="o").setImageBytesCol("b").setWidth(50) \
        .setHeight(40)
    out = t.transform(DataFrame({"b": _obj([b"rawimage"])}))
    assert out["o"].tolist()[0] == b"\x89PNGthumb"
    assert seen["ct"] == "application/octet-stream" and seen["body"] == b"rawimage"
    assert m.log[0][2] == {"width": ["50"], "height": ["40"]}


def test_async_polling(mock):
    state = {"polls": 0}

    def start(p, q, h, b):
        r = make_response("", 202, "Accepted")
        r["headers"].append({"name": "Operation-Location", "value": m.base + "/ops/1"})
        return r

    def poll(p, q, h, b):
        state["polls"] += 1
        assert h["ocp-apim-subscription-key"] == "k"
        if state["polls"] < 3:
            return make_response({"status": "running"})
        return make_response({"status": "succeeded", "analyzeResult": {"readResults": [{"lines": ["hello"]}]}})

    m = mock({"/read/analyze": start, "/ops/1": poll})
    t = S.ReadImage(url=m.base + "/vision/v3.2/read/analyze", outputCol="o", pollingDelay=1).setSubscriptionKey("k") \
        .setImageUrlCol("u")
    out = t.transform(DataFrame({"u": _obj(["http://x/a.png"])}))
    assert out["o"].tolist()[0]["status"] == "succeeded" and state["polls"] == 3


def test_openai_completion_chat_embedding_prompt(mock):
    def comp(p, q, h, b):
        body = json.loads(b)
        assert h["api-key"] == "sk"
        return make_response({"choices": [{"text": "a,b, c", "index": 0}], "echo": body})

    def chat(p, q, h, b):
        body = json.loads(b)
        return make_response({"choices": [{"message": {"role": "assistant",
                                                       "content": "{\"n\": %d}" % len(body["messages"])}}]})

    def emb(p, q, h, b):
        return make_response({"data": [{"embedding": [0.5, 1.5, 2.5]}]})

    m = mock({"/completions": lambda p, q, h, b: chat(p, q, h, b) if "/chat/" in p else comp(p, q, h, b),
              "/embeddings": emb})
    c = S.OpenAICompletion(url=m.base + "/", outputCol="o").setSubscriptionKey("sk").setDeploymentName("dep") \
        .setPromptCol("p").setMaxTokens(20).setTemperature(0.0).setLogProbs(2)
    out = c.transform(DataFrame({"p": _obj(["hello"])}))
    echo = out["o"].tolist()[0]["echo"]
    assert echo == {"max_tokens": 20, "temperature": 0.0, "logprobs": 2, "prompt": "hello"}
    meth, path, q, h, _ = m.log[0]
    assert path == "/openai/deployments/dep/completions" and q["api-version"] == ["2024-02-01"]

    ch = S.OpenAIChatCompletion(url=m.base, outputCol="o").setSubscriptionKey("sk").setDeploymentName("d") \
        .setMessagesCol("m")
    out = ch.transform(DataFrame({"m": _obj([[{"role": "system", "content": "x"}, {"role": "user", "content": "y"}]])}))
    assert out["o"].tolist()[0]["choices"][0]["message"]["content"] == '{"n": 2}'

    e = S.OpenAIEmbedding(url=m.base, outputCol="v").setSubscriptionKey("sk").setDeploymentName("e").setTextCol("t")
    v = e.transform(DataFrame({"t": _obj(["x"])}))["v"].tolist()[0]
    assert v.dtype == np.float32 and v.tolist() == [0.5, 1.5, 2.5]

    pr = S.OpenAIPrompt(promptTemplate="List {thing}", postProcessing="csv", outputCol="out")
    pr.set("completion", S.OpenAICompletion(url=m.base).setSubscriptionKey("sk").setDeploymentName("dep"))
    res = pr.transform(DataFrame({"thing": _obj(["letters"])}))
    assert res["out"].tolist()[0] == ["a", "b", " c"]
    assert "List letters" in json.dumps(m.log[-1][4].decode())
    prj = S.OpenAIPrompt(promptTemplate="{q}", postProcessing="json", outputCol="out")
    prj.set("completion", S.OpenAIChatCompletion(url=m.base).setSubscriptionKey("sk").setDeploymentName("d"))
    assert prj.transform(DataFrame({"q": _obj(["z"])}))["out"].tolist()[0] == {"n": 1}


def test_simple_detect_anomalies_groups_and_explodes(mock):
    def entire(p, q, h, b):
        s = json.loads(b)["series"]
        vals = [pt["value"] for pt in s]
        return make_response({"isAnomaly": [v > 50 for v in vals], "expectedValues": [1.0] * len(vals),
                              "upperMargins": [0.0] * len(vals), "lowerMargins": [0.0] * len(vals),
                              "isPositiveAnomaly": [v > 50 for v in vals], "isNegativeAnomaly": [False] * len(vals),
                              "period": 0})

    m = mock({"/entire/detect": entire})
    ts = [f"2024-01-{d:02d}T00:00:00Z" for d in range(1, 13)]
    rows_g = ["a"] * 12 + ["b"] * 12
    vals = [1.0] * 12 + [2.0] * 11 + [99.0]
    order = np.random.default_rng(0).permutation(24)
    df = DataFrame({"timestamp": _obj([(ts * 2)[i] for i in order]), "value": np.asarray(vals)[order],
                    "g": _obj([rows_g[i] for i in order])})
    t = S.SimpleDetectAnomalies(url=m.base + "/timeseries/entire/detect", outputCol="o", groupbyCol="g") \
        .setSubscriptionKey("k").setGranularity("daily")
    out = t.transform(df)
    flags = [r["isAnomaly"] for r in out["o"].tolist()]
    assert sum(flags) == 1 and out["value"][flags.index(True)] == 99.0
    assert len(m.log) == 2 and json.loads(m.log[0][4])["granularity"] == "daily"


def test_form_ontology_learner():
    r1 = {"analyzeResult": {"documents": [{"fields": {"Total": {"type": "number", "valueNumber": 10.5},
                                                     "Vendor": {"type": "string", "valueString": "A"}}}]}}
    r2 = {"analyzeResult": {"documents": [{"fields": {"Total": {"type": "number", "valueNumber": 3},
                                                     "Items": {"type": "array", "valueArray": [
                                                         {"type": "object", "valueObject": {
                                                             "Name": {"type": "string", "valueString": "x"}}}]}}}]}}
    df = DataFrame({"res": _obj([r1, r2])})
    model = S.FormOntologyLearner(inputCol="res", outputCol="ont").fit(df)
    out = model.transform(df)["ont"].tolist()
    assert out[0] == {"Total": 10.5, "Vendor": "A", "Items": None}
    assert out[1]["Items"] == [{"Name": "x"}] and out[1]["Vendor"] is None


def test_text_to_speech_and_maps(mock):
    m = mock({"/cognitiveservices/v1": lambda p, q, h, b: make_response(b"RIFFaudio"),
              "/batch/json": lambda p, q, h, b: make_response({"batchItems": [{"q": i["query"]} for i in
                                                                               json.loads(b)["batchItems"]]})})
    t = S.TextToSpeech(url=m.base + "/cognitiveservices/v1", outputCol="o").setSubscriptionKey("k").setTextCol("t")
    out = t.transform(DataFrame({"t": _obj(["hi & bye"])}))
    assert out["o"].tolist()[0] == b"RIFFaudio"
    _, _, _, h, body = m.log[0]
    assert h["content-type"] == "application/ssml+xml" and b"hi &amp; bye" in body
    g = S.AddressGeocoder(url=m.base + "/search/address/batch/json", outputCol="o").setSubscriptionKey("mk") \
        .setAddressCol("a")
    res = g.transform(DataFrame({"a": _obj([["1 Main St", "2 Side Rd"]])}))["o"].tolist()[0]
    assert [r["q"] for r in res] == ["?query=1 Main St&limit=1", "?query=2 Side Rd&limit=1"]
    assert m.log[1][2]["subscription-key"] == ["mk"] and m.log[1][2]["api-version"] == ["1.0"]


def test_bing_search_get_and_url_explode(mock):
    m = mock({"/images/search": lambda p, q, h, b: make_response(
        {"value": [{"contentUrl": f"http://img/{q['q'][0]}/{i}"} for i in range(int(q['count'][0]))]})})
    t = S.BingImageSearch(url=m.base + "/v7.0/images/search", outputCol="images").setSubscriptionKey("k") \
        .setQCol("q").setCount(2)
    out = t.transform(DataFrame({"q": _obj(["cats", "dogs"])}))
    assert m.log[0][0] == "GET" and m.log[0][4] is None
    urls = S.BingImageSearch.getUrlTransformer("images", "url").transform(out)
    assert urls["url"].tolist() == ["http://img/cats/0", "http://img/cats/1", "http://img/dogs/0", "http://img/dogs/1"]


def test_service_param_persistence_roundtrip(tmp_path):
    t = S.TextSentiment(url="http://x/").setSubscriptionKey("k").setTextCol("text").setLanguage("en")
    t.save(str(tmp_path / "ts"))
    from synapseml_amd.core.serialize import load_stage

    t2 = load_stage(str(tmp_path / "ts"))
    assert t2.getTextCol() == "text" and t2.getLanguage() == "en" and t2.getSubscriptionKey() == "k"


class _FakeChain:
    """Stands in for a langchain LLMChain (langchain is not installed): uppercases the prompt,
    fails on 'boom', and records the OpenAI environment it saw."""

    def __init__(self):
        self.seen_env = None

    def run(self, x):
        import os

        self.seen_env = os.environ.get("OPENAI_API_KEY")
        if x == "boom":
            raise RuntimeError("rate limited")
        return {"text": x.upper()}


class _Runnable:
    def invoke(self, x):
        class Msg:
            content = f"<{x}>"

        return Msg()


def test_langchain_transformer_rows_errors_env_and_persistence(tmp_path):
    import os

    chain = _FakeChain()
    t = S.LangchainTransformer(inputCol="q", outputCol="a", chain=chain, subscriptionKey="k123", concurrency=4)
    df = DataFrame({"q": _obj(["hi", "boom", "there"])})
    out = t.transform(df)
    assert out["a"].tolist() == ["HI", None, "THERE"]
    assert out["errorCol"][0] is None and "rate limited" in out["errorCol"][1]
    assert chain.seen_env == "k123" and os.environ.get("OPENAI_API_KEY") != "k123"  # restored afterwards
    r = S.LangchainTransformer(inputCol="q", outputCol="a", chain=_Runnable()).transform(df)
    assert r["a"].tolist() == ["<hi>", "<boom>", "<there>"]
    t.save(str(tmp_path / "lc"))
    back = S.LangchainTransformer.load(str(tmp_path / "lc"))
    assert back.transform(df)["a"].tolist() == ["HI", None, "THERE"]
    with pytest.raises(ValueError):
        S.LangchainTransformer(inputCol="q", outputCol="a").transform(df)


def test_text_analyze_tasks_and_unpack(mock):
    def start(p, q, h, b):
        body = json.loads(b)
        assert body["tasks"]["entityRecognitionTasks"] == [{"parameters": {"model-version": "latest"}}]
        assert body["tasks"]["keyPhraseExtractionTasks"] == []
        state["docs"] = body["analysisInput"]["documents"]
        r = make_response("", 202, "Accepted")
        r["headers"].append({"name": "Operation-Location", "value": m.base + "/analyze/jobs/7?x=1"})
        return r

    def poll(p, q, h, b):
        assert q["$top"] == ["25"] and q["x"] == ["1"]
        res = lambda tag: [{"results": {"documents": [{"id": d["id"], "tag": tag} for d in state["docs"]],
                                        "errors": []}}]
        return make_response({"status": "succeeded", "tasks": {
            "entityRecognitionTasks": res("ner"), "entityLinkingTasks": res("link"),
            "entityRecognitionPiiTasks": res("pii"), "keyPhraseExtractionTasks": [],
            "sentimentAnalysisTasks": res("sent")}})

    state = {}
    m = mock({"/analyze": start, "/analyze/jobs/7": poll})
    t = S.TextAnalyze(url=m.base + "/text/analytics/v3.1/analyze", outputCol="o", pollingDelay=1) \
        .setSubscriptionKey("k").setTextCol("t").setIncludeKeyPhraseExtraction(False)
    out = t.transform(DataFrame({"t": _obj([["a", "b"], "c"])}))["o"].tolist()
    assert [d["entityRecognition"]["tag"] for d in out[0]] == ["ner", "ner"]
    assert out[0][1]["pii"]["id"] == "1" and out[0][0]["keyPhraseExtraction"] is None
    assert out[1]["sentimentAnalysis"]["tag"] == "sent"


def test_multivariate_fit_detect_and_last(mock, tmp_path):
    ts = [f"2021-01-01T00:0{i}:00Z" for i in range(6)]
    df = DataFrame({"timestamp": _obj(ts[::-1]), "a": np.arange(6.0)[::-1].copy(), "b": np.ones(6)})
    seen = {}

    def train(p, q, h, b):
        body = json.loads(b)
        seen["train"] = body
        r = make_response("", 201, "Created")
        r["headers"].append({"name": "Location", "value": m.base + "/multivariate/models/m1"})
        return r

    def model(p, q, h, b):
        seen["polls"] = seen.get("polls", 0) + 1
        st = "RUNNING" if seen["polls"] < 2 else "READY"
        return make_response({"modelId": "m1", "modelInfo": {"status": st, "diagnosticsInfo": {"x": 1}}})

    def batch(p, q, h, b):
        seen["batch"] = json.loads(b)
        r = make_response("", 202, "Accepted")
        return make_response({"resultId": "r9", "summary": {"status": "CREATED"}}, 202, "Accepted")

    def result(p, q, h, b):
        return make_response({"summary": {"status": "READY"}, "results": [
            {"timestamp": t, "value": {"isAnomaly": i == 3, "severity": 0.5 * (i == 3)}} for i, t in enumerate(ts)]})

    def last(p, q, h, b):
        body = json.loads(b)
        seen.setdefault("last", []).append(body)
        tl = body["variables"][0]["timestamps"][-1]
        return make_response({"results": [{"timestamp": tl, "value": {"isAnomaly": tl.endswith("05:00Z")}}]})

    m = mock({"/models": train, "/models/m1": model, "/m1:detect-batch": batch, "/detect-batch/r9": result,
              "/m1:detect-last": last})
    est = S.SimpleFitMultivariateAnomaly(url=m.base + "/multivariate/models", pollingDelay=1, inputCols=["a", "b"],
                                         intermediateSaveDir=str(tmp_path), startTime="2021-01-01T00:00:00Z",
                                         endTime="2021-01-01T00:05:00Z").setSubscriptionKey("k")
    model_ = est.fit(df)
    assert seen["train"]["dataSchema"] == "OneTable" and seen["train"]["slidingWindow"] == 300
    assert seen["train"]["alignPolicy"] == {"alignMode": "Outer", "fillNAMethod": "Linear"}
    csv = open(seen["train"]["dataSource"]).read().splitlines()
    assert csv[0] == "timestamp,a,b" and csv[1].startswith("2021-01-01T00:00:00Z,0.0")  # sorted by time
    assert model_.getModelId() == "m1" and model_.getDiagnosticsInfo() == {"x": 1}
    out = model_.transform(df)
    assert out["timestamp"].tolist() == ts and out["isAnomaly"].tolist() == [i == 3 for i in range(6)]
    assert seen["batch"]["topContributorCount"] == 10
    dl = S.DetectLastMultivariateAnomaly(url=m.base + "/multivariate/models", modelId="m1", batchSize=2,
                                         inputVariablesCols=["a", "b"], outputCol="o").setSubscriptionKey("k")
    o2 = dl.transform(df)
    assert o2["isAnomaly"].tolist() == [False] * 5 + [True]
    assert [len(x["variables"][0]["values"]) for x in seen["last"]] == [1, 2, 3, 3, 3, 3]


def test_speech_sdk_chunks_long_wav_and_conversation(mock):
    import io
    import wave

    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(1000)
        w.writeframes(b"\x00\x01" * 2500)  # 2.5 s
    calls = []

    def rec(p, q, h, b):
        calls.append((h["content-type"], len(b)))
        return make_response({"RecognitionStatus": "Success", "DisplayText": f"part{len(calls)}", "Offset": 5,
                              "Duration": 10})

    m = mock({"/cognitiveservices/v1": rec})
    df = DataFrame({"audio": _obj([buf.getvalue()])})
    t = S.SpeechToTextSDK(url=m.base + "/speech/recognition/conversation/cognitiveservices/v1", outputCol="o",
                          chunkSeconds=1.0).setSubscriptionKey("k").setAudioDataCol("audio").setLanguage("en-US")
    out = t.transform(df)
    assert len(calls) == 3 and calls[0][0].startswith("audio/wav")
    assert out["o"].tolist()[1]["Offset"] == 5 + 10_000_000 and out.count() == 3
    t2 = S.ConversationTranscription(url=t.getUrl(), outputCol="o", chunkSeconds=2.0, streamIntermediateResults=False) \
        .setSubscriptionKey("k").setAudioDataCol("audio").setParticipantsJson('[{"name": "a"}]')
    res = t2.transform(df)["o"].tolist()[0]
    assert [r["SpeakerId"] for r in res] == ["Unidentified"] * 2
    with pytest.raises(ValueError):
        S.SpeechToTextSDK(url=t.getUrl()).setSubscriptionKey("k").setAudioDataCol("audio").setFileType("mp3") \
            .transform(df)
