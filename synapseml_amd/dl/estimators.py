"""DeepVisionClassifier / DeepTextClassifier (reference: deep-learning/.../dl/
{DeepVisionClassifier, DeepVisionModel, DeepTextClassifier, DeepTextModel,
LitDeepTextModel, PredictionParams}.py).

Params keep the reference's snake_case keyword names (``num_classes``,
``additional_layers_to_train``, ``batch_size`` ...) with CamelCase
``setX``/``getX`` accessors. Images may be file paths (the reference's
input), image rows, encoded bytes or HWC arrays; they are decoded, resized
and normalised by the image stack (the fused K19 kernel on the GPU). Text
uses the checkpoint's architecture (BERT/RoBERTa/DistilBERT family via
``transformers`` config classes) random-initialised — no weights can be
downloaded — with a deterministic hashing word-piece tokenizer unless a local
tokenizer directory is given."""
from __future__ import annotations

import re
import zlib
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ..core.dataframe import DataFrame
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Estimator, Model
from . import backbones
from .trainer import TrainConfig, fit, predict


def _camel(name: str) -> str:
    parts = name.split("_")
    return "".join(p[:1].upper() + p[1:] for p in parts)


class _SnakeParams(Params):
    """CamelCase accessors for snake_case params (setNumClasses -> num_classes)."""

    @classmethod
    def _params_hook(cls):
        for name in cls._params_decl:
            if "_" not in name:
                continue
            c = _camel(name)
            if not hasattr(cls, "set" + c):
                setattr(cls, "set" + c, (lambda n: lambda self, v: self.set(n, v))(name))
            if not hasattr(cls, "get" + c):
                setattr(cls, "get" + c, (lambda n: lambda self: self.getOrDefault(n))(name))


class _TrainParams(_SnakeParams):
    batch_size = Param("number of samples per step (per process)", 16, T.toInt)
    epochs = Param("number of epochs", 1, T.toInt)
    learning_rate = Param("learning rate", 1e-3, T.toFloat)
    optimizer_name = Param("optimizer: adam, adamw, sgd, rmsprop", "adam", T.toString)
    loss_name = Param("loss: cross_entropy, nll, mse", "cross_entropy", T.toString)
    weight_decay = Param("weight decay", 0.0, T.toFloat)
    random_seed = Param("seed", 0, T.toInt)
    use_gpu = Param("train on the GPU when one is visible", True, T.toBoolean)
    label_col = Param("label column name.", "label", T.toString)
    prediction_col = Param("prediction column name.", "prediction", T.toString)
    num_classes = Param("number of target classes", None, T.toInt)
    num_proc = Param("number of training processes (one per GPU); >1 runs torch.distributed data parallel over "
                     "the partition runtime", 1, T.toInt)

    def _cfg(self) -> TrainConfig:
        return TrainConfig(epochs=self.getOrDefault("epochs"), batch_size=self.getOrDefault("batch_size"),
                           learning_rate=self.getOrDefault("learning_rate"),
                           optimizer=self.getOrDefault("optimizer_name"), loss=self.getOrDefault("loss_name"),
                           weight_decay=self.getOrDefault("weight_decay"), seed=self.getOrDefault("random_seed"),
                           use_gpu=self.getOrDefault("use_gpu"))

    def _labels(self, df) -> torch.Tensor:
        y = np.asarray(df[self.getOrDefault("label_col")], dtype=np.float64)
        return torch.as_tensor(y.astype(np.int64))


# ---------------------------------------------------------------------- vision
_MEAN = [0.485, 0.456, 0.406]
_STD = [0.229, 0.224, 0.225]


def images_to_tensor(values: List[Any], size: int, use_gpu: bool, transform_fn=None) -> torch.Tensor:
    """Decode + resize(size) + centre crop + RGB + ImageNet normalise -> [N,3,size,size] float32; then
    ``transform_fn`` (the reference's transform_fn: a torchvision-style callable) on every [3,size,size] image."""
    t = _images_to_tensor(values, size, use_gpu)
    if transform_fn is not None:
        t = torch.stack([torch.as_tensor(transform_fn(img)) for img in t]).to(t.device).float()
    return t


def _images_to_tensor(values: List[Any], size: int, use_gpu: bool) -> torch.Tensor:
    from ..image.schema import to_array
    from ..image.transformer import ImageTransformer

    arrays = []
    for v in values:
        if isinstance(v, str):
            with open(v, "rb") as fh:
                v = fh.read()
        a = to_array(v)
        if a is None:
            raise ValueError("could not decode an input image")
        arrays.append(a)
    it = ImageTransformer(inputCol="image", outputCol="t").resize(height=size, width=size) \
        .normalize(_MEAN, _STD, 1.0 / 255).setTensorChannelOrder("RGB")
    if use_gpu and torch.cuda.is_available():
        t = it.device_tensors(arrays)
        if t is not None:
            return t.float()
    return torch.as_tensor(np.stack([it.process_host(a) for a in arrays]).astype(np.float32))


class _VisionParams(_TrainParams):
    backbone = Param("backbone of the deep vision classifier (resnet18/34/50/101/152, resnext50_32x4d, "
                     "resnext101_32x8d, wide_resnet50_2, resnet_tiny)", "resnet50", T.toString)
    additional_layers_to_train = Param("number of last layers to fine tune for the model, should be between 0 "
                                       "and 3", 0, T.toInt)
    dropout_aux = Param("numeric value that's applied to googlenet InceptionAux module's dropout layer only",
                        0.7, T.toFloat)
    image_col = Param("image column name.", "image", T.toString)
    image_size = Param("square input size fed to the backbone", 224, T.toInt)
    weights = Param("optional local state dict / safetensors of backbone weights", None, T.toString)
    transform_fn = Param("callable applied to every decoded, normalised [3, H, W] image tensor (training and "
                         "inference), e.g. a torchvision.transforms.Compose", None, complex=True)

    def setDropoutAUX(self, value):  # noqa: N802  (reference spelling)
        return self.set("dropout_aux", float(value))

    def getDropoutAUX(self):  # noqa: N802
        return self.getOrDefault("dropout_aux")

    def _images(self, df):
        return images_to_tensor(df[self.getOrDefault("image_col")].tolist(), self.getOrDefault("image_size"),
                                self.getOrDefault("use_gpu"), self.getOrDefault("transform_fn"))


class DeepVisionModel(Model, _VisionParams):
    model = Param("trained torch module", None, complex=True)

    def setTransformationFn(self, fn):  # noqa: N802  (reference DeepVisionModel spelling)
        return self.set("transform_fn", fn)

    def getTransformationFn(self):  # noqa: N802
        return self.getOrDefault("transform_fn")

    def getOptimizer(self):  # noqa: N802
        """the optimizer the model was trained with (name; the torch optimizer is not kept after training)"""
        return self.getOrDefault("optimizer_name")

    def get_prediction_fn(self):
        """images (bytes / paths / decoded rows) -> class probabilities [N, num_classes] (numpy)"""
        def fn(images):
            X = images_to_tensor(list(images), self.getOrDefault("image_size"), self.getOrDefault("use_gpu"),
                                 self.getOrDefault("transform_fn"))
            return torch.softmax(predict(self.getOrDefault("model"), X, use_gpu=self.getOrDefault("use_gpu")),
                                 dim=1).numpy()

        return fn

    def _transform(self, df):
        prob = self.get_prediction_fn()(df[self.getOrDefault("image_col")].tolist())
        return df.withColumn("probability", prob).withColumn(self.getOrDefault("prediction_col"),
                                                             prob.argmax(1).astype(np.float64))


def _vision_task(est, part, rank, world):
    """One data-parallel rank: build the same (seeded) network, train on this rank's partition; rank 0 returns
    the weights."""
    torch.manual_seed(est.getOrDefault("random_seed"))
    net = backbones.build(est.getOrDefault("backbone"), est.getOrDefault("num_classes"), est.getOrDefault("weights"))
    backbones.head_and_trainable(net, est.getOrDefault("additional_layers_to_train"))
    X = est._images(part)
    hist = fit(net, X, est._labels(part), est._cfg(), shard=False)
    hist["world"] = world
    return ({k: v.cpu() for k, v in net.state_dict().items()}, hist) if rank == 0 else None


class DeepVisionClassifier(Estimator, _VisionParams):
    def get_model_class(self):
        return DeepVisionModel

    def _fit(self, df):
        if self.getOrDefault("num_classes") is None:
            raise ValueError("num_classes must be set")
        nproc = self.getOrDefault("num_proc") or 1
        if nproc > 1:
            import functools

            from ..parallel.runtime import run_partitions

            res = run_partitions(functools.partial(_vision_task, self), df, num_workers=nproc,
                                 use_gpu=self.getOrDefault("use_gpu") and torch.cuda.is_available())
            state, hist = res[0]
            net = backbones.build(self.getOrDefault("backbone"), self.getOrDefault("num_classes"))
            net.load_state_dict(state)
        else:
            torch.manual_seed(self.getOrDefault("random_seed"))
            net = backbones.build(self.getOrDefault("backbone"), self.getOrDefault("num_classes"),
                                  self.getOrDefault("weights"))
            backbones.head_and_trainable(net, self.getOrDefault("additional_layers_to_train"))
            X = self._images(df)
            hist = fit(net, X, self._labels(df), self._cfg())
            hist["world"] = 1
        m = DeepVisionModel(**{k: v for k, v in self.extractParamMap().items() if k in DeepVisionModel._params_decl})
        m.set("model", net.cpu())
        m.history = hist
        return m


# ---------------------------------------------------------------------- text
_PRESETS = {
    # name: (model_type, hidden, layers, heads, intermediate, vocab, max_pos)
    "bert-base-uncased": ("bert", 768, 12, 12, 3072, 30522, 512),
    "bert-base-cased": ("bert", 768, 12, 12, 3072, 28996, 512),
    "bert-large-uncased": ("bert", 1024, 24, 16, 4096, 30522, 512),
    "distilbert-base-uncased": ("distilbert", 768, 6, 12, 3072, 30522, 512),
    "roberta-base": ("roberta", 768, 12, 12, 3072, 50265, 514),
    "microsoft/deberta-v3-base": ("deberta-v2", 768, 12, 12, 3072, 128100, 512),
    "tiny-bert": ("bert", 32, 2, 2, 64, 4096, 128),
}


class HashingWordPieceTokenizer:
    """Deterministic stand-in for a pretrained tokenizer: lower-cased word/punctuation split, words hashed
    (crc32) into the vocabulary above the special ids; [CLS] ... [SEP] + padding."""

    PAD, UNK, CLS, SEP = 0, 100, 101, 102

    def __init__(self, vocab_size: int):
        self.vocab_size = vocab_size
        self.base = 1000 if vocab_size > 2000 else 4

    def ids(self, text: str) -> List[int]:
        words = re.findall(r"\w+|[^\w\s]", (text or "").lower())
        span = self.vocab_size - self.base
        return [self.base + zlib.crc32(w.encode("utf-8")) % span for w in words]

    def __call__(self, texts: List[str], max_length: int) -> Dict[str, torch.Tensor]:
        cls_, sep = (self.CLS, self.SEP) if self.vocab_size > 200 else (1, 2)
        ids = np.zeros((len(texts), max_length), dtype=np.int64)
        mask = np.zeros_like(ids)
        for i, t in enumerate(texts):
            seq = [cls_] + self.ids(t)[: max_length - 2] + [sep]
            ids[i, :len(seq)] = seq
            mask[i, :len(seq)] = 1
        return {"input_ids": torch.as_tensor(ids), "attention_mask": torch.as_tensor(mask)}


def build_text_model(checkpoint: str, num_classes: int, local_dir: Optional[str] = None):
    import transformers as tf

    if local_dir:
        model = tf.AutoModelForSequenceClassification.from_pretrained(local_dir, num_labels=num_classes,
                                                                      local_files_only=True)
        tok = tf.AutoTokenizer.from_pretrained(local_dir, local_files_only=True)
        return model, lambda texts, n: dict(tok(texts, max_length=n, truncation=True, padding="max_length",
                                               return_tensors="pt"))
    if checkpoint not in _PRESETS:
        raise ValueError(f"unknown checkpoint {checkpoint!r} without a local copy; known: {sorted(_PRESETS)}")
    kind, h, L, heads, inter, vocab, maxpos = _PRESETS[checkpoint]
    if kind == "distilbert":
        cfg = tf.DistilBertConfig(vocab_size=vocab, dim=h, n_layers=L, n_heads=heads, hidden_dim=inter,
                                  max_position_embeddings=maxpos, num_labels=num_classes)
    else:
        cfg_cls = {"bert": tf.BertConfig, "roberta": tf.RobertaConfig, "deberta-v2": tf.DebertaV2Config}[kind]
        cfg = cfg_cls(vocab_size=vocab, hidden_size=h, num_hidden_layers=L, num_attention_heads=heads,
                      intermediate_size=inter, max_position_embeddings=maxpos, num_labels=num_classes)
    model = tf.AutoModelForSequenceClassification.from_config(cfg)
    tok = HashingWordPieceTokenizer(vocab)
    return model, lambda texts, n: tok(texts, n)


def _text_forward(m, x):
    return m(**x).logits


class _TextParams(_TrainParams):
    checkpoint = Param("checkpoint of the deep text classifier", "bert-base-uncased", T.toString)
    additional_layers_to_train = Param("number of last encoder layers to fine tune (None/-1 = all)", -1, T.toInt)
    text_col = Param("text column name.", "text", T.toString)
    max_token_len = Param("max_token_len for the tokenizer", 128, T.toInt)
    tokenizer_dir = Param("optional local directory with a pretrained model + tokenizer", None, T.toString)
    tokenizer = Param("tokenizer callable (texts, max_length) -> encodings; the checkpoint's own when unset",
                      None, complex=True)
    train_from_scratch = Param("train every layer (True) or only the last additional_layers_to_train encoder "
                               "layers and the head (False)", True, T.toBoolean)


class DeepTextModel(Model, _TextParams):
    model = Param("trained torch module", None, complex=True)

    def getOptimizer(self):  # noqa: N802
        return self.getOrDefault("optimizer_name")

    def get_prediction_fn(self):
        """texts -> class probabilities [N, num_classes] (numpy)"""
        def fn(texts):
            enc = self.getOrDefault("tokenizer")(list(map(str, texts)), self.getOrDefault("max_token_len"))
            logits = predict(self.getOrDefault("model"), enc, use_gpu=self.getOrDefault("use_gpu"),
                             forward=_text_forward)
            return torch.softmax(logits, dim=1).numpy()

        return fn

    def _transform(self, df):
        prob = self.get_prediction_fn()(df[self.getOrDefault("text_col")].tolist())
        return df.withColumn("probability", prob).withColumn(self.getOrDefault("prediction_col"),
                                                             prob.argmax(1).astype(np.float64))


class DeepTextClassifier(Estimator, _TextParams):
    def get_model_class(self):
        return DeepTextModel

    def _fit(self, df):
        if self.getOrDefault("num_classes") is None:
            raise ValueError("num_classes must be set")
        net, tok = build_text_model(self.getOrDefault("checkpoint"), self.getOrDefault("num_classes"),
                                    self.getOrDefault("tokenizer_dir"))
        if self.getOrDefault("tokenizer") is not None:
            tok = self.getOrDefault("tokenizer")
        k = None if self.getOrDefault("train_from_scratch") else self.getOrDefault("additional_layers_to_train")
        if not self.getOrDefault("train_from_scratch") and (k is None or k < 0):
            raise ValueError("train_from_scratch=False needs additional_layers_to_train >= 0")
        if k is not None and k >= 0:
            for p in net.base_model.parameters():
                p.requires_grad = False
            layers = None
            for attr in ("encoder.layer", "transformer.layer"):
                obj = net.base_model
                try:
                    for a in attr.split("."):
                        obj = getattr(obj, a)
                    layers = obj
                    break
                except AttributeError:
                    continue
            for layer in (list(layers)[-k:] if layers is not None and k > 0 else []):
                for p in layer.parameters():
                    p.requires_grad = True
        enc = tok(list(map(str, df[self.getOrDefault("text_col")].tolist())), self.getOrDefault("max_token_len"))
        hist = fit(net, enc, self._labels(df), self._cfg(), forward=_text_forward)
        m = DeepTextModel(**{k2: v for k2, v in self.extractParamMap().items() if k2 in DeepTextModel._params_decl})
        m.set("model", net.cpu())
        m.set("tokenizer", tok)
        m.history = hist
        return m


__all__ = ["DeepVisionClassifier", "DeepVisionModel", "DeepTextClassifier", "DeepTextModel",
           "HashingWordPieceTokenizer", "images_to_tensor", "build_text_model"]
