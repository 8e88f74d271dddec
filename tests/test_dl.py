"""Deep vision / text classifiers (reference tests: deep-learning/src/test/python/
synapsemltest/dl/test_deep_{vision,text}_classifier.py, which fine-tune pretrained
zoo models on flowers / text datasets; here: random-init backbones on synthetic
separable data, CPU, plus a gloo world-size-2 DDP run)."""
import os

import numpy as np
import pytest
import torch

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.dl import DeepTextClassifier, DeepVisionClassifier, HashingWordPieceTokenizer, TrainConfig, fit
from synapseml_amd.dl import backbones


def _obj(v):
    a = np.empty(len(v), dtype=object)
    for i, x in enumerate(v):
        a[i] = x
    return a


def _images(n, seed=0):
    rng = np.random.default_rng(seed)
    imgs, y = [], []
    for i in range(n):
        lab = i % 2
        a = rng.integers(0, 60, size=(40, 48, 3), dtype=np.uint8)
        if lab:
            a[:, :, 2] = 220  # red in BGR order
        imgs.append(a)
        y.append(float(lab))
    return imgs, np.asarray(y)


def test_backbone_zoo_shapes_and_freezing():
    for name in ["resnet18", "resnet50", "resnext50_32x4d", "wide_resnet50_2"]:
        m = backbones.build(name, num_classes=7)
        assert m.fc.out_features == 7
    m = backbones.build("resnet50", 5)
    assert sum(p.numel() for p in m.parameters()) > 23_000_000
    backbones.head_and_trainable(m, 1)
    trainable = {n.split(".")[0] for n, p in m.named_parameters() if p.requires_grad}
    assert trainable == {"fc", "layer4"}
    with pytest.raises(ValueError):
        backbones.head_and_trainable(m, 4)
    with pytest.raises(ValueError):
        backbones.build("nope", 2)
    out = backbones.build("resnet_tiny", 3)(torch.randn(2, 3, 64, 64))
    assert out.shape == (2, 3)


def test_deep_vision_classifier_learns_color():
    imgs, y = _images(48)
    df = DataFrame({"image": _obj(imgs), "label": y})
    clf = DeepVisionClassifier(backbone="resnet_tiny", num_classes=2, batch_size=16, epochs=8, learning_rate=0.01,
                               additional_layers_to_train=3, image_size=32, use_gpu=False)
    assert clf.getNumClasses() == 2 and clf.getAdditionalLayersToTrain() == 3
    model = clf.fit(df)
    assert model.history["loss"][-1] < model.history["loss"][0]
    out = model.transform(df)
    acc = (out["prediction"] == y).mean()
    assert acc >= 0.9
    assert out["probability"].shape == (48, 2)


def test_deep_vision_from_paths(tmp_path):
    from synapseml_amd.image.schema import encode_png

    imgs, y = _images(8, seed=1)
    paths = []
    for i, a in enumerate(imgs):
        p = tmp_path / f"{i}.png"
        p.write_bytes(encode_png(a))
        paths.append(str(p))
    df = DataFrame({"image": _obj(paths), "label": y})
    m = DeepVisionClassifier(backbone="resnet_tiny", num_classes=2, batch_size=4, epochs=1, image_size=32,
                             use_gpu=False).fit(df)
    assert m.transform(df).count() == 8


def test_hashing_tokenizer_deterministic():
    tok = HashingWordPieceTokenizer(30522)
    a = tok(["Hello, world!", "hello world"], 8)
    assert a["input_ids"][0, 0] == 101 and a["input_ids"][0, 5] == 102
    assert a["input_ids"][0, 1] == a["input_ids"][1, 1]  # case-insensitive
    assert a["attention_mask"][1].tolist() == [1, 1, 1, 1, 0, 0, 0, 0]


def test_deep_text_classifier_tiny():
    pos = ["great movie loved it", "wonderful acting great plot", "loved the music", "great fun"]
    neg = ["terrible movie hated it", "awful acting bad plot", "hated the music", "bad boring"]
    texts = (pos + neg) * 4
    y = np.asarray(([1.0] * 4 + [0.0] * 4) * 4)
    df = DataFrame({"text": _obj(texts), "label": y})
    clf = DeepTextClassifier(checkpoint="tiny-bert", num_classes=2, batch_size=8, epochs=15, learning_rate=3e-3,
                             max_token_len=16, use_gpu=False)
    m = clf.fit(df)
    out = m.transform(df)
    assert (out["prediction"] == y).mean() >= 0.9


def _ddp_task(part, rank, world):
    torch.manual_seed(0)
    model = torch.nn.Linear(4, 2)
    X = torch.randn(64, 4, generator=torch.Generator().manual_seed(1))
    Y = (X[:, 0] > 0).long()
    fit(model, X, Y, TrainConfig(epochs=3, batch_size=8, learning_rate=0.1, use_gpu=False))
    return [p.detach().clone() for p in model.parameters()]


def test_ddp_gloo_world2_keeps_replicas_identical():
    from synapseml_amd.parallel.runtime import run_partitions

    res = run_partitions(_ddp_task, DataFrame({"x": np.arange(4)}, num_partitions=2), num_workers=2)
    for a, b in zip(res[0], res[1]):
        torch.testing.assert_close(a, b)


def test_deep_vision_num_proc_2():
    imgs, y = _images(16, seed=2)
    df = DataFrame({"image": _obj(imgs), "label": y}, num_partitions=2)
    m = DeepVisionClassifier(backbone="resnet_tiny", num_classes=2, batch_size=4, epochs=1, image_size=32,
                             use_gpu=False, num_proc=2).fit(df)
    assert m.history["world"] == 2
    assert m.transform(df)["probability"].shape == (16, 2)
