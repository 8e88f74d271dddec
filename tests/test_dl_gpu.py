"""DeepVisionClassifier / DeepTextClassifier fine-tuning on the MI355X (bf16
autocast, channels_last, the trainer's device path) — the CPU suite covers
the same estimators on the host (tests/test_dl.py)."""
import numpy as np
import pytest
import torch

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.dl import DeepTextClassifier, DeepVisionClassifier, TrainConfig, fit

pytestmark = pytest.mark.gpu


def _obj(v):
    a = np.empty(len(v), dtype=object)
    for i, x in enumerate(v):
        a[i] = x
    return a


def test_gpu_deep_vision_classifier_resnet18():
    rng = np.random.default_rng(0)
    imgs, y = [], []
    for i in range(96):
        a = rng.integers(0, 60, size=(40, 48, 3), dtype=np.uint8)
        if i % 2:
            a[:, :, 2] = 220
        imgs.append(a)
        y.append(float(i % 2))
    y = np.asarray(y)
    df = DataFrame({"image": _obj(imgs), "label": y})
    clf = DeepVisionClassifier(backbone="resnet18", num_classes=2, batch_size=32, epochs=6, learning_rate=0.01,
                               additional_layers_to_train=3, image_size=64, use_gpu=True)
    model = clf.fit(df)
    assert model.history["loss"][-1] < model.history["loss"][0]
    out = model.transform(df)
    assert (out["prediction"] == y).mean() >= 0.9


def test_gpu_trainer_bf16_channels_last_matches_loss_scale():
    """The device trainer (bf16 autocast + channels_last) reduces the loss like the fp32 CPU trainer."""
    torch.manual_seed(0)
    X = torch.randn(256, 3, 16, 16)
    Y = (X[:, 0].mean(dim=(1, 2)) > 0).long()
    losses = {}
    for gpu in (False, True):
        torch.manual_seed(1)
        m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.ReLU(), torch.nn.AdaptiveAvgPool2d(1),
                                torch.nn.Flatten(), torch.nn.Linear(8, 2))
        hist = fit(m, X, Y, TrainConfig(epochs=8, batch_size=32, learning_rate=0.05, use_gpu=gpu))
        losses[gpu] = hist["loss"] if isinstance(hist, dict) else hist
    assert losses[True][-1] < losses[True][0]
    assert abs(losses[True][-1] - losses[False][-1]) < 0.2


def test_gpu_deep_text_classifier_tiny():
    pos = ["great movie loved it", "wonderful acting great plot", "loved the music", "great fun"]
    neg = ["terrible movie hated it", "awful acting bad plot", "hated the music", "bad boring"]
    texts = (pos + neg) * 4
    y = np.asarray(([1.0] * 4 + [0.0] * 4) * 4)
    df = DataFrame({"text": _obj(texts), "label": y})
    clf = DeepTextClassifier(checkpoint="tiny-bert", num_classes=2, batch_size=8, epochs=15, learning_rate=3e-3,
                             max_token_len=16, use_gpu=True)
    out = clf.fit(df).transform(df)
    assert (out["prediction"] == y).mean() >= 0.9
