"""Deep-learning estimators (reference: deep-learning/.../synapse/ml/dl/**):
data-parallel fine-tuning over torch.distributed (RCCL on MI355X)."""
from .backbones import available as available_backbones
from .estimators import (DeepTextClassifier, DeepTextModel, DeepVisionClassifier, DeepVisionModel,
                         HashingWordPieceTokenizer)
from .trainer import TrainConfig, fit, predict

__all__ = ["DeepVisionClassifier", "DeepVisionModel", "DeepTextClassifier", "DeepTextModel",
           "HashingWordPieceTokenizer", "TrainConfig", "fit", "predict", "available_backbones"]
