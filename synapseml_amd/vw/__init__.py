"""Vowpal Wabbit-compatible online learning (reference: vw/ module, SURVEY
§2.2.3): native C++ learner (``_vw``) with a HIP hogwild SGD path, hashing
featurizers, regressor/classifier/contextual-bandit/generic estimators,
progressive validation, DSJson/CSE bandit-log transformers and off-policy
estimators."""
from .featurizer import (VowpalWabbitFeaturizer, VowpalWabbitInteractions, VowpalWabbitMurmur,
                         VowpalWabbitMurmurWithPrefix, murmur_hash, sort_and_distinct)
from .learners import (VowpalWabbitClassificationModel, VowpalWabbitClassifier, VowpalWabbitGeneric,
                       VowpalWabbitGenericModel, VowpalWabbitGenericProgressive, VowpalWabbitProgressive,
                       VowpalWabbitRegressionModel, VowpalWabbitRegressor)
from .bandit import ContextualBanditMetrics, VowpalWabbitContextualBandit, VowpalWabbitContextualBanditModel
from .transformers import VectorZipper, VowpalWabbitCSETransformer, VowpalWabbitDSJsonTransformer
from .policyeval import CressieRead, CressieReadInterval, Ips, KahanSum, Snips

__all__ = [n for n in dir() if n[0].isupper() or n in ("murmur_hash", "sort_and_distinct")]
