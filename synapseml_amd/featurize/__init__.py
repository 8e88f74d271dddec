"""Featurization (reference: core/.../featurize) plus the
SparkML feature primitives it builds on (ml.py)."""
from .featurize import (CleanMissingData, CleanMissingDataModel, CountSelector, CountSelectorModel, DataConversion,
                        Featurize, IndexToValue, MultiNGram, PageSplitter, TextFeaturizer, TextFeaturizerModel,
                        ValueIndexer, ValueIndexerModel, categorical_metadata)
from .ml import (IDF, HashingTF, IDFModel, NGram, OneHotEncoder, OneHotEncoderModel, RegexTokenizer, StopWordsRemover,
                 StringIndexer, StringIndexerModel, Tokenizer, VectorAssembler, FastVectorAssembler)

__all__ = [n for n in dir() if not n.startswith("_")]
