"""General-purpose pipeline stages (reference: core/.../stages/*.scala,
SURVEY §2.2.5 "Mini-batching" and "Other stages")."""
from .batching import (DynamicBufferedBatcher, DynamicMiniBatchTransformer, FixedBatcher, FixedBufferedBatcher,
                       FixedMiniBatchTransformer, FlattenBatch, HasMiniBatcher, TimeIntervalBatcher,
                       TimeIntervalMiniBatchTransformer)
from .basic import (Cacher, ClassBalancer, ClassBalancerModel, DropColumns, EnsembleByKey, Explode, Lambda,
                    MultiColumnAdapter, PartitionConsolidator, RenameColumn, Repartition, SelectColumns,
                    StratifiedRepartition, SummarizeData, TextPreprocessor, Timer, TimerModel, Trie, UDFTransformer,
                    UnicodeNormalize)

__all__ = [n for n in dir() if not n.startswith("_")]
