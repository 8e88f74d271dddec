"""User hooks around LightGBM training (reference: lightgbm/.../LightGBMDelegate.scala:12-61)."""
from __future__ import annotations


class LightGBMDelegate:
    def beforeTrainBatch(self, batchIndex, log, dataset, previousBooster):  # noqa: N802,N803
        pass

    def afterTrainBatch(self, batchIndex, log, dataset, booster):  # noqa: N802,N803
        pass

    def beforeGenerateTrainDataset(self, batchIndex, partitionId, columnParams, schema, log, trainParams):  # noqa: N802,N803
        pass

    def afterGenerateTrainDataset(self, batchIndex, partitionId, columnParams, schema, log, trainParams):  # noqa: N802,N803
        pass

    def beforeGenerateValidDataset(self, batchIndex, partitionId, columnParams, schema, log, trainParams):  # noqa: N802,N803
        pass

    def afterGenerateValidDataset(self, batchIndex, partitionId, columnParams, schema, log, trainParams):  # noqa: N802,N803
        pass

    def beforeTrainIteration(self, batchIndex, partitionId, curIters, log, trainParams, booster, hasValid):  # noqa: N802,N803
        pass

    def afterTrainIteration(self, batchIndex, partitionId, curIters, log, trainParams, booster, hasValid,  # noqa: N802,N803
                            isFinished, trainEvalResults, validEvalResults):  # noqa: N803
        pass

    def getLearningRate(self, batchIndex, partitionId, curIters, log, trainParams, previousLearningRate):  # noqa: N802,N803
        return previousLearningRate
