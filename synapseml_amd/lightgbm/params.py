"""LightGBM estimator params: names, docs and defaults of the reference
(lightgbm/.../params/LightGBMParams.scala, 652 LoC) plus the column params."""
from __future__ import annotations

from ..core.contracts import (HasFeaturesCol, HasInitScoreCol, HasLabelCol, HasPredictionCol,
                              HasValidationIndicatorCol, HasWeightCol)
from ..core.params import Param, TypeConverters as T


class LightGBMExecutionParams(HasFeaturesCol):
    passThroughArgs = Param("Direct string to pass the parameters to LightGBM (first wins)", "", T.toString)
    parallelism = Param("Tree learner parallelism: data_parallel or voting_parallel", "data_parallel", T.toString)
    topK = Param("The top_k value used in Voting parallel", 20, T.toInt)
    defaultListenPort = Param("The default listen port on executors, used for testing", 12400, T.toInt)
    driverListenPort = Param("The listen port on a driver. Default value is 0 (random)", 0, T.toInt)
    timeout = Param("Timeout in seconds", 1200.0, T.toFloat)
    useBarrierExecutionMode = Param("Barrier execution mode (all tasks start together)", False, T.toBoolean)
    samplingMode = Param("Data sampling for streaming mode: global, subset, or fixed", "subset", T.toString)
    samplingSubsetSize = Param("Specify subset size N for the sampling mode 'subset'", 1000000, T.toInt)
    referenceDataset = Param("The reference Dataset (bin boundaries) serialized as bytes", None, complex=True)
    executionMode = Param("Deprecated. Please use dataTransferMode.", None, T.toString)
    dataTransferMode = Param("How data is transferred: streaming or bulk", "streaming", T.toString)
    microBatchSize = Param("Micro-batch size for streaming ingestion", 100, T.toInt)
    useSingleDatasetMode = Param("Use single dataset execution mode (one dataset per executor)", True, T.toBoolean)
    numBatches = Param("If greater than 0, splits data into separate batches during training", 0, T.toInt)
    repartitionByGroupingColumn = Param("Repartition training data by the grouping column", True, T.toBoolean)
    numTasks = Param("Advanced parameter to specify the number of tasks", 0, T.toInt)
    chunkSize = Param("Advanced parameter: chunk size for copying data to native", 10000, T.toInt)
    matrixType = Param("Advanced: dense or sparse native matrix; auto detects", "auto", T.toString)
    numThreads = Param("Number of threads for LightGBM (0 = default)", 0, T.toInt)
    maxStreamingOMPThreads = Param("Max OpenMP threads per task in streaming mode", 16, T.toInt)
    deviceType = Param("Compute device: gpu (MI355X, default) or cpu", "gpu", T.toString)


class LightGBMDatasetParams(LightGBMExecutionParams):
    isEnableSparse = Param("Used to enable/disable sparse optimization", True, T.toBoolean)
    useMissing = Param("Set to false to disable the special handling of missing values", True, T.toBoolean)
    zeroAsMissing = Param("Set to true to treat all zero as missing values", False, T.toBoolean)


class LightGBMLearnerParams(LightGBMDatasetParams):
    earlyStoppingRound = Param("Early stopping round", 0, T.toInt)
    improvementTolerance = Param("Tolerance to consider improvement in metric", 0.0, T.toFloat)
    monotoneConstraints = Param("Monotone constraints per feature", [], T.toListInt)
    monotoneConstraintsMethod = Param("Monotone constraints method: basic, intermediate, advanced", "basic", T.toString)
    monotonePenalty = Param("Monotone penalty", 0.0, T.toFloat)
    topRate = Param("The retain ratio of large gradient data. Only used in goss.", 0.2, T.toFloat)
    otherRate = Param("The retain ratio of small gradient data. Only used in goss.", 0.1, T.toFloat)
    maxBin = Param("Max bin", 255, T.toInt)
    binSampleCount = Param("Number of samples considered at computing histogram bins", 200000, T.toInt)
    dropRate = Param("Dropout rate: a fraction of previous trees to drop during the dropout", 0.1, T.toFloat)
    maxDrop = Param("Max number of dropped trees during one boosting iteration", 50, T.toInt)
    skipDrop = Param("Probability of skipping the dropout procedure during a boosting iteration", 0.5, T.toFloat)
    xGBoostDartMode = Param("Set this to true to use xgboost dart mode", False, T.toBoolean)
    uniformDrop = Param("Set this to true to use uniform drop in dart mode", False, T.toBoolean)
    slotNames = Param("List of slot names in the features column", [], T.toListString)
    categoricalSlotIndexes = Param("List of categorical column indexes, the slot index in the features column", [], T.toListInt)
    categoricalSlotNames = Param("List of categorical column slot names", [], T.toListString)
    baggingFraction = Param("Bagging fraction", 1.0, T.toFloat)
    posBaggingFraction = Param("Positive Bagging fraction", 1.0, T.toFloat)
    negBaggingFraction = Param("Negative Bagging fraction", 1.0, T.toFloat)
    featureFraction = Param("Feature fraction", 1.0, T.toFloat)
    featureFractionByNode = Param("Feature fraction by node", None, T.toFloat)
    seed = Param("Main seed, used to generate other seeds", None, T.toInt)
    deterministic = Param("Used only with cpu devide type. Setting this to true should ensure stable results", False, T.toBoolean)
    baggingSeed = Param("Bagging seed", 3, T.toInt)
    featureFractionSeed = Param("Feature fraction seed", 2, T.toInt)
    extraSeed = Param("Random seed for selecting threshold when extra_trees is true", 6, T.toInt)
    dropSeed = Param("Random seed to choose dropping models. Only used in dart.", 4, T.toInt)
    dataRandomSeed = Param("Random seed for sampling data to construct histogram bins.", 1, T.toInt)
    objectiveSeed = Param("Random seed for objectives, if random process is needed.", 5, T.toInt)
    minDataPerGroup = Param("minimal number of data per categorical group", 100, T.toInt)
    maxCatThreshold = Param("limit number of split points considered for categorical features", 32, T.toInt)
    catl2 = Param("L2 regularization in categorical split", 10.0, T.toFloat)
    catSmooth = Param("this can reduce the effect of noises in categorical features", 10.0, T.toFloat)
    maxCatToOnehot = Param("when number of categories <= this, one-vs-other split is used", 4, T.toInt)
    numIterations = Param("Number of iterations, LightGBM constructs num_class * num_iterations trees", 100, T.toInt)
    learningRate = Param("Learning rate or shrinkage rate", 0.1, T.toFloat)
    numLeaves = Param("Number of leaves", 31, T.toInt)
    baggingFreq = Param("Bagging frequency", 0, T.toInt)
    maxDepth = Param("Max depth", -1, T.toInt)
    minSumHessianInLeaf = Param("Minimal sum hessian in one leaf", 1e-3, T.toFloat)
    modelString = Param("LightGBM model to retrain", "", T.toString)
    checkpointDir = Param("Directory for periodic training checkpoints (model text); fit resumes from the latest "
                          "one when resumeFromCheckpoint is set", None, T.toString)
    checkpointInterval = Param("Write a checkpoint every this many iterations (0 = off)", 0, T.toInt)
    resumeFromCheckpoint = Param("Resume from the latest checkpoint in checkpointDir if one exists and was written "
                                 "by the same job (same params and data)", False, T.toBoolean)
    verbosity = Param("Verbosity where lt 0 is Fatal, eq 0 is Error, eq 1 is Info, gt 1 is Debug", -1, T.toInt)
    boostFromAverage = Param("Adjusts initial score to the mean of labels for faster convergence", True, T.toBoolean)
    boostingType = Param("Default gbdt = traditional Gradient Boosting Decision Tree. Options: gbdt, rf, dart, goss", "gbdt", T.toString)
    lambdaL1 = Param("L1 regularization", 0.0, T.toFloat)
    lambdaL2 = Param("L2 regularization", 0.0, T.toFloat)
    isProvideTrainingMetric = Param("Whether output metric result over training dataset.", False, T.toBoolean)
    metric = Param("Metrics to be evaluated on the evaluation data", "", T.toString)
    minGainToSplit = Param("The minimal gain to perform split", 0.0, T.toFloat)
    maxDeltaStep = Param("Used to limit the max output of tree leaves", 0.0, T.toFloat)
    maxBinByFeature = Param("Max number of bins for each feature", [], T.toListInt)
    minDataPerBin = Param("Minimal number of data inside one bin", 3, T.toInt)
    minDataInLeaf = Param("Minimal number of data in one leaf. Can be used to deal with over-fitting.", 20, T.toInt)
    objective = Param("The Objective", "regression", T.toString)
    fobj = Param("Customized objective function: fobj(preds, dataset) -> (grad, hess)", None, complex=True)
    delegate = Param("Delegate hooks (LightGBMDelegate)", None, complex=True)
    startIteration = Param("Sets the start index of the iteration to predict", 0, T.toInt)
    leafPredictionCol = Param("Predicted leaf indices's column name", "", T.toString)
    featuresShapCol = Param("Output SHAP vector column name after prediction containing the feature contribution values", "", T.toString)
    predictDisableShapeCheck = Param("control whether or not LightGBM raises an error when you try to predict on data with a different number of features than the training data", False, T.toBoolean)


class LightGBMParams(LightGBMLearnerParams, HasLabelCol, HasWeightCol, HasInitScoreCol, HasValidationIndicatorCol,
                     HasPredictionCol):
    pass


class LightGBMModelParams(HasFeaturesCol, HasPredictionCol):
    lightGBMBooster = Param("The trained LightGBM booster", None, complex=True)
    startIteration = Param("Sets the start index of the iteration to predict", 0, T.toInt)
    numIterations = Param("Sets the total number of iterations used in the prediction", -1, T.toInt)
    leafPredictionCol = Param("Predicted leaf indices's column name", "", T.toString)
    featuresShapCol = Param("Output SHAP vector column name after prediction containing the feature contribution values", "", T.toString)
    predictDisableShapeCheck = Param("control whether or not LightGBM raises an error when you try to predict on data with a different number of features than the training data", False, T.toBoolean)
    deviceType = Param("Device used for batch scoring: gpu or cpu", "gpu", T.toString)
