"""Model families: SparkML-API base learners (linear, naive Bayes, MLP, trees on
the native GBDT engine) and evaluators. LightGBM / VW / ONNX / DL live in
their own packages."""
from .evaluation import (BinaryClassificationEvaluator, MulticlassClassificationEvaluator, RegressionEvaluator, auc,
                         classification_metrics, confusion_matrix, regression_metrics)
from .linear import (LinearRegression, LinearRegressionModel, LogisticRegression, LogisticRegressionModel,
                     MultilayerPerceptronClassificationModel, MultilayerPerceptronClassifier, NaiveBayes,
                     NaiveBayesModel)
from .trees import (DecisionTreeClassificationModel, DecisionTreeClassifier, DecisionTreeRegressionModel,
                    DecisionTreeRegressor, GBTClassificationModel, GBTClassifier, GBTRegressionModel, GBTRegressor,
                    RandomForestClassificationModel, RandomForestClassifier, RandomForestRegressionModel,
                    RandomForestRegressor)

__all__ = [n for n in dir() if not n.startswith("_")]
