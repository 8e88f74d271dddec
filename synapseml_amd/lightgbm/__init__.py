"""MI355X-native gradient boosting with the reference's LightGBM API."""
from .base import InstrumentationMeasures, LightGBMBase
from .booster import LightGBMBooster
from .delegate import LightGBMDelegate
from .models import (LightGBMClassificationModel, LightGBMClassifier, LightGBMRanker, LightGBMRankerModel,
                     LightGBMRegressionModel, LightGBMRegressor)

__all__ = [
    "InstrumentationMeasures", "LightGBMBase", "LightGBMBooster", "LightGBMDelegate", "LightGBMClassificationModel",
    "LightGBMClassifier", "LightGBMRanker", "LightGBMRankerModel", "LightGBMRegressionModel", "LightGBMRegressor",
]
