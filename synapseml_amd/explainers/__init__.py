"""Model interpretability: KernelSHAP and LIME for tabular / vector / image /
text inputs, ICE/PDP, and the regression + superpixel helpers they use
(reference: core/.../explainers, core/.../image/Superpixel*)."""
from .ice import ICETransformer
from .local import (ImageLIME, ImageSHAP, LocalExplainer, TabularLIME, TabularSHAP, TextLIME, TextSHAP, VectorLIME,
                    VectorSHAP, shap_coalitions)
from .regression import lasso, least_squares
from .superpixel import SuperpixelTransformer, censor, clusters_of, slic

__all__ = [n for n in dir() if not n.startswith("_")]
