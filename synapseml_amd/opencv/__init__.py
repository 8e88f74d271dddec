"""OpenCV-semantics image stages under the reference's ``synapse.ml.opencv``
namespace (reference: opencv/src/main/scala/.../opencv/*). Implemented in
``synapseml_amd.image`` (host OpenMP + fused HIP kernels)."""
from ..image import ImageSetAugmenter, ImageTransformer  # noqa: F401

__all__ = ["ImageTransformer", "ImageSetAugmenter"]
