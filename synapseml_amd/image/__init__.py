"""Image processing (reference: opencv/ ImageTransformer & ImageSetAugmenter,
core/ image UnrollImage / Superpixel): OpenCV-semantics stages on native host
kernels and the fused batched HIP preprocess kernel (K19)."""
from .schema import (CV_8UC1, CV_8UC3, CV_8UC4, decode_bytes, encode_png, images_column, make_image_row,
                     read_binary_files, read_images, row_to_array)
from .transformer import (Blur, CenterCropImage, ColorFormat, CropImage, Flip, GaussianKernel, ImageSetAugmenter,
                          ImageTransformer, ResizeImage, ResizeImageTransformer, Threshold, UnrollBinaryImage,
                          UnrollImage, roll, unroll)

__all__ = [n for n in dir() if not n.startswith("_")]
