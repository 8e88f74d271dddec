"""ImageTransformer, ImageSetAugmenter, UnrollImage / UnrollBinaryImage,
ResizeImageTransformer.

Reference: opencv/.../ImageTransformer.scala:31-725 (stages 68-283, tensor
conversion 335-415, transform 643-686), ImageSetAugmenter.scala:18-77,
core/.../image/UnrollImage.scala:27-250.

Execution: stage semantics are the OpenCV ones (csrc/image/image_ops.h). On
the MI355X the common inference pipeline — decode → resize → (center)crop →
channel reorder → normalize → CHW tensor — runs as ONE batched HIP kernel
(K19, csrc/image/image_gpu.hip) over a packed host→device upload. Every other
stage list (resize incl. keepAspectRatio, crop, centerCrop, colorFormat, flip,
blur, threshold, gaussianKernel, optionally followed by toTensor) runs on the
device too, as batched K20 launches over images of one shape that stay
resident in HBM from the upload to the last stage; results are bit-identical
to the host kernels (deviceType="cpu").
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..core.contracts import HasInputCol, HasOutputCol
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Transformer
from ..ops import native
from .schema import make_image_row, row_to_array, to_array

# The reference keys every stage map by "action" (ImageTransformerStage.stageNameKey,
# ImageTransformer.scala:39); maps written by an older build of this package used
# "stageName" and are still read.
STAGE_NAME = "action"
_LEGACY_STAGE_NAME = "stageName"


def stage_action(stage: dict) -> str:
    """The stage's name ("resize", "crop", ...) from a reference-style map."""
    if STAGE_NAME in stage:
        return stage[STAGE_NAME]
    if _LEGACY_STAGE_NAME in stage:
        return stage[_LEGACY_STAGE_NAME]
    raise KeyError(f"image stage map has no {STAGE_NAME!r} key: {stage!r}")


class _Stage:
    """Named stage-map builders (the reference's ImageTransformer stage objects,
    ImageTransformer.scala:31-283): ``ResizeImage.stageName == "resize"`` and
    ``ResizeImage.make(height=.., width=..)`` gives the map an ImageTransformer
    ``stages`` list holds."""

    stageName = ""

    @classmethod
    def make(cls, **params) -> dict:
        return {STAGE_NAME: cls.stageName, **params}


class ResizeImage(_Stage):
    stageName = "resize"


class CropImage(_Stage):
    stageName = "crop"


class CenterCropImage(_Stage):
    stageName = "centercrop"


class ColorFormat(_Stage):
    stageName = "colorformat"


class Flip(_Stage):
    stageName = "flip"


class Blur(_Stage):
    stageName = "blur"


class Threshold(_Stage):
    stageName = "threshold"


class GaussianKernel(_Stage):
    stageName = "gaussiankernel"


def _img():
    return native.load("_image")


_COPY_POOL: Optional[ThreadPoolExecutor] = None


def _parallel_copy(dst_views, srcs) -> None:
    """dst_views[i][...] = srcs[i] on a small thread pool (numpy releases the GIL for plain copies), in at most
    16 tasks of consecutive images (a task per image cost more than its copy: r6 pass 19)."""
    global _COPY_POOL
    n = len(srcs)
    if n < 8:
        for d, a in zip(dst_views, srcs):
            d[...] = a
        return
    if _COPY_POOL is None:
        _COPY_POOL = ThreadPoolExecutor(max_workers=16)
    nt = min(16, n)

    def put(t):
        for k in range(n * t // nt, n * (t + 1) // nt):
            dst_views[k][...] = srcs[k]

    list(_COPY_POOL.map(put, range(nt)))


def _gather_images(dst: np.ndarray, arrays) -> None:
    """dst[j] = arrays[j] for equally shaped uint8 images: one native call, copies spread over a thread team
    with the GIL released (falls back to the pool for non-contiguous sources)."""
    try:
        if dst.dtype != np.uint8 or any(a.dtype != np.uint8 for a in arrays):
            raise TypeError("non-uint8 image")
        _img().gather_into(list(arrays), dst.ctypes.data, int(dst[0].nbytes))
    except (ValueError, TypeError):
        _parallel_copy([dst[j] for j in range(len(arrays))], list(arrays))


def _bulk_copy(host: np.ndarray, n: int) -> np.ndarray:
    """The first n images of a (reused) pinned slot copied into a fresh array, in parallel (native team)."""
    fresh = np.empty((n,) + host.shape[1:], dtype=host.dtype)
    if n:
        _img().copy_parallel(fresh.ctypes.data, host.ctypes.data, int(fresh.nbytes))
    return fresh


def _image_rows(host: np.ndarray, n: int, origins) -> list:
    """Image rows of the first n HWC images of a (reused) pinned slot: the rows' data bytes are made and
    filled in parallel by one native call (numpy's tobytes per row held the GIL: ~27 us per 150 KB row)."""
    if n == 0:
        return []
    h, w = int(host.shape[1]), int(host.shape[2])
    c = int(host.shape[3]) if host.ndim == 4 else 1
    if c not in (1, 3, 4):
        return [make_image_row(host[j], origins[j]) for j in range(n)]
    datas = _img().split_bytes(host.ctypes.data, n, h * w * c)
    mode = {1: 0, 3: 16, 4: 24}[c]
    return [{"origin": origins[j], "height": h, "width": w, "nChannels": c, "mode": mode, "data": datas[j]}
            for j in range(n)]


def _gpu_ok(device_type: str) -> bool:
    dt = (device_type or "auto").lower()
    if dt == "cpu":
        return False
    try:
        import torch

        ok = torch.cuda.is_available()
    except Exception:
        ok = False
    if dt in ("gpu", "cuda", "rocm") and not ok:
        raise RuntimeError("deviceType='gpu' requested but no HIP device is visible")
    return ok


# ---------------------------------------------------------------------- stage application (host)
def resize_target(stage: dict, h: int, w: int) -> Tuple[int, int]:
    if "size" in stage:
        size = int(stage["size"])
        if stage.get("keepAspectRatio", False):
            ratio = size / min(w, h)
            return _jround(ratio * h), _jround(ratio * w)
        return size, size
    return int(stage["height"]), int(stage["width"])


def _jround(x: float) -> int:
    """java.lang.Math.round (half up)."""
    return int(np.floor(x + 0.5))


def center_crop_rect(stage: dict, h: int, w: int) -> Tuple[int, int, int, int]:
    ch, cw = min(int(stage["height"]), h), min(int(stage["width"]), w)
    y = h // 2 - ch // 2
    x = w // 2 - cw // 2
    return y, x, ch, cw


def apply_stage(stage: dict, a: np.ndarray) -> np.ndarray:
    lib = _img()
    name = stage_action(stage)
    if name == "resize":
        th, tw = resize_target(stage, a.shape[0], a.shape[1])
        out = lib.resize(a, th, tw)
        return out if out.ndim == 3 else out[:, :, None]
    if name == "crop":
        x, y, h, w = int(stage["x"]), int(stage["y"]), int(stage["height"]), int(stage["width"])
        if x + w > a.shape[1] or y + h > a.shape[0]:
            raise ValueError("crop rectangle outside the image")
        return np.ascontiguousarray(a[y:y + h, x:x + w])
    if name == "centercrop":
        y, x, ch, cw = center_crop_rect(stage, a.shape[0], a.shape[1])
        return np.ascontiguousarray(a[y:y + ch, x:x + cw])
    if name == "colorformat":
        out = lib.cvt_color(a, int(stage["format"]))
        return out if out.ndim == 3 else out[:, :, None]
    if name == "flip":
        code = int(stage.get("flipCode", 1))
        if code == 0:
            return np.ascontiguousarray(a[::-1])
        if code > 0:
            return np.ascontiguousarray(a[:, ::-1])
        return np.ascontiguousarray(a[::-1, ::-1])
    if name == "blur":
        # Imgproc.blur(image, dst, new Size(height, width)): Size(width=height, height=width)
        kw, kh = int(stage["height"]), int(stage["width"])
        out = lib.box_blur(a, kw, kh)
        return out if out.ndim == 3 else out[:, :, None]
    if name == "threshold":
        out = lib.threshold(a, float(stage["threshold"]), float(stage["maxVal"]), int(stage["type"]))
        return out if out.ndim == 3 else out[:, :, None]
    if name == "gaussiankernel":
        k = lib.gaussian_kernel(int(stage["apertureSize"]), float(stage["sigma"]))
        out = lib.column_filter(a, k)
        return out if out.ndim == 3 else out[:, :, None]
    raise ValueError(f"unknown image stage {name}")


def channel_map(c: int, order: str, auto_color: bool) -> List[int]:
    """Output channel k <- source channel (extractChannels, ImageTransformer.scala:344-374)."""
    rgb = order.lower() == "rgb"
    if c >= 3:
        return [2, 1, 0] if rgb else [0, 1, 2]
    if c == 1 and auto_color:
        return [0, 0, 0]
    return list(range(c))


# ---------------------------------------------------------------------- transformer
class ImageTransformer(Transformer, HasInputCol, HasOutputCol):
    stages = Param("Image transformation stages", [], T.identity)
    toTensor = Param("Convert output image to tensor in the shape of (C * H * W)", False, T.toBoolean)
    tensorElementType = Param("The element data type for the output tensor (float | double)", "float", T.toString)
    tensorChannelOrder = Param("The color channel order of the output channels. Valid values are RGB and BGR.",
                               "RGB", T.toString)
    normalizeMean = Param("The mean value to use for normalization for each channel", None, T.identity)
    normalizeStd = Param("The standard deviation to use for normalization for each channel", None, T.identity)
    colorScaleFactor = Param("The scale factor for color values.", None, T.toFloat)
    autoConvertToColor = Param("Whether to automatically convert black and white images to color", False,
                               T.toBoolean)
    ignoreDecodingErrors = Param("Whether to throw on decoding errors or just return null", False, T.toBoolean)
    deviceType = Param("auto | cpu | gpu — where batches of images are processed", "auto", T.toString)
    batchSize = Param("Images per device batch", 256, T.toInt)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(inputCol="image", outputCol=self.uid + "_output")

    # ---- builder API
    def _add(self, stage: dict) -> "ImageTransformer":
        self.set("stages", list(self.getStages() or []) + [stage])
        return self

    def resize(self, size=None, keep_aspect_ratio=True, height: Optional[int] = None, width: Optional[int] = None,
               keepAspectRatio: Optional[bool] = None):  # noqa: N803
        if keepAspectRatio is not None:
            keep_aspect_ratio = keepAspectRatio
        if height is not None and width is not None:
            return self._add({STAGE_NAME: "resize", "height": int(height), "width": int(width)})
        if isinstance(size, tuple):
            return self._add({STAGE_NAME: "resize", "height": int(size[1]), "width": int(size[0])})
        if isinstance(keep_aspect_ratio, (int, np.integer)) and not isinstance(keep_aspect_ratio, bool):
            # Scala form resize(height, width)
            return self._add({STAGE_NAME: "resize", "height": int(size), "width": int(keep_aspect_ratio)})
        if size is None or int(size) < 0:
            raise ValueError("size should be non-negative")
        return self._add({STAGE_NAME: "resize", "size": int(size), "keepAspectRatio": bool(keep_aspect_ratio)})

    def crop(self, x: int, y: int, height: int, width: int):
        if min(x, y, height, width) < 0:
            raise ValueError("crop values should be non-negative")
        return self._add({STAGE_NAME: "crop", "x": x, "y": y, "height": height, "width": width})

    def centerCrop(self, height: int, width: int):  # noqa: N802
        if min(height, width) < 0:
            raise ValueError("crop values should be non-negative")
        return self._add({STAGE_NAME: "centercrop", "height": height, "width": width})

    def colorFormat(self, format: int):  # noqa: N802,A002
        return self._add({STAGE_NAME: "colorformat", "format": int(format)})

    def flip(self, flip_code: int = 1):
        return self._add({STAGE_NAME: "flip", "flipCode": int(flip_code)})

    def blur(self, height: float, width: float):
        return self._add({STAGE_NAME: "blur", "height": float(height), "width": float(width)})

    def threshold(self, threshold: float, max_val: float, threshold_type: int):
        return self._add({STAGE_NAME: "threshold", "threshold": float(threshold), "maxVal": float(max_val),
                          "type": int(threshold_type)})

    def gaussianKernel(self, aperture_size: int, sigma: float):  # noqa: N802
        return self._add({STAGE_NAME: "gaussiankernel", "apertureSize": int(aperture_size), "sigma": float(sigma)})

    def normalize(self, mean: Sequence[float], std: Sequence[float], color_scale_factor: float):
        self.set("toTensor", True)
        self.set("normalizeMean", [float(v) for v in mean])
        self.set("normalizeStd", [float(v) for v in std])
        self.set("colorScaleFactor", float(color_scale_factor))
        return self

    # ---- execution
    def _fused_plan(self, shapes: List[tuple]):
        """(resize_h, resize_w, crop) when the stage list maps onto K19 for a batch of (h, w, c) shapes."""
        st = list(self.getStages() or [])
        if not self.getToTensor() or self.getTensorElementType().lower() != "float":
            return None
        rs = None
        crop = None
        i = 0
        if i < len(st) and stage_action(st[i]) == "resize":
            if "size" in st[i] and st[i].get("keepAspectRatio", False):
                return None
            rs = resize_target(st[i], 1, 1)
            i += 1
        if i < len(st) and stage_action(st[i]) in ("centercrop", "crop"):
            crop = st[i]
            i += 1
        if i != len(st):
            return None
        hw = {tuple(sh[:2]) for sh in shapes}
        if rs is None and len(hw) != 1:
            return None
        base_h, base_w = rs if rs is not None else next(iter(hw))
        if crop is None:
            cy, cx, ch, cw = 0, 0, base_h, base_w
        elif stage_action(crop) == "centercrop":
            cy, cx, ch, cw = center_crop_rect(crop, base_h, base_w)
        else:
            cy, cx, ch, cw = int(crop["y"]), int(crop["x"]), int(crop["height"]), int(crop["width"])
            if cy + ch > base_h or cx + cw > base_w:
                return None
        if len({sh[2] for sh in shapes}) != 1:
            return None
        return (rs or (0, 0)), (cy, cx, ch, cw)

    def _norm_params(self, cout: int):
        mean = self.getNormalizeMean() or [0.0] * cout
        std = self.getNormalizeStd() or [1.0] * cout
        if len(mean) != cout or len(std) != cout:
            raise ValueError(f"channelLength: {cout}, means length: {len(mean)}, std length: {len(std)}")
        scale = self.getColorScaleFactor()
        return [float(m) for m in mean], [float(s) for s in std], float(scale if scale is not None else 1.0)

    def device_tensors(self, arrays: List[np.ndarray], dtype: str = "float32", nhwc: bool = False,
                       src_rgb: bool = False):
        """Run the fused K19 path on a batch; returns a device tensor [B,C,H,W] or None if not applicable.
        ``src_rgb``: the 3-channel arrays are in RGB order (decode_bytes_rgb) instead of OpenCV's BGR; the
        kernel's channel map absorbs the difference."""
        import torch

        shapes = [a.shape for a in arrays]
        if not arrays or self._fused_plan(shapes) is None:
            return None
        sizes = [a.size for a in arrays]
        offsets = np.zeros(len(arrays), np.int64)
        offsets[1:] = np.cumsum(sizes)[:-1]
        host = torch.empty(int(sum(sizes)), dtype=torch.uint8, pin_memory=True)
        hv = host.numpy()
        try:  # back to back, one native call (the offsets are the running sizes)
            if any(a.dtype != np.uint8 for a in arrays):
                raise TypeError("non-uint8 image")
            _img().gather_into(list(arrays), hv.ctypes.data, 0)
        except (ValueError, TypeError):
            _parallel_copy([hv[o:o + a.size] for a, o in zip(arrays, offsets)], [a.reshape(-1) for a in arrays])
        return self.device_tensors_packed(host, offsets, shapes, dtype, nhwc, src_rgb)

    def device_tensors_packed(self, host, offsets: np.ndarray, shapes: List[tuple], dtype: str = "float32",
                              nhwc: bool = False, src_rgb: bool = False):
        """:meth:`device_tensors` on images already packed into one pinned uint8 buffer (image i at
        ``offsets[i]``, HWC ``shapes[i]``) - e.g. written there directly by the native JPEG decoder."""
        import torch

        plan = self._fused_plan(shapes)
        if plan is None or not shapes:
            return None
        (rh, rw), (cy, cx, ch, cw) = plan
        c = shapes[0][2]
        cmap = channel_map(c, self.getTensorChannelOrder(), self.getAutoConvertToColor())
        if src_rgb and c == 3:
            cmap = [2 - k for k in cmap]
        mean, std, scale = self._norm_params(len(cmap))
        dims = np.array([[sh[0], sh[1], sh[2]] for sh in shapes], np.int32).reshape(-1)
        dev = torch.device("cuda", torch.cuda.current_device())
        src = host.to(dev, non_blocking=True)
        off_d = torch.from_numpy(np.ascontiguousarray(offsets, np.int64)).to(dev, non_blocking=True)
        dims_d = torch.from_numpy(dims).to(dev, non_blocking=True)
        tdt = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}[dtype]
        B = len(shapes)
        out = torch.empty((B, ch, cw, len(cmap)) if nhwc else (B, len(cmap), ch, cw), dtype=tdt, device=dev)
        if min(rh, rw) == 0:
            for sh in shapes:
                if cy + ch > sh[0] or cx + cw > sh[1]:
                    raise ValueError("crop rectangle outside the image")
        _img().preprocess_batch_device(src.data_ptr(), off_d.data_ptr(), dims_d.data_ptr(), B, ch, cw, rh, rw, cy, cx,
                                       cmap, scale, mean, std, {torch.float32: 0, torch.float16: 1,
                                                                torch.bfloat16: 2}[tdt], int(nhwc), out.data_ptr(),
                                       torch.cuda.current_stream(dev).cuda_stream, [int(v) for v in dims])
        if nhwc:
            out = out.permute(0, 3, 1, 2)  # logical NCHW view, channels-last memory
        # keep the upload buffers alive until the kernel has consumed them
        out._sml_keepalive = (host, src, off_d, dims_d)
        return out

    # ---- K20: any stage list on the device, one uniform-shape batch at a time
    _DEVICE_STAGES = ("resize", "crop", "centercrop", "colorformat", "flip", "blur", "threshold", "gaussiankernel")

    def run_stages_device(self, batch):
        """The stage list on a batch of equally shaped HWC uint8 images ([B, h, w, c]: numpy, or a pinned torch
        tensor) on the MI355X; returns the resident device result [B, h', w', c'] (torch uint8) or None when a
        stage has no device form for this shape (the host path then runs)."""
        import torch

        stages = list(self.getStages() or [])
        if any(stage_action(st) not in self._DEVICE_STAGES for st in stages) or batch.ndim != 4:
            return None
        lib = _img()
        dev = torch.device("cuda", torch.cuda.current_device())
        stream = torch.cuda.current_stream(dev).cuda_stream
        if isinstance(batch, np.ndarray):
            batch = torch.from_numpy(np.ascontiguousarray(batch)).pin_memory()
        x = batch.to(dev, non_blocking=True)
        keep = [x]
        for st in stages:
            B, h, w, c = x.shape
            name = stage_action(st)
            if c not in (1, 3, 4) and name in ("resize", "crop", "centercrop", "flip"):
                return None
            if name == "resize":
                th, tw = resize_target(st, h, w)
                y = torch.empty((B, th, tw, c), dtype=torch.uint8, device=dev)
                lib.resize_batch_device(x.data_ptr(), B, h, w, c, y.data_ptr(), th, tw, stream)
            elif name in ("crop", "centercrop"):
                if name == "crop":
                    cy, cx, ch, cw = int(st["y"]), int(st["x"]), int(st["height"]), int(st["width"])
                    if cx + cw > w or cy + ch > h:
                        raise ValueError("crop rectangle outside the image")
                else:
                    cy, cx, ch, cw = center_crop_rect(st, h, w)
                y = torch.empty((B, ch, cw, c), dtype=torch.uint8, device=dev)
                lib.crop_flip_batch_device(x.data_ptr(), B, h, w, c, y.data_ptr(), ch, cw, cy, cx, -1, stream)
            elif name == "colorformat":
                code = int(st["format"])
                cout = lib.cvt_channels_out(code, c)
                y = torch.empty((B, h, w, cout), dtype=torch.uint8, device=dev)
                lib.cvt_color_device(x.data_ptr(), B * h * w, c, code, y.data_ptr(), stream)
            elif name == "flip":
                y = torch.empty_like(x)
                lib.flip_batch_device(x.data_ptr(), B, h, w, c, y.data_ptr(), int(st.get("flipCode", 1)), stream)
            elif name == "blur":
                y = torch.empty_like(x)
                # Imgproc.blur(image, dst, new Size(height, width)): Size(width=height, height=width)
                lib.box_blur_batch_device(x.data_ptr(), B, h, w, c, y.data_ptr(), int(st["height"]), int(st["width"]),
                                          stream)
            elif name == "threshold":
                y = torch.empty_like(x)
                lib.threshold_device(x.data_ptr(), x.numel(), y.data_ptr(), float(st["threshold"]), float(st["maxVal"]),
                                     int(st["type"]), stream)
            else:  # gaussiankernel
                k = lib.gaussian_kernel(int(st["apertureSize"]), float(st["sigma"]))
                y = torch.empty_like(x)
                lib.column_filter_batch_device(x.data_ptr(), B, h, w, c, y.data_ptr(), list(k), stream)
            keep.append(y)
            x = y
        x._sml_keepalive = keep
        return x

    def tensors_from_device_images(self, x, dtype: str = "float32"):
        """toTensor of a resident [B, h, w, c] uint8 batch: the K19 kernel with no resize / crop."""
        import torch

        B, h, w, c = x.shape
        cmap = channel_map(c, self.getTensorChannelOrder(), self.getAutoConvertToColor())
        mean, std, scale = self._norm_params(len(cmap))
        dev = x.device
        offsets = torch.arange(B, dtype=torch.int64, device=dev) * (h * w * c)
        dims = torch.tensor([h, w, c] * B, dtype=torch.int32, device=dev)
        tdt = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}[dtype]
        out = torch.empty((B, len(cmap), h, w), dtype=tdt, device=dev)
        _img().preprocess_batch_device(x.data_ptr(), offsets.data_ptr(), dims.data_ptr(), B, h, w, 0, 0, 0, 0, cmap,
                                       scale, mean, std, {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[tdt],
                                       0, out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        out._sml_keepalive = (x, offsets, dims)
        return out

    def _transform_device(self, arrays: List[Optional[np.ndarray]], valid: List[int], out: np.ndarray,
                          origins: List[str]) -> set:
        """Device execution of the stage list (K19 fused when it applies, else K20 stage kernels over
        uniform-shape batches). Returns the row indices it produced.

        Two-slot pipeline per batch: the host fills pinned input slot k % 2 while the device runs batch k - 1
        (H2D, kernels, D2H into pinned output slot), and the rows of batch k - 1 are built while batch k runs
        on the device; a slot is refilled only after its event (batch k - 2's D2H) has completed. The pinned
        slots come from torch's caching host allocator, so repeated calls reuse them."""
        import torch

        done = set()
        bs = max(1, self.getBatchSize())
        to_tensor = self.getToTensor()
        float_tensor = to_tensor and self.getTensorElementType().lower() == "float"
        fused = to_tensor and self._fused_plan([arrays[i].shape for i in valid]) is not None
        if fused:
            def launch_fused(idx, slot):
                return self.device_tensors([arrays[i] for i in idx])

            self._pipeline(valid, bs, launch_fused, None, lambda host, idx: self._emit_float(host, idx, out, done),
                           out, done)
            return done
        groups: Dict[tuple, List[int]] = {}
        for i in valid:
            groups.setdefault(arrays[i].shape, []).append(i)

        def emit(host, idx):
            if float_tensor:  # one bulk copy out of the reused pinned slot; the rows are views of it
                host = _bulk_copy(host, len(idx))
            elif not to_tensor:  # image rows: their data bytes filled in parallel
                rows = _image_rows(host, len(idx), [origins[i] for i in idx])
                for j, i in enumerate(idx):
                    out[i] = rows[j]
                    done.add(i)
                return
            for j, i in enumerate(idx):
                a = host[j]
                out[i] = a if float_tensor else self._finish_host(a)
                done.add(i)

        for shape, members in groups.items():
            if len(shape) != 3:
                continue
            nb = min(bs, len(members))
            ins = [torch.empty((nb,) + tuple(shape), dtype=torch.uint8, pin_memory=True) for _ in range(2)]

            def launch(idx, slot, ins=ins):
                sv = ins[slot].numpy()
                _gather_images(sv, [arrays[i] for i in idx])
                x = self.run_stages_device(ins[slot][:len(idx)])
                if x is None:
                    return None
                return self.tensors_from_device_images(x) if float_tensor else x

            if not self._pipeline(members, bs, launch, ins, emit, out, done):
                break
        return done

    @staticmethod
    def _pipeline(members, bs, launch, ins, emit, out, done) -> bool:
        """Batches of `members` through launch(idx, slot) -> device result (None: not on the device), D2H into
        pinned output slot (slot = batch % 2), emit(host, idx) one batch behind. False if a launch declined."""
        import torch

        outs = [None, None]
        ev = [None, None]
        pending = None

        def finish(slot, idx):
            ev[slot].synchronize()
            emit(outs[slot].numpy(), idx)

        ok = True
        for k, s in enumerate(range(0, len(members), bs)):
            slot = k & 1
            idx = members[s:s + bs]
            if ev[slot] is not None:
                ev[slot].synchronize()  # batch k - 2 left both slots (its rows were built at step k - 1)
            res = launch(idx, slot)
            if res is None:
                ok = False
                break
            shp = (min(bs, len(members)),) + tuple(res.shape[1:])
            if outs[slot] is None or tuple(outs[slot].shape) != shp or outs[slot].dtype != res.dtype:
                outs[slot] = torch.empty(shp, dtype=res.dtype, pin_memory=True)
            outs[slot][:len(idx)].copy_(res, non_blocking=True)
            ev[slot] = torch.cuda.Event()
            ev[slot].record()
            if pending is not None:
                finish(*pending)
            pending = (slot, idx)
        if pending is not None:
            finish(*pending)
        return ok

    def _emit_float(self, host, idx, out, done) -> None:
        fresh = _bulk_copy(host, len(idx))  # the pinned slot is reused by the batch after next
        for j, i in enumerate(idx):
            out[i] = fresh[j]
            done.add(i)

    def _finish_host(self, a: np.ndarray):
        """toTensor of one processed image on the host (tensorElementType double: the reference's fp64)."""
        cmap = channel_map(a.shape[2], self.getTensorChannelOrder(), self.getAutoConvertToColor())
        mean, std, scale = self._norm_params(len(cmap))
        if self.getTensorElementType().lower() == "double":
            src = a[:, :, cmap].astype(np.float64).transpose(2, 0, 1)
            return (src * scale - np.asarray(mean)[:, None, None]) / np.asarray(std)[:, None, None]
        return _img().to_tensor(np.ascontiguousarray(a), cmap, scale, mean, std)

    def process_host(self, a: np.ndarray):
        for st in self.getStages() or []:
            a = apply_stage(st, a)
        if not self.getToTensor():
            return a
        cmap = channel_map(a.shape[2], self.getTensorChannelOrder(), self.getAutoConvertToColor())
        mean, std, scale = self._norm_params(len(cmap))
        t = _img().to_tensor(np.ascontiguousarray(a), cmap, scale, mean, std)
        if self.getTensorElementType().lower() == "double":
            # the reference normalises in float64: recompute exactly
            src = a[:, :, cmap].astype(np.float64).transpose(2, 0, 1)
            return (src * scale - np.asarray(mean)[:, None, None]) / np.asarray(std)[:, None, None]
        return t

    def decode_column(self, df: DataFrame) -> List[Optional[np.ndarray]]:
        col = df[self.getInputCol()].tolist()
        ign = self.getIgnoreDecodingErrors()
        if len(col) > 8 and any(isinstance(v, (bytes, bytearray)) for v in col[:8]):
            with ThreadPoolExecutor(max_workers=8) as ex:
                return list(ex.map(lambda v: to_array(v, ign), col))
        return [to_array(v, ign) for v in col]

    def _transform(self, df: DataFrame) -> DataFrame:
        arrays = self.decode_column(df)
        n = len(arrays)
        out = np.empty(n, dtype=object)
        valid = [i for i, a in enumerate(arrays) if a is not None]
        col = df[self.getInputCol()]
        origins = [(v.get("origin", "") if isinstance(v, dict) else "") for v in (col.tolist() if valid else [])]
        done = set()
        if valid and _gpu_ok(self.getDeviceType()):
            done = self._transform_device(arrays, valid, out, origins)
        for i in valid:
            if i in done:
                continue
            r = self.process_host(arrays[i])
            out[i] = r if self.getToTensor() else make_image_row(r, origins[i])
        return df.withColumn(self.getOutputCol(), out)


class ImageSetAugmenter(Transformer, HasInputCol, HasOutputCol):
    flipLeftRight = Param("Symmetric Left-Right", True, T.toBoolean)
    flipUpDown = Param("Symmetric Up-Down", False, T.toBoolean)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(inputCol="image", outputCol=self.uid + "_output")

    def _transform(self, df: DataFrame) -> DataFrame:
        base = df.withColumn(self.getOutputCol(), df[self.getInputCol()])
        parts = [base]
        for enabled, code in ((self.getFlipLeftRight(), 1), (self.getFlipUpDown(), 0)):
            if enabled:
                t = ImageTransformer(inputCol=self.getInputCol(), outputCol=self.getOutputCol()).flip(code)
                parts.append(t.transform(df))
        out = parts[0]
        for p in parts[1:]:
            out = out.union(p)
        return out


def unroll(row) -> np.ndarray:
    """Image row -> CHW float vector. Like the reference (UnrollImage.scala:31-51)
    a 0 byte unrolls to 256.0 (its signed-byte conversion maps b <= 0 to b + 256)."""
    a = row_to_array(row).astype(np.float64)
    v = a.transpose(2, 0, 1).reshape(-1)
    return np.where(v > 0, v, v + 256.0)


def roll(values, origin: str, height: int, width: int, n_channels: int, mode: int) -> dict:
    v = np.clip(np.rint(np.asarray(values, dtype=np.float64)), 0, 255).astype(np.uint8)
    a = v.reshape(3, height, width).transpose(1, 2, 0)
    row = make_image_row(a, origin)
    row["nChannels"], row["mode"] = n_channels, mode
    return row


class UnrollImage(Transformer, HasInputCol, HasOutputCol):
    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(inputCol="image", outputCol=self.uid + "_output")

    def _transform(self, df: DataFrame) -> DataFrame:
        col = df[self.getInputCol()]
        out = np.empty(len(col), dtype=object)
        for i, r in enumerate(col.tolist()):
            out[i] = None if r is None else DenseVector(unroll(r))
        return df.withColumn(self.getOutputCol(), out)


class UnrollBinaryImage(Transformer, HasInputCol, HasOutputCol):
    """Encoded bytes -> unrolled vector, optionally resized (UnrollImage.scala:195-250)."""

    width = Param("the width of the image", None, T.toInt)
    height = Param("the height of the image", None, T.toInt)
    nChannels = Param("the number of channels of the target image", None, T.toInt)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(inputCol="image", outputCol=self.uid + "_output")

    def _transform(self, df: DataFrame) -> DataFrame:
        col = df[self.getInputCol()]
        out = np.empty(len(col), dtype=object)
        for i, b in enumerate(col.tolist()):
            if b is None:
                out[i] = None
                continue
            a = to_array(b, ignore_errors=True)
            if a is None:
                out[i] = None
                continue
            if self.getHeight() and self.getWidth():
                a = apply_stage({STAGE_NAME: "resize", "height": self.getHeight(), "width": self.getWidth()}, a)
            nc = self.getNChannels()
            if nc == 1 and a.shape[2] >= 3:
                a = _img().cvt_color(np.ascontiguousarray(a[:, :, :3]), 6)[:, :, None]
            elif nc == 3 and a.shape[2] == 1:
                a = np.repeat(a, 3, axis=2)
            elif nc == 3 and a.shape[2] == 4:
                a = np.ascontiguousarray(a[:, :, :3])
            out[i] = DenseVector(unroll({"height": a.shape[0], "width": a.shape[1], "nChannels": a.shape[2],
                                         "data": a.tobytes()}))
        return df.withColumn(self.getOutputCol(), out)


class ResizeImageTransformer(Transformer, HasInputCol, HasOutputCol):
    """Resize (and optionally change channels) of image rows (core/.../image/ResizeImageTransformer.scala)."""

    width = Param("the width of the image", None, T.toInt)
    height = Param("the height of the image", None, T.toInt)
    nChannels = Param("the number of channels of the target image", None, T.toInt)

    def _transform(self, df: DataFrame) -> DataFrame:
        col = df[self.getInputCol()]
        out = np.empty(len(col), dtype=object)
        for i, r in enumerate(col.tolist()):
            if r is None:
                out[i] = None
                continue
            a = to_array(r)
            a = apply_stage({STAGE_NAME: "resize", "height": self.getHeight(), "width": self.getWidth()}, a)
            nc = self.getNChannels()
            if nc == 1 and a.shape[2] >= 3:
                a = _img().cvt_color(np.ascontiguousarray(a[:, :, :3]), 6)[:, :, None]
            out[i] = make_image_row(a, r.get("origin", "") if isinstance(r, dict) else "")
        return df.withColumn(self.getOutputCol(), out)
