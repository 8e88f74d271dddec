"""Image rows (Spark ImageSchema layout: origin, height, width, nChannels,
mode, data — data is row-major BGR(A)/gray uint8) and decoding.

Reference: opencv/.../ImageTransformer.scala:285-330 (row2mat / decodeImage),
core/.../schema/ImageSchemaUtils.scala; mode codes CV_8UC1=0, CV_8UC3=16,
CV_8UC4=24. Baseline JPEGs decode natively (csrc/image/jpeg_decode.cpp, pixel-identical to
PIL's libjpeg), everything else (progressive JPEG, PNG, BMP, ...) through PIL."""
from __future__ import annotations

import io
import os
from typing import Iterable, List, Optional

import numpy as np

from ..core.dataframe import DataFrame

CV_8UC1, CV_8UC3, CV_8UC4 = 0, 16, 24
_MODE_OF = {1: CV_8UC1, 3: CV_8UC3, 4: CV_8UC4}
IMAGE_FIELDS = ("origin", "height", "width", "nChannels", "mode", "data")


def make_image_row(arr: np.ndarray, origin: str = "") -> dict:
    """HWC (or HW) uint8 array in OpenCV channel order -> image row."""
    a = np.ascontiguousarray(arr, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    h, w, c = a.shape
    if c not in _MODE_OF:
        raise ValueError(f"unsupported channel count {c}")
    return {"origin": origin, "height": int(h), "width": int(w), "nChannels": int(c), "mode": _MODE_OF[c],
            "data": a.tobytes()}


def row_to_array(row) -> np.ndarray:
    """image row -> HWC uint8 array (a view on the row's bytes)."""
    h, w, c = int(row["height"]), int(row["width"]), int(row["nChannels"])
    data = row["data"]
    a = np.frombuffer(bytes(data) if not isinstance(data, (bytes, bytearray, memoryview)) else data, dtype=np.uint8)
    if a.size != h * w * c:
        raise ValueError(f"image data has {a.size} bytes, expected {h * w * c}")
    return a.reshape(h, w, c)


def decode_bytes(data: bytes) -> np.ndarray:
    """Encoded image bytes -> HWC uint8 in OpenCV order (BGR / BGRA / gray). Baseline JPEGs go through
    the native decoder (same pixels as PIL, no GIL held), everything else through PIL."""
    from PIL import Image

    if bytes(data[:2]) == b"\xff\xd8":
        a = decode_jpeg_native(data)
        if a is not None:
            return np.ascontiguousarray(a[:, :, ::-1]) if a.shape[2] == 3 else a

    with Image.open(io.BytesIO(bytes(data))) as im:
        if im.mode in ("L", "1", "I;16", "I", "F"):
            a = np.asarray(im.convert("L"))
            return a[:, :, None]
        if im.mode in ("RGBA", "LA", "PA") or (im.mode == "P" and "transparency" in im.info):
            a = np.asarray(im.convert("RGBA"))
            return np.ascontiguousarray(a[:, :, [2, 1, 0, 3]])
        a = np.asarray(im.convert("RGB"))
        return np.ascontiguousarray(a[:, :, ::-1])


def decode_bytes_rgb(data: bytes):
    """Encoded bytes -> (HWC uint8, is_rgb). RGB images (every JPEG) come back in RGB order straight from the
    decoder - no convert() copy and no BGR flip; the fused device preprocess maps channels itself. Other
    modes fall back to decode_bytes (OpenCV order, is_rgb False)."""
    from PIL import Image

    if bytes(data[:2]) == b"\xff\xd8":
        a = decode_jpeg_native(data)
        if a is not None:
            return (a, True) if a.shape[2] == 3 else (a, False)
    with Image.open(io.BytesIO(bytes(data))) as im:
        if im.mode == "RGB":
            return np.asarray(im), True
    return decode_bytes(data), False


def decode_jpeg_native(data: bytes) -> Optional[np.ndarray]:
    """Baseline JPEG -> HWC uint8 (RGB, or gray as HxWx1) with the native decoder (csrc/image/jpeg_decode.cpp,
    pixel-identical to PIL's libjpeg decode), or None when the file is outside its scope (progressive,
    CMYK, ...), the extension is not built, or ``SML_NATIVE_JPEG=0`` (A/B against PIL)."""
    if os.environ.get("SML_NATIVE_JPEG", "1") == "0":
        return None
    try:
        from ..ops import native

        a = native.load("_image").jpeg_decode(bytes(data))
    except (ImportError, OSError):
        return None
    if a is None:
        return None
    return a if a.ndim == 3 else a[:, :, None]


def pack_decoded(values, ignore_errors: bool = False, threads: int = 8, pinned: bool = False):
    """Decode a batch of image values (encoded bytes, image rows or arrays) into ONE contiguous uint8 buffer.

    JPEGs in the native decoder's scope are decoded by a pool of native threads straight into the buffer
    (no per-image Python, no GIL, no intermediate array); everything else goes through PIL / the row
    readers and is copied in. With ``pinned`` the buffer is page-locked host memory, ready for an
    asynchronous H2D copy. Returns ``(buf, offsets, shapes, rgb, ok)``: image i is ``shapes[i]`` (h, w, c)
    at ``offsets[i]``; ``rgb[i]`` marks 3-channel images in RGB order (JPEG decodes) rather than OpenCV's
    BGR; ``ok[i]`` is False for an undecodable value (only with ``ignore_errors``; otherwise it raises).
    """
    n = len(values)
    shapes: List[Optional[tuple]] = [None] * n
    rgb = [False] * n
    arrays: List[Optional[np.ndarray]] = [None] * n
    jidx, jbytes = [], []
    for i, v in enumerate(values):
        if isinstance(v, (bytes, bytearray, memoryview)):
            jidx.append(i)
            jbytes.append(v if isinstance(v, bytes) else bytes(v))
    lib = None
    native_idx: List[int] = []
    if jbytes and os.environ.get("SML_NATIVE_JPEG", "1") != "0":
        try:
            from ..ops import native

            lib = native.load("_image")
        except (ImportError, OSError):
            lib = None
    if lib is not None:
        info = lib.jpeg_probe(jbytes)
        for k, i in enumerate(jidx):
            h, w, c, sup = (int(x) for x in info[k])
            if sup:
                shapes[i] = (h, w, c)
                rgb[i] = c == 3
                native_idx.append(i)
    native_set = set(native_idx)

    def fallback(i):
        v = values[i]
        try:
            if isinstance(v, (bytes, bytearray, memoryview)):
                a, r = decode_bytes_rgb(v)
            else:
                a, r = to_array(v, ignore_errors), False
        except Exception:
            if ignore_errors:
                return None, False
            raise
        if a is not None and a.ndim == 2:
            a = a[:, :, None]
        return a, r

    for i in range(n):
        if i not in native_set:
            arrays[i], rgb[i] = fallback(i)
            if arrays[i] is not None:
                shapes[i] = arrays[i].shape
    sizes = np.array([int(np.prod(sh)) if sh is not None else 0 for sh in shapes], np.int64)
    offsets = np.zeros(n, np.int64)
    if n:
        offsets[1:] = np.cumsum(sizes)[:-1]
    total = int(sizes.sum())
    if pinned:
        import torch

        buf = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=True)
        view, ptr = buf.numpy(), buf.data_ptr()
    else:
        buf = view = np.empty(max(total, 1), np.uint8)
        ptr = view.ctypes.data
    if native_idx:
        nb = [values[i] if isinstance(values[i], bytes) else bytes(values[i]) for i in native_idx]
        okn = lib.jpeg_decode_into(nb, ptr, max(total, 1), [int(offsets[i]) for i in native_idx],
                                   [int(sizes[i]) for i in native_idx], max(1, int(threads)))
        for k, i in enumerate(native_idx):
            if not okn[k]:  # corrupt / truncated: let PIL decide (it may recover or raise)
                a, r = fallback(i)
                if a is not None and a.shape != shapes[i]:
                    a = None
                arrays[i], rgb[i] = a, r
                if a is None:
                    shapes[i] = None
    for i in range(n):
        a = arrays[i]
        if a is not None:
            view[offsets[i]:offsets[i] + a.size] = np.ascontiguousarray(a).reshape(-1)
    ok = [sh is not None for sh in shapes]
    if not ignore_errors and not all(ok) and any(v is not None for v, o in zip(values, ok) if not o):
        raise ValueError("undecodable image in batch")
    return buf, offsets, shapes, rgb, ok


def encode_png(arr: np.ndarray) -> bytes:
    """HWC OpenCV-order array -> PNG bytes."""
    from PIL import Image

    a = np.asarray(arr, dtype=np.uint8)
    if a.ndim == 3 and a.shape[2] == 1:
        a = a[:, :, 0]
    if a.ndim == 3 and a.shape[2] == 3:
        a = a[:, :, ::-1]
    elif a.ndim == 3 and a.shape[2] == 4:
        a = a[:, :, [2, 1, 0, 3]]
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(a)).save(buf, format="PNG")
    return buf.getvalue()


def to_array(value, ignore_errors: bool = False) -> Optional[np.ndarray]:
    """Accept an image row (dict), encoded bytes, or an array."""
    try:
        if value is None:
            return None
        if isinstance(value, dict):
            return row_to_array(value)
        if isinstance(value, (bytes, bytearray, memoryview)):
            return decode_bytes(value)
        if isinstance(value, np.ndarray):
            return value if value.ndim == 3 else value[:, :, None]
        if hasattr(value, "asDict"):
            return row_to_array(value.asDict())
        raise TypeError(f"cannot interpret {type(value)} as an image")
    except Exception:
        if ignore_errors:
            return None
        raise


def read_images(path: str, recursive: bool = True, sample_ratio: float = 1.0, seed: int = 0,
                num_partitions: int = 1, drop_invalid: bool = True) -> DataFrame:
    """Directory of image files -> DataFrame with an ``image`` column (spark.read.image)."""
    files = _list_files(path, recursive)
    rng = np.random.default_rng(seed)
    rows = []
    for f in files:
        if sample_ratio < 1.0 and rng.random() > sample_ratio:
            continue
        with open(f, "rb") as fh:
            data = fh.read()
        try:
            rows.append(make_image_row(decode_bytes(data), origin=f))
        except Exception:
            if not drop_invalid:
                rows.append(None)
    col = np.empty(len(rows), dtype=object)
    for i, r in enumerate(rows):
        col[i] = r
    return DataFrame({"image": col}, num_partitions=num_partitions)


def read_binary_files(path: str, recursive: bool = True, num_partitions: int = 1) -> DataFrame:
    """Directory -> DataFrame(path, bytes) (BinaryFileFormat.scala:111-250)."""
    files = _list_files(path, recursive)
    data = np.empty(len(files), dtype=object)
    for i, f in enumerate(files):
        with open(f, "rb") as fh:
            data[i] = fh.read()
    return DataFrame({"path": np.array(files, dtype=object), "bytes": data}, num_partitions=num_partitions)


def _list_files(path: str, recursive: bool) -> List[str]:
    if os.path.isfile(path):
        return [path]
    out = []
    for root, dirs, files in os.walk(path):
        for f in sorted(files):
            out.append(os.path.join(root, f))
        if not recursive:
            break
    return sorted(out)


def images_column(arrays: Iterable[np.ndarray], origins: Optional[Iterable[str]] = None) -> np.ndarray:
    arrs = list(arrays)
    ors = list(origins) if origins is not None else [""] * len(arrs)
    col = np.empty(len(arrs), dtype=object)
    for i, (a, o) in enumerate(zip(arrs, ors)):
        col[i] = make_image_row(a, o)
    return col
