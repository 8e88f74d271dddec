"""Image rows (Spark ImageSchema layout: origin, height, width, nChannels,
mode, data — data is row-major BGR(A)/gray uint8) and decoding.

Reference: opencv/.../ImageTransformer.scala:285-330 (row2mat / decodeImage),
core/.../schema/ImageSchemaUtils.scala; mode codes CV_8UC1=0, CV_8UC3=16,
CV_8UC4=24. Decoding uses PIL (JPEG/PNG/BMP/...)."""
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
    """Encoded image bytes -> HWC uint8 in OpenCV order (BGR / BGRA / gray)."""
    from PIL import Image

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

    with Image.open(io.BytesIO(bytes(data))) as im:
        if im.mode == "RGB":
            return np.asarray(im), True
    return decode_bytes(data), False


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
