"""Binary file IO (reference: core/.../io/binary/BinaryFileFormat.scala:111-250,
BinaryFileReader.scala; Python io/binary/BinaryFileReader.py).

``read_binary_files`` returns a DataFrame(path, bytes). With ``inspectZip``
zip archives are expanded into one row per member (path ``archive.zip/member``);
``sampleRatio`` keeps a seeded Bernoulli subsample of files."""
from __future__ import annotations

import io
import os
import zipfile
from typing import Callable, List, Optional

import numpy as np

from ..core.dataframe import DataFrame

BinaryFileFields = ["path", "bytes"]


def _list_files(path: str, recursive: bool, path_filter: Optional[Callable[[str], bool]]) -> List[str]:
    if os.path.isfile(path):
        files = [path]
    else:
        files = []
        for root, dirs, names in os.walk(path):
            dirs.sort()
            files.extend(os.path.join(root, f) for f in sorted(names))
            if not recursive:
                break
    files = sorted(files)
    return [f for f in files if path_filter is None or path_filter(f)]


def read_binary_files(path: str, recursive: bool = False, sampleRatio: float = 1.0,  # noqa: N803
                      inspectZip: bool = True, seed: int = 0, num_partitions: int = 1,  # noqa: N803
                      path_filter: Optional[Callable[[str], bool]] = None) -> DataFrame:
    if not 0.0 < sampleRatio <= 1.0:
        raise ValueError("sampleRatio must be in (0, 1]")
    rng = np.random.default_rng(seed)
    paths, blobs = [], []

    def keep() -> bool:
        return sampleRatio >= 1.0 or rng.random() < sampleRatio

    for f in _list_files(path, recursive, path_filter):
        if inspectZip and f.lower().endswith(".zip"):
            with zipfile.ZipFile(f) as z:
                for info in sorted(z.infolist(), key=lambda i: i.filename):
                    if info.is_dir() or not keep():
                        continue
                    paths.append(f + "/" + info.filename)
                    blobs.append(z.read(info))
            continue
        if not keep():
            continue
        with open(f, "rb") as fh:
            paths.append(f)
            blobs.append(fh.read())
    pcol = np.empty(len(paths), dtype=object)
    bcol = np.empty(len(paths), dtype=object)
    for i, (p, b) in enumerate(zip(paths, blobs)):
        pcol[i], bcol[i] = p, b
    return DataFrame({"path": pcol, "bytes": bcol}, num_partitions=num_partitions)


def write_binary_files(df: DataFrame, directory: str, path_col: str = "path", bytes_col: str = "bytes") -> List[str]:
    """Write each row's bytes to ``directory/basename(path)``."""
    os.makedirs(directory, exist_ok=True)
    out = []
    for p, b in zip(df[path_col].tolist(), df[bytes_col].tolist()):
        dst = os.path.join(directory, os.path.basename(str(p)))
        with open(dst, "wb") as fh:
            fh.write(b)
        out.append(dst)
    return out


def zip_bytes(members: dict) -> bytes:
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        for name, data in members.items():
            z.writestr(name, data)
    return buf.getvalue()


__all__ = ["read_binary_files", "write_binary_files", "zip_bytes", "BinaryFileFields"]
