"""Local model repository (reference: core/src/main/python/synapse/ml/downloader/
ModelDownloader.py:15-169 and the Scala ModelDownloader, which fetch CNTK/ONNX
zoo models from a blob server).

There is no network, so the "remote" is any directory (or file:// URL) that
holds a ``MANIFEST`` (JSON lines of ModelSchema) plus the model files; models
are copied into ``localPath`` and verified by sha256 like the reference."""
from __future__ import annotations

import hashlib
import json
import os
import shutil
from dataclasses import asdict, dataclass, field
from typing import Iterator, List, Optional

DEFAULT_URL = "file:///nonexistent-offline-model-server/"


@dataclass
class ModelSchema:
    name: str
    dataset: str
    modelType: str  # noqa: N815
    uri: str
    hash: str
    size: int
    inputNode: int = 0  # noqa: N815
    numLayers: int = 0  # noqa: N815
    layerNames: List[str] = field(default_factory=list)  # noqa: N815

    def __repr__(self):
        return f"ModelSchema<name: {self.name}, dataset: {self.dataset}, loc: {self.uri}>"

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @staticmethod
    def from_json(s: str) -> "ModelSchema":
        return ModelSchema(**json.loads(s))


def _path_of(url: str) -> str:
    return url[len("file://"):] if url.startswith("file://") else url


def sha256_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


class ModelDownloader:
    def __init__(self, sparkSession=None, localPath: str = ".", serverURL: str = DEFAULT_URL):  # noqa: N803
        self.localPath = localPath
        self.serverURL = serverURL
        os.makedirs(localPath, exist_ok=True)

    @staticmethod
    def _manifest(root: str) -> List[ModelSchema]:
        p = os.path.join(root, "MANIFEST")
        if not os.path.exists(p):
            return []
        with open(p) as f:
            return [ModelSchema.from_json(line) for line in f if line.strip()]

    def localModels(self) -> Iterator[ModelSchema]:  # noqa: N802
        return iter(self._manifest(self.localPath))

    def remoteModels(self) -> Iterator[ModelSchema]:  # noqa: N802
        return iter(self._manifest(_path_of(self.serverURL)))

    def downloadModel(self, model: ModelSchema) -> ModelSchema:  # noqa: N802
        src = _path_of(model.uri) if os.path.isabs(_path_of(model.uri)) else \
            os.path.join(_path_of(self.serverURL), _path_of(model.uri))
        dst = os.path.join(self.localPath, os.path.basename(src))
        if not (os.path.exists(dst) and sha256_file(dst) == model.hash):
            shutil.copyfile(src, dst)
        if sha256_file(dst) != model.hash:
            os.remove(dst)
            raise IOError(f"hash mismatch for {model.name}")
        local = ModelSchema(**{**asdict(model), "uri": "file://" + os.path.abspath(dst)})
        known = [m for m in self._manifest(self.localPath) if m.name != model.name]
        with open(os.path.join(self.localPath, "MANIFEST"), "w") as f:
            for m in known + [local]:
                f.write(m.to_json() + "\n")
        return local

    def downloadByName(self, name: str) -> ModelSchema:  # noqa: N802
        for m in self.remoteModels():
            if m.name == name:
                return self.downloadModel(m)
        raise KeyError(f"no model named {name} at {self.serverURL}")

    def downloadModels(self, models: Optional[List[ModelSchema]] = None) -> List[ModelSchema]:  # noqa: N802
        return [self.downloadModel(m) for m in (models if models is not None else list(self.remoteModels()))]


__all__ = ["ModelDownloader", "ModelSchema", "sha256_file"]
