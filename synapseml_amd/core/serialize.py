"""Stage persistence in the SparkML directory layout.

``<path>/metadata/part-00000`` holds one JSON line with ``class``,
``timestamp``, ``sparkVersion``, ``uid``, ``paramMap``, ``defaultParamMap`` and
``complexParamLocs``; every non-JSON ("complex") param is written under
``<path>/complexParams/<name>`` by type, as the reference's
ComplexParamsSerializer does (core/.../org/apache/spark/ml/
ComplexParamsSerializer.scala:35-183, Serializer.scala:41-47):

* nested stages  -> a nested stage directory
* DataFrames     -> ``data.npz`` (columns) + ``schema.json``
* ``bytes``      -> a Java-serialization-compatible ``byte[]`` stream
* everything else JSON-able -> ``value.json``; otherwise pickle of OUR OWN
  objects only (files this framework wrote).
"""
from __future__ import annotations

import importlib
import io
import json
import os
import pickle
import shutil
import struct
import time
from typing import Any

import numpy as np

SPARK_VERSION = "3.4.1"

# Java serialization of a byte[]: STREAM_MAGIC, STREAM_VERSION, TC_ARRAY,
# TC_CLASSDESC "[B" serialVersionUID 0xACF317F8060854E0, SC_SERIALIZABLE,
# 0 fields, TC_ENDBLOCKDATA, TC_NULL superclass, int32 length, bytes.
_JAVA_BYTE_ARRAY_HEADER = bytes.fromhex("aced0005757200025b42acf317f8060854e0020000787000")[:-1]


def java_serialize_bytes(b: bytes) -> bytes:
    return _JAVA_BYTE_ARRAY_HEADER + struct.pack(">i", len(b)) + b


def java_deserialize_bytes(data: bytes) -> bytes:
    if not data.startswith(_JAVA_BYTE_ARRAY_HEADER):
        raise ValueError("not a Java-serialized byte[] stream")
    (n,) = struct.unpack(">i", data[len(_JAVA_BYTE_ARRAY_HEADER): len(_JAVA_BYTE_ARRAY_HEADER) + 4])
    off = len(_JAVA_BYTE_ARRAY_HEADER) + 4
    return data[off: off + n]


def _jsonable(v: Any) -> bool:
    try:
        json.dumps(v)
        return True
    except (TypeError, ValueError):
        return False


def _to_json_value(v: Any):
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, np.ndarray):
        return v.tolist()
    return v


def class_path(obj_or_cls) -> str:
    cls = obj_or_cls if isinstance(obj_or_cls, type) else type(obj_or_cls)
    return f"{cls.__module__}.{cls.__qualname__}"


def load_class(path: str):
    mod, _, name = path.rpartition(".")
    return getattr(importlib.import_module(mod), name)


def _write_complex(value: Any, d: str) -> str:
    os.makedirs(d, exist_ok=True)
    from .pipeline import PipelineStage
    from .dataframe import DataFrame

    if isinstance(value, PipelineStage):
        value.save(os.path.join(d, "stage"), overwrite=True)
        return "stage"
    if isinstance(value, (list, tuple)) and value and all(isinstance(v, PipelineStage) for v in value):
        for i, s in enumerate(value):
            s.save(os.path.join(d, f"stage_{i:04d}"), overwrite=True)
        with open(os.path.join(d, "count"), "w") as f:
            f.write(str(len(value)))
        return "stages"
    if isinstance(value, DataFrame):
        arrays, kinds = {}, {}
        for k, c in value._cols.items():
            if c.dtype == object:
                kinds[k] = "object"
                arrays[k] = np.frombuffer(pickle.dumps(c.tolist()), dtype=np.uint8)
            else:
                kinds[k] = "array"
                arrays[k] = c
        np.savez(os.path.join(d, "data.npz"), **arrays)
        with open(os.path.join(d, "schema.json"), "w") as f:
            json.dump({"kinds": kinds, "columns": value.columns, "meta": value._meta}, f)
        return "dataframe"
    if hasattr(value, "_sml_save") and hasattr(type(value), "_sml_load"):
        value._sml_save(d)
        return "custom:" + class_path(value)
    if isinstance(value, (bytes, bytearray)):
        with open(os.path.join(d, "data.bin"), "wb") as f:
            f.write(java_serialize_bytes(bytes(value)))
        return "bytes"
    if isinstance(value, np.ndarray):
        np.save(os.path.join(d, "array.npy"), value, allow_pickle=False)
        return "ndarray"
    if _jsonable(value):
        with open(os.path.join(d, "value.json"), "w") as f:
            json.dump(value, f)
        return "json"
    with open(os.path.join(d, "object.pkl"), "wb") as f:
        pickle.dump(value, f)
    return "pickle"


def _read_complex(d: str, kind: str) -> Any:
    from .pipeline import PipelineStage
    from .dataframe import DataFrame

    if kind == "stage":
        return PipelineStage.load(os.path.join(d, "stage"))
    if kind == "stages":
        with open(os.path.join(d, "count")) as f:
            n = int(f.read())
        return [PipelineStage.load(os.path.join(d, f"stage_{i:04d}")) for i in range(n)]
    if kind == "dataframe":
        with open(os.path.join(d, "schema.json")) as f:
            sch = json.load(f)
        z = np.load(os.path.join(d, "data.npz"), allow_pickle=False)
        cols = {}
        for k in sch["columns"]:
            if sch["kinds"][k] == "object":
                # our own writer produced this pickle (see _write_complex)
                lst = pickle.loads(z[k].tobytes())
                arr = np.empty(len(lst), dtype=object)
                for i, v in enumerate(lst):
                    arr[i] = v
                cols[k] = arr
            else:
                cols[k] = z[k]
        return DataFrame(cols, metadata=sch.get("meta"))
    if kind.startswith("custom:"):
        return load_class(kind[len("custom:"):])._sml_load(d)
    if kind == "bytes":
        with open(os.path.join(d, "data.bin"), "rb") as f:
            return java_deserialize_bytes(f.read())
    if kind == "ndarray":
        return np.load(os.path.join(d, "array.npy"), allow_pickle=False)
    if kind == "json":
        with open(os.path.join(d, "value.json")) as f:
            return json.load(f)
    with open(os.path.join(d, "object.pkl"), "rb") as f:
        return pickle.load(f)


def save_stage(stage, path: str, overwrite: bool = False) -> None:
    if os.path.exists(path):
        if not overwrite:
            raise FileExistsError(f"{path} already exists; use overwrite=True")
        shutil.rmtree(path)
    os.makedirs(os.path.join(path, "metadata"))
    param_map, default_map, locs = {}, {}, {}
    decl = stage._params_decl
    for k, v in stage._paramMap.items():
        if decl[k].complex or not _jsonable(_to_json_value(v)):
            if v is not None:
                locs[k] = _write_complex(v, os.path.join(path, "complexParams", k))
        else:
            param_map[k] = _to_json_value(v)
    default_locs = {}
    for k, v in stage._defaultParamMap.items():
        if k in decl and not decl[k].complex and _jsonable(_to_json_value(v)):
            default_map[k] = _to_json_value(v)
        elif k in decl and v is not None and k not in stage._paramMap:
            # complex defaults built by the constructor (e.g. ImageFeaturizer's inner ONNXModel): a load
            # does not run the constructor, so they are written like complex params
            default_locs[k] = _write_complex(v, os.path.join(path, "complexDefaultParams", k))
    meta = {
        "class": class_path(stage),
        "timestamp": int(time.time() * 1000),
        "sparkVersion": SPARK_VERSION,
        "uid": stage.uid,
        "paramMap": param_map,
        "defaultParamMap": default_map,
    }
    if locs:
        meta["complexParamLocs"] = {k: f"complexParams/{k}#{kind}" for k, kind in locs.items()}
    if default_locs:
        meta["complexDefaultParamLocs"] = {k: f"complexDefaultParams/{k}#{kind}" for k, kind in default_locs.items()}
    with open(os.path.join(path, "metadata", "part-00000"), "w") as f:
        f.write(json.dumps(meta) + "\n")
    open(os.path.join(path, "metadata", "_SUCCESS"), "w").close()
    stage._save_extra(path)


def load_stage(path: str):
    with open(os.path.join(path, "metadata", "part-00000")) as f:
        meta = json.loads(f.readline())
    cls = load_class(meta["class"])
    obj = cls.__new__(cls)
    from .params import Params

    Params.__init__(obj, uid=meta["uid"])
    obj._init_state()
    for k, v in meta.get("defaultParamMap", {}).items():
        if k in obj._params_decl:
            obj._defaultParamMap[k] = v
    for k, v in meta.get("paramMap", {}).items():
        if k in obj._params_decl:
            obj._paramMap[k] = v
    for k, loc in meta.get("complexParamLocs", {}).items():
        rel, _, kind = loc.partition("#")
        obj._paramMap[k] = _read_complex(os.path.join(path, rel), kind)
    for k, loc in meta.get("complexDefaultParamLocs", {}).items():
        rel, _, kind = loc.partition("#")
        if k in obj._params_decl:
            obj._defaultParamMap[k] = _read_complex(os.path.join(path, rel), kind)
    obj._load_extra(path)
    return obj
