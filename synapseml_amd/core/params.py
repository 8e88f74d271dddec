"""Typed parameters with defaults, generated getters/setters and param maps.

Mirrors SparkML ``Params`` as used throughout the reference:
every stage exposes ``setX``/``getX`` per param, keyword constructors,
``explainParams``, ``copy(extra)`` and a JSON-serialisable param map that the
persistence layer writes to ``metadata/part-00000``.
"""
from __future__ import annotations

import copy as _copy
import uuid
from typing import Any, Callable, Dict, Optional


class _NoDefault:
    def __repr__(self) -> str:
        return "<no default>"


NO_DEFAULT = _NoDefault()


class TypeConverters:
    @staticmethod
    def identity(v):
        return v

    @staticmethod
    def toInt(v):  # noqa: N802
        if isinstance(v, bool):
            raise TypeError("expected int, got bool")
        return int(v)

    @staticmethod
    def toFloat(v):  # noqa: N802
        return float(v)

    @staticmethod
    def toBoolean(v):  # noqa: N802
        if isinstance(v, str):
            return v.lower() in ("true", "1", "yes")
        return bool(v)

    @staticmethod
    def toString(v):  # noqa: N802
        return str(v)

    @staticmethod
    def toListInt(v):  # noqa: N802
        return [int(x) for x in v]

    @staticmethod
    def toListFloat(v):  # noqa: N802
        return [float(x) for x in v]

    @staticmethod
    def toListString(v):  # noqa: N802
        return [str(x) for x in v]

    @staticmethod
    def toDictStrStr(v):  # noqa: N802
        return {str(k): str(x) for k, x in dict(v).items()}


class Param:
    """A parameter declared as a class attribute of a :class:`Params` subclass.

    ``complex=True`` marks params that are not JSON values (models, bytes,
    DataFrames, functions): they are persisted under ``complexParams/<name>``
    like the reference's ComplexParam (core/.../serialize/ComplexParam.scala).
    """

    def __init__(self, doc: str = "", default: Any = NO_DEFAULT, converter: Optional[Callable] = None,
                 name: Optional[str] = None, complex: bool = False):
        self.name = name
        self.doc = doc
        self.default = default
        self.converter = converter or TypeConverters.identity
        self.complex = complex

    def __set_name__(self, owner, name):
        if self.name is None:
            self.name = name

    def __repr__(self) -> str:
        return f"Param({self.name})"


def _cap(name: str) -> str:
    return name[0].upper() + name[1:]


class ParamsMeta(type):
    def __new__(mcs, clsname, bases, ns):
        cls = super().__new__(mcs, clsname, bases, ns)
        params: Dict[str, Param] = {}
        for b in reversed(cls.__mro__[1:]):
            params.update(getattr(b, "_params_decl", {}))
        for k, v in ns.items():
            if isinstance(v, Param):
                if v.name is None:
                    v.name = k
                params[v.name] = v
        cls._params_decl = params
        for pname in params:
            getter, setter = "get" + _cap(pname), "set" + _cap(pname)
            if not hasattr(cls, getter):
                setattr(cls, getter, _make_getter(pname))
            if not hasattr(cls, setter):
                setattr(cls, setter, _make_setter(pname))
        hook = getattr(cls, "_params_hook", None)
        if hook is not None:
            hook()
        return cls


def _make_getter(name):
    def g(self):
        return self.getOrDefault(name)

    g.__name__ = "get" + _cap(name)
    return g


def _make_setter(name):
    def s(self, value):
        return self.set(name, value)

    s.__name__ = "set" + _cap(name)
    return s


class Params(metaclass=ParamsMeta):
    _params_decl: Dict[str, Param] = {}

    def __init__(self, uid: Optional[str] = None, **kwargs):
        self.uid = uid or f"{type(self).__name__}_{uuid.uuid4().hex[:12]}"
        self._paramMap: Dict[str, Any] = {}
        self._defaultParamMap: Dict[str, Any] = {
            k: p.default for k, p in self._params_decl.items() if p.default is not NO_DEFAULT
        }
        self.setParams(**kwargs)

    # ---------------------------------------------------------------- access
    @property
    def params(self):
        return [self._params_decl[k] for k in sorted(self._params_decl)]

    def hasParam(self, name: str) -> bool:  # noqa: N802
        return name in self._params_decl

    def getParam(self, name: str) -> Param:  # noqa: N802
        return self._params_decl[name]

    def setParams(self, **kwargs):  # noqa: N802
        for k, v in kwargs.items():
            if v is None and k not in self._paramMap and self._defaultParamMap.get(k) is None:
                continue
            self.set(k, v)
        return self

    def set(self, name: str, value: Any):
        if name not in self._params_decl:
            raise AttributeError(f"{type(self).__name__} has no param {name!r}")
        p = self._params_decl[name]
        self._paramMap[name] = p.converter(value) if value is not None else None
        return self

    def clear(self, name: str):
        self._paramMap.pop(name, None)
        return self

    def _setDefault(self, **kwargs):  # noqa: N802
        for k, v in kwargs.items():
            self._defaultParamMap[k] = v
        return self

    def isSet(self, name: str) -> bool:  # noqa: N802
        return name in self._paramMap

    def hasDefault(self, name: str) -> bool:  # noqa: N802
        return name in self._defaultParamMap

    def isDefined(self, name: str) -> bool:  # noqa: N802
        return self.isSet(name) or self.hasDefault(name)

    def getOrDefault(self, name: str):  # noqa: N802
        if name in self._paramMap:
            return self._paramMap[name]
        if name in self._defaultParamMap:
            return self._defaultParamMap[name]
        if name in self._params_decl:
            return None
        raise AttributeError(name)

    def getDefault(self, name: str):  # noqa: N802
        return self._defaultParamMap.get(name)

    def extractParamMap(self, extra: Optional[dict] = None) -> Dict[str, Any]:  # noqa: N802
        m = dict(self._defaultParamMap)
        m.update(self._paramMap)
        if extra:
            m.update(extra)
        return m

    def explainParam(self, name: str) -> str:  # noqa: N802
        p = self._params_decl[name]
        vals = []
        if self.hasDefault(name):
            vals.append(f"default: {self.getDefault(name)!r}")
        if self.isSet(name):
            vals.append(f"current: {self._paramMap[name]!r}")
        return f"{name}: {p.doc} ({', '.join(vals) if vals else 'undefined'})"

    def explainParams(self) -> str:  # noqa: N802
        return "\n".join(self.explainParam(k) for k in sorted(self._params_decl))

    def copy(self, extra: Optional[dict] = None):
        that = _copy.copy(self)
        that._paramMap = dict(self._paramMap)
        that._defaultParamMap = dict(self._defaultParamMap)
        if extra:
            for k, v in extra.items():
                that.set(k if isinstance(k, str) else k.name, v)
        return that

    def _copyValues(self, to: "Params", extra: Optional[dict] = None):  # noqa: N802
        for k, v in self.extractParamMap(extra).items():
            if to.hasParam(k) and (k in self._paramMap or (extra and k in extra)):
                to.set(k, v)
        return to

    def __repr__(self) -> str:
        return self.uid
