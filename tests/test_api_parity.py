"""Public methods of the reference's Python classes (every ``src/main/python`` class whose name this package
also defines) exist on the classes here - a guard against API drift. The reference tree is read only for
method names; JVM-bridge plumbing (java / spark conversions) has no counterpart."""
import ast
import importlib
import inspect
import os
import pkgutil

import pytest

REF = "/root/reference"
JVM_ONLY = {"fromJava", "toJava", "from_java", "to_java", "getJavaPackage", "to_java_params"}


def _ref_classes():
    out = {}
    for root, _, files in os.walk(REF):
        if "src/main/python" not in root:
            continue
        for f in files:
            if f.endswith(".py"):
                try:
                    tree = ast.parse(open(os.path.join(root, f)).read())
                except (SyntaxError, UnicodeDecodeError):
                    continue
                for node in tree.body:
                    if isinstance(node, ast.ClassDef):
                        out.setdefault(node.name, set()).update(
                            n.name for n in node.body if isinstance(n, ast.FunctionDef) and not n.name.startswith("_"))
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_reference_python_methods_present():
    import synapseml_amd

    ours = {}
    for m in pkgutil.walk_packages(synapseml_amd.__path__, "synapseml_amd."):
        try:
            mod = importlib.import_module(m.name)
        except Exception:  # noqa: BLE001 - optional GPU / platform modules
            continue
        for n, c in inspect.getmembers(mod, inspect.isclass):
            if c.__module__.startswith("synapseml_amd"):
                ours.setdefault(n, c)
    missing = {}
    for cname, methods in _ref_classes().items():
        if cname in ours:
            miss = sorted(m for m in methods - JVM_ONLY if not hasattr(ours[cname], m))
            if miss:
                missing[cname] = miss
    assert not missing, missing
