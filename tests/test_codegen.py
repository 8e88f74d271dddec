"""R binding generator (reference CORE/codegen/RCodegen.scala + generated testthat suites).
No R interpreter exists in this image, so the test checks what R would execute: every generated
constructor imports an existing module/class, passes only declared params to setParams, and the
sources are lexically balanced; the exported set covers every stage."""
import importlib
import re

from synapseml_amd.codegen import all_stages, generate_r, r_literal, snake


def _strip_strings(src):
    return re.sub(r'"(\\.|[^"\\])*"', '""', "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#")))


def test_r_package_generation(tmp_path):
    out = tmp_path / "pkg"
    exported = generate_r(str(out))
    stages = all_stages()
    assert len(exported) == len(stages) + 6 and len(set(exported)) == len(exported)
    ns = (out / "NAMESPACE").read_text()
    assert all(f"export({e})" in ns for e in exported)
    n_checked = 0
    for rfile in (out / "R").glob("*.R"):
        src = rfile.read_text()
        code = _strip_strings(src)
        for o, c in ("()", "{}", "[]"):
            assert code.count(o) == code.count(c), (rfile.name, o)
        for m in re.finditer(r'(sml_\w+) <- function\((.*?)\) \{\n  mod <- reticulate::import\("([\w.]+)".*?\n'
                             r'  stage <- .*?mod\$(\w+)\(\)', src, re.S):
            fname, sig, module, cls_name = m.groups()
            cls = getattr(importlib.import_module(module), cls_name)
            assert fname == "sml_" + snake(cls_name)
            params = [a.split(" = ")[0] for a in sig.split(", ")][:-1]
            assert set(params) == set(getattr(cls, "_params_decl", {}))
            n_checked += 1
    assert n_checked == len(stages)
    assert "sml_light_gbm_classifier" in exported and "sml_vowpal_wabbit_classifier" in exported


def test_r_literals_and_names():
    assert r_literal(True) == "TRUE" and r_literal(3) == "3L" and r_literal(0.5) == "0.5"
    assert r_literal('a"b') == '"a\\"b"' and r_literal([1, "x"]) == 'list(1L, "x")' and r_literal(None) == "NULL"
    assert r_literal(object()) is None
    assert snake("LightGBMClassifier") == "light_gbm_classifier" and snake("TextSHAP") == "text_shap"


def _c_api():
    import os

    from synapseml_amd.codegen import load_c_api, native_library_path

    if not os.path.exists(native_library_path()):
        import pytest

        pytest.skip("libsml_gbdt.so not built")
    return load_c_api()


def test_native_c_api_trains_and_predicts_like_the_python_engine():
    """The engine's C ABI (libsml_gbdt.so), driven through ctypes with the signature table the .NET binding
    is generated from: train / eval / predict / save / reload, equal to the pybind engine on the same data."""
    import ctypes as C

    import numpy as np

    from synapseml_amd.ops import native

    lib = _c_api()
    rng = np.random.default_rng(0)
    X = rng.standard_normal((3000, 6)).astype(np.float32)
    y = (X[:, 0] + X[:, 1] * X[:, 2] > 0).astype(np.float32)
    params = b"objective=binary num_leaves=15 metric=auc device_type=cpu"
    ds = C.c_void_p()
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    assert lib.SML_DatasetCreateFromMat(X.ctypes.data_as(C.c_void_p), 0, 3000, 6, params, fp(y), C.byref(ds)) == 0
    n = C.c_int32()
    assert lib.SML_DatasetGetNumData(ds, C.byref(n)) == 0 and n.value == 3000
    bst = C.c_void_p()
    assert lib.SML_BoosterCreate(ds, params, C.byref(bst)) == 0
    fin = C.c_int()
    for _ in range(10):
        assert lib.SML_BoosterUpdateOneIter(bst, C.byref(fin)) == 0
    it = C.c_int()
    assert lib.SML_BoosterGetCurrentIteration(bst, C.byref(it)) == 0 and it.value == 10
    ne = C.c_int()
    assert lib.SML_BoosterGetEval(bst, 0, 0, C.byref(ne), None) == 0 and ne.value == 1
    ev = (C.c_double * ne.value)()
    ev[0] = -7.0
    # a buffer too small for the metric list is left untouched (only the count is reported)
    assert lib.SML_BoosterGetEval(bst, 0, 0, C.byref(ne), ev) == 0 and ne.value == 1 and ev[0] == -7.0
    assert lib.SML_BoosterGetEval(bst, 0, ne.value, C.byref(ne), ev) == 0 and 0.9 < ev[0] <= 1.0
    ln = C.c_int64()
    assert lib.SML_BoosterPredictForMat(bst, X.ctypes.data_as(C.c_void_p), 0, 3000, 6, 1, 0, -1, C.byref(ln), None) == 0
    out = np.zeros(ln.value)
    assert lib.SML_BoosterPredictForMat(bst, X.ctypes.data_as(C.c_void_p), 0, 3000, 6, 1, 0, -1, C.byref(ln),
                                        out.ctypes.data_as(C.POINTER(C.c_double))) == 0
    need = C.c_int64()
    assert lib.SML_BoosterSaveModelToString(bst, 0, -1, 0, C.byref(need), None) == 0
    buf = C.create_string_buffer(need.value)
    assert lib.SML_BoosterSaveModelToString(bst, 0, -1, need.value, C.byref(need), buf) == 0
    model = buf.value.decode()
    # the same model through the Python engine: identical predictions
    pb = native.gbdt().Booster.from_model_string(model)
    np.testing.assert_allclose(pb.predict(X.astype(np.float64), 1, 0, -1)[:, 0], out, rtol=1e-12, atol=1e-12)
    b2 = C.c_void_p()
    assert lib.SML_BoosterLoadModelFromString(model.encode(), C.byref(b2)) == 0
    # errors come back as -1 + a message, never a crash
    bad = C.c_void_p()
    assert lib.SML_BoosterLoadModelFromString(b"not a model", C.byref(bad)) == -1
    assert lib.SML_GetLastError()
    for h, f in ((b2, lib.SML_BoosterFree), (bst, lib.SML_BoosterFree), (ds, lib.SML_DatasetFree)):
        assert f(h) == 0


def test_dotnet_binding_matches_the_c_abi(tmp_path):
    """Generated C#: one DllImport per C ABI entry with the table's arity, each an exported symbol of the
    built library (resolved through the same ctypes loader the previous test executes)."""
    import re

    from synapseml_amd.codegen import C_API, generate_dotnet

    path = generate_dotnet(str(tmp_path))
    src = open(path).read()
    code = _strip_strings(src)
    for o, c in ("()", "{}", "[]"):
        assert code.count(o) == code.count(c), o
    decls = dict(re.findall(r"internal static extern int (SML_\w+)\((.*?)\);", src))
    assert set(decls) == {n for n, _ in C_API}
    for name, args in C_API:
        assert len([p for p in decls[name].split(",") if p.strip()]) == len(args), name
    lib = _c_api()
    for name, _ in C_API:
        assert getattr(lib, name) is not None
    assert "class GbdtBooster : IDisposable" in src and "class GbdtDataset : IDisposable" in src
