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
