"""Language-binding generator (reference: CORE/codegen/{CodeGen,Wrappable,RCodegen,PyCodegen}.scala and
CORE/param/RWrappableParam.scala - the reference generates Python/R/.NET wrappers from its Scala params).

Here every stage is already a Python class, so the Python "wrappers" are the classes themselves; what
this module generates is the R package: one constructor per stage (``sml_<snake_name>(...)``) that
imports the stage through reticulate, sets the non-NULL params, and returns the live Python object,
plus ``sml_fit`` / ``sml_transform`` / ``sml_save`` / ``sml_load`` and R <-> DataFrame conversion.
A testthat file per module constructs every stage (the reference's generated R tests do the same).

usage: ``python -m synapseml_amd.codegen --r-out build/R/synapsemlamd``"""
from __future__ import annotations

import argparse
import importlib
import inspect
import os
import pkgutil
import re
from typing import Dict, List, Optional, Tuple

R_PACKAGE = "synapsemlamd"


def all_stages() -> Dict[str, type]:
    """Every public PipelineStage class defined in the package, keyed by ``module.Class``."""
    import synapseml_amd
    from .core.pipeline import Estimator, Model, PipelineStage, Transformer

    base = {PipelineStage, Transformer, Estimator, Model}
    seen = {}
    for m in pkgutil.walk_packages(synapseml_amd.__path__, "synapseml_amd."):
        if m.name.split(".")[-1].startswith("_") or m.name.endswith(".codegen"):
            continue
        try:
            mod = importlib.import_module(m.name)
        except Exception:  # noqa: BLE001 - optional dependencies stay out of the bindings
            continue
        for name, obj in vars(mod).items():
            if inspect.isclass(obj) and issubclass(obj, PipelineStage) and obj not in base \
                    and not name.startswith("_") and obj.__module__ == mod.__name__:
                seen[f"{obj.__module__}.{name}"] = obj
    return dict(sorted(seen.items()))


def snake(name: str) -> str:
    """LightGBMClassifier -> light_gbm_classifier, TextSHAP -> text_shap (reference RCodegen naming)."""
    s = re.sub(r"([A-Z]+)([A-Z][a-z])", r"\1_\2", name)
    s = re.sub(r"([a-z0-9])([A-Z])", r"\1_\2", s)
    return s.lower()


def r_literal(v) -> Optional[str]:
    """An R literal for a Python default, or None when it has no faithful R spelling."""
    if v is None:
        return "NULL"
    if isinstance(v, bool):
        return "TRUE" if v else "FALSE"
    if isinstance(v, int):
        return f"{v}L" if abs(v) < 2 ** 31 else repr(float(v))
    if isinstance(v, float):
        if v != v:
            return "NaN"
        if v in (float("inf"), float("-inf")):
            return "Inf" if v > 0 else "-Inf"
        return repr(v)
    if isinstance(v, str):
        return '"' + v.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n") + '"'
    if isinstance(v, (list, tuple)):
        items = [r_literal(x) for x in v]
        if any(i is None for i in items):
            return None
        return "list(" + ", ".join(items) + ")"
    return None


def _r_doc(text: str) -> str:
    return " ".join((text or "").split()).replace("%", "\\%")[:300]


def r_function(path: str, cls: type) -> Tuple[str, str]:
    """(function name, R source) for one stage."""
    module, name = path.rsplit(".", 1)
    fname = "sml_" + snake(name)
    decl = getattr(cls, "_params_decl", {})
    pnames = sorted(decl)
    summary = _r_doc((inspect.getdoc(cls) or name).split("\n")[0])
    lines = [f"#' {name}", "#'", f"#' {summary}", "#'"]
    for p in pnames:
        d = decl[p].default
        dflt = "" if d is None or d.__class__.__name__ == "_NoDefault" else r_literal(d)
        extra = f" (default {dflt})" if dflt else ""
        lines.append(f"#' @param {p} {_r_doc(decl[p].doc) or p}{extra}")
    lines += ["#' @param uid optional stage uid", f"#' @return a \\code{{{path}}} Python object", "#' @export"]
    sig = ", ".join([f"{p} = NULL" for p in pnames] + ["uid = NULL"])
    lines.append(f"{fname} <- function({sig}) {{")
    lines.append(f'  mod <- reticulate::import("{module}", delay_load = FALSE)')
    lines.append(f"  stage <- if (is.null(uid)) mod${name}() else mod${name}(uid = uid)")
    if pnames:
        lines.append("  args <- Filter(Negate(is.null), list(" + ", ".join(f"{p} = {p}" for p in pnames) + "))")
        lines.append("  if (length(args) > 0) do.call(stage$setParams, .sml_py_args(args))")
    lines.append("  stage")
    lines.append("}")
    return fname, "\n".join(lines) + "\n"


_R_RUNTIME = '''# Runtime helpers shared by the generated stage constructors.

.sml_py_args <- function(args) {
  # R integers stay integers, length-1 vectors become scalars, longer vectors become lists
  lapply(args, function(a) if (is.atomic(a) && length(a) > 1) as.list(a) else a)
}

#' Convert an R data.frame to a synapseml_amd DataFrame
#' @param df an R data.frame
#' @param num_partitions partitions of the result
#' @export
sml_data_frame <- function(df, num_partitions = 1L) {
  core <- reticulate::import("synapseml_amd.core.dataframe")
  core$DataFrame$fromPandas(reticulate::r_to_py(df), num_partitions = as.integer(num_partitions))
}

#' Collect a synapseml_amd DataFrame into an R data.frame
#' @param df a synapseml_amd DataFrame
#' @export
sml_collect <- function(df) reticulate::py_to_r(df$toPandas())

.sml_as_py_df <- function(df) if (is.data.frame(df)) sml_data_frame(df) else df

#' Fit an estimator
#' @param stage a stage from one of the sml_* constructors
#' @param df an R data.frame or a synapseml_amd DataFrame
#' @export
sml_fit <- function(stage, df) stage$fit(.sml_as_py_df(df))

#' Transform with a transformer or fitted model
#' @param stage a transformer or model
#' @param df an R data.frame or a synapseml_amd DataFrame
#' @param collect return an R data.frame instead of the Python DataFrame
#' @export
sml_transform <- function(stage, df, collect = TRUE) {
  out <- stage$transform(.sml_as_py_df(df))
  if (collect) sml_collect(out) else out
}

#' Save a stage (SparkML directory layout)
#' @param stage stage to save
#' @param path directory
#' @export
sml_save <- function(stage, path) invisible(stage$save(path))

#' Load any saved stage
#' @param path directory written by sml_save
#' @export
sml_load <- function(path) {
  ser <- reticulate::import("synapseml_amd.core.serialize")
  ser$load_stage(path)
}
'''


def generate_r(out_dir: str, version: str = "0.2.0") -> List[str]:
    """Write the R package under ``out_dir``; returns the exported function names."""
    stages = all_stages()
    by_module: Dict[str, List[Tuple[str, str]]] = {}
    for path, cls in stages.items():
        top = path.split(".")[1]
        by_module.setdefault(top, []).append(r_function(path, cls))
    os.makedirs(os.path.join(out_dir, "R"), exist_ok=True)
    os.makedirs(os.path.join(out_dir, "tests", "testthat"), exist_ok=True)
    exported = ["sml_data_frame", "sml_collect", "sml_fit", "sml_transform", "sml_save", "sml_load"]
    with open(os.path.join(out_dir, "R", "runtime.R"), "w") as f:
        f.write(_R_RUNTIME)
    for top, funcs in sorted(by_module.items()):
        with open(os.path.join(out_dir, "R", f"{top}.R"), "w") as f:
            f.write(f"# Generated by synapseml_amd.codegen - stages of synapseml_amd.{top}\n\n")
            f.write("\n".join(src for _, src in funcs))
        with open(os.path.join(out_dir, "tests", "testthat", f"test-{top}.R"), "w") as f:
            f.write(f"# Generated: every stage of synapseml_amd.{top} constructs and round-trips its uid\n")
            for fname, _ in funcs:
                f.write(f'test_that("{fname} constructs", {{\n  s <- {fname}()\n'
                        f'  expect_true(nchar(s$uid) > 0)\n}})\n')
        exported += [fn for fn, _ in funcs]
    with open(os.path.join(out_dir, "NAMESPACE"), "w") as f:
        f.write("# Generated by synapseml_amd.codegen\n" + "".join(f"export({e})\n" for e in exported))
    with open(os.path.join(out_dir, "DESCRIPTION"), "w") as f:
        f.write(f"Package: {R_PACKAGE}\nType: Package\nTitle: R bindings for synapseml_amd\nVersion: {version}\n"
                "Description: Generated reticulate wrappers for every synapseml_amd pipeline stage.\n"
                "License: MIT\nImports: reticulate\nSuggests: testthat\nEncoding: UTF-8\n")
    with open(os.path.join(out_dir, "tests", "testthat.R"), "w") as f:
        f.write(f"library(testthat)\nlibrary({R_PACKAGE})\ntest_check(\"{R_PACKAGE}\")\n")
    return exported


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--r-out", default=os.path.join("build", "R", R_PACKAGE))
    a = ap.parse_args(argv)
    names = generate_r(a.r_out)
    print(f"{len(names)} R functions -> {a.r_out}")


if __name__ == "__main__":
    main()
