"""Language-binding generator (reference: CORE/codegen/{CodeGen,Wrappable,RCodegen,PyCodegen}.scala and
CORE/param/RWrappableParam.scala - the reference generates Python/R/.NET wrappers from its Scala params).

Here every stage is already a Python class, so the Python "wrappers" are the classes themselves; what
this module generates is the R package: one constructor per stage (``sml_<snake_name>(...)``) that
imports the stage through reticulate, sets the non-NULL params, and returns the live Python object,
plus ``sml_fit`` / ``sml_transform`` / ``sml_save`` / ``sml_load`` and R <-> DataFrame conversion.
A testthat file per module constructs every stage (the reference's generated R tests do the same).

The .NET binding (``generate_dotnet``) is a P/Invoke layer over the engine's C ABI (libsml_gbdt.so).

usage: ``python -m synapseml_amd.codegen --r-out build/R/synapsemlamd --dotnet-out build/dotnet``"""
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


# ====================================================================== native C ABI + .NET
# The GBDT engine's C ABI (csrc/gbdt/c_api.cpp, libsml_gbdt.so) as data: (name, [(arg, C type)]). Every
# function returns int (0 ok, -1 error; SML_GetLastError for the message). The ctypes binding below and the
# generated C# P/Invoke layer are both derived from this one table, and the ctypes side is executed by the
# tests against the built library, so the .NET signatures are checked by construction.
C_API: List[Tuple[str, List[Tuple[str, str]]]] = [
    ("SML_DatasetCreateFromMat", [("data", "void*"), ("data_type", "int"), ("nrow", "int32"), ("ncol", "int32"),
                                  ("parameters", "char*"), ("label", "float*"), ("out", "void**")]),
    ("SML_DatasetSetWeight", [("dataset", "void*"), ("weight", "float*"), ("n", "int32")]),
    ("SML_DatasetGetNumData", [("dataset", "void*"), ("out", "int32*")]),
    ("SML_DatasetFree", [("dataset", "void*")]),
    ("SML_BoosterCreate", [("train", "void*"), ("parameters", "char*"), ("out", "void**")]),
    ("SML_BoosterAddValidData", [("booster", "void*"), ("valid", "void*")]),
    ("SML_BoosterLoadModelFromString", [("model", "char*"), ("out", "void**")]),
    ("SML_BoosterFree", [("booster", "void*")]),
    ("SML_BoosterUpdateOneIter", [("booster", "void*"), ("is_finished", "int*")]),
    ("SML_BoosterGetCurrentIteration", [("booster", "void*"), ("out", "int*")]),
    ("SML_BoosterGetNumClasses", [("booster", "void*"), ("out", "int*")]),
    ("SML_BoosterGetEval", [("booster", "void*"), ("data_idx", "int"), ("buffer_len", "int"), ("out_len", "int*"),
                            ("out_results", "double*")]),
    ("SML_BoosterPredictForMat", [("booster", "void*"), ("data", "void*"), ("data_type", "int"), ("nrow", "int32"),
                                  ("ncol", "int32"), ("predict_type", "int"), ("start_iteration", "int"),
                                  ("num_iteration", "int"), ("out_len", "int64*"), ("out_result", "double*")]),
    ("SML_BoosterSaveModelToString", [("booster", "void*"), ("start_iteration", "int"), ("num_iteration", "int"),
                                      ("buffer_len", "int64"), ("out_len", "int64*"), ("out_str", "char*")]),
]

_CS_TYPES = {"void*": "IntPtr", "void**": "out IntPtr", "int": "int", "int32": "int", "int*": "out int",
             "int32*": "out int", "int64": "long", "int64*": "out long", "float*": "float[]",
             "double*": "double[]", "char*": "string"}
_CS_OVERRIDE = {("SML_BoosterSaveModelToString", "out_str"): "byte[]",
                ("SML_DatasetCreateFromMat", "data"): "float[]", ("SML_BoosterPredictForMat", "data"): "float[]"}


def native_library_path() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libsml_gbdt.so")


def load_c_api(path: Optional[str] = None):
    """ctypes binding of libsml_gbdt.so with argtypes / restype from C_API."""
    import ctypes as C

    ct = {"void*": C.c_void_p, "void**": C.POINTER(C.c_void_p), "int": C.c_int, "int32": C.c_int32,
          "int*": C.POINTER(C.c_int), "int32*": C.POINTER(C.c_int32), "int64": C.c_int64,
          "int64*": C.POINTER(C.c_int64), "float*": C.POINTER(C.c_float), "double*": C.POINTER(C.c_double),
          "char*": C.c_char_p}
    lib = C.CDLL(path or native_library_path())
    for name, args in C_API:
        f = getattr(lib, name)
        f.argtypes = [ct[t] for _, t in args]
        f.restype = C.c_int
    lib.SML_GetLastError.restype = C.c_char_p
    lib.SML_GetLastError.argtypes = []
    return lib


def generate_dotnet(out_dir: str, namespace: str = "SynapseML.Amd") -> str:
    """C# binding of the native engine: a P/Invoke layer over libsml_gbdt.so (every C_API entry) and
    managed Dataset / Booster classes (IDisposable handles, errors raised as SynapseMLException) - the .NET
    surface the reference generates for its stages (CORE/codegen/DotnetCodegen.scala), over this engine's C
    ABI instead of a JVM bridge. Returns the path of the generated .cs file."""
    os.makedirs(out_dir, exist_ok=True)
    lines = ["// <auto-generated> by synapseml_amd.codegen.generate_dotnet - do not edit </auto-generated>",
             "using System;", "using System.Runtime.InteropServices;", "using System.Text;", "",
             f"namespace {namespace}", "{",
             "    public sealed class SynapseMLException : Exception",
             "    {", "        public SynapseMLException(string message) : base(message) { }", "    }", "",
             "    internal static class NativeMethods", "    {",
             '        private const string Lib = "sml_gbdt";', "",
             "        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]",
             "        internal static extern IntPtr SML_GetLastError();"]
    for name, args in C_API:
        ps = []
        for a, t in args:
            cst = _CS_OVERRIDE.get((name, a), _CS_TYPES[t])
            ps.append(f"{cst} {a}")
        lines += ["", "        [DllImport(Lib, CallingConvention = CallingConvention.Cdecl)]",
                  f"        internal static extern int {name}({', '.join(ps)});"]
    lines += ["", "        internal static void Check(int rc)", "        {",
              "            if (rc != 0) throw new SynapseMLException(Marshal.PtrToStringAnsi(SML_GetLastError()));",
              "        }", "    }", "",
              "    /// <summary>Binned training data (LightGBM Dataset semantics) owned by the native engine.</summary>",
              "    public sealed class GbdtDataset : IDisposable", "    {",
              "        internal IntPtr Handle;", "",
              "        public GbdtDataset(float[] rowMajor, int nrow, int ncol, float[] label, string parameters = \"\")",
              "        {",
              "            NativeMethods.Check(NativeMethods.SML_DatasetCreateFromMat(rowMajor, 0, nrow, ncol, parameters, label, out Handle));",
              "        }", "",
              "        public int NumData", "        {",
              "            get { NativeMethods.Check(NativeMethods.SML_DatasetGetNumData(Handle, out int n)); return n; }",
              "        }", "",
              "        public void SetWeight(float[] weight) =>",
              "            NativeMethods.Check(NativeMethods.SML_DatasetSetWeight(Handle, weight, weight.Length));", "",
              "        public void Dispose()", "        {",
              "            if (Handle != IntPtr.Zero) { NativeMethods.SML_DatasetFree(Handle); Handle = IntPtr.Zero; }",
              "        }", "    }", "",
              "    /// <summary>Gradient-boosted trees (device_type=gpu trains on the MI355X).</summary>",
              "    public sealed class GbdtBooster : IDisposable", "    {",
              "        private IntPtr handle;", "",
              "        public GbdtBooster(GbdtDataset train, string parameters)", "        {",
              "            NativeMethods.Check(NativeMethods.SML_BoosterCreate(train.Handle, parameters, out handle));",
              "        }", "",
              "        private GbdtBooster(IntPtr h) { handle = h; }", "",
              "        public static GbdtBooster FromModelString(string model)", "        {",
              "            NativeMethods.Check(NativeMethods.SML_BoosterLoadModelFromString(model, out IntPtr h));",
              "            return new GbdtBooster(h);", "        }", "",
              "        public void AddValidData(GbdtDataset valid) =>",
              "            NativeMethods.Check(NativeMethods.SML_BoosterAddValidData(handle, valid.Handle));", "",
              "        /// <returns>true when no further tree could be grown</returns>",
              "        public bool UpdateOneIter()", "        {",
              "            NativeMethods.Check(NativeMethods.SML_BoosterUpdateOneIter(handle, out int finished));",
              "            return finished != 0;", "        }", "",
              "        public int CurrentIteration", "        {",
              "            get { NativeMethods.Check(NativeMethods.SML_BoosterGetCurrentIteration(handle, out int i)); return i; }",
              "        }", "",
              "        public double[] GetEval(int dataIdx)", "        {",
              "            NativeMethods.Check(NativeMethods.SML_BoosterGetEval(handle, dataIdx, 0, out int n, null));",
              "            var r = new double[n];",
              "            NativeMethods.Check(NativeMethods.SML_BoosterGetEval(handle, dataIdx, r.Length, out n, r));",
              "            return r;", "        }", "",
              "        /// <param name=\"predictType\">0 raw, 1 normal, 2 leaf index, 3 contributions</param>",
              "        public double[] Predict(float[] rowMajor, int nrow, int ncol, int predictType = 1, int numIteration = -1)",
              "        {",
              "            NativeMethods.Check(NativeMethods.SML_BoosterPredictForMat(handle, rowMajor, 0, nrow, ncol, predictType, 0, numIteration, out long len, null));",
              "            var r = new double[len];",
              "            NativeMethods.Check(NativeMethods.SML_BoosterPredictForMat(handle, rowMajor, 0, nrow, ncol, predictType, 0, numIteration, out len, r));",
              "            return r;", "        }", "",
              "        public string SaveModelToString(int numIteration = -1)", "        {",
              "            NativeMethods.Check(NativeMethods.SML_BoosterSaveModelToString(handle, 0, numIteration, 0, out long need, null));",
              "            var buf = new byte[need];",
              "            NativeMethods.Check(NativeMethods.SML_BoosterSaveModelToString(handle, 0, numIteration, need, out need, buf));",
              "            return Encoding.UTF8.GetString(buf, 0, (int)need - 1);", "        }", "",
              "        public void Dispose()", "        {",
              "            if (handle != IntPtr.Zero) { NativeMethods.SML_BoosterFree(handle); handle = IntPtr.Zero; }",
              "        }", "    }", "}", ""]
    path = os.path.join(out_dir, f"{namespace}.Gbdt.cs")
    with open(path, "w") as f:
        f.write("\n".join(lines))
    return path


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--r-out", default=os.path.join("build", "R", R_PACKAGE))
    ap.add_argument("--dotnet-out", default=os.path.join("build", "dotnet"))
    a = ap.parse_args(argv)
    names = generate_r(a.r_out)
    print(f"{len(names)} R functions -> {a.r_out}")
    print(f".NET binding -> {generate_dotnet(a.dotnet_out)}")


if __name__ == "__main__":
    main()
