"""Wheel build: compiles the native gfx950 extensions (tools/build_native.py: g++ for the
host runtime, hipcc --offload-arch=gfx950 for the kernels) into the package before the
usual setuptools build, so the wheel carries the .so files next to their Python modules.
Set SML_SKIP_NATIVE=1 to package the Python sources only (the native modules then fail
loudly at first use)."""
import os
import subprocess
import sys

from setuptools import Distribution, find_packages, setup
from setuptools.command.build_py import build_py


class BuildWithNative(build_py):
    def run(self):
        if os.environ.get("SML_SKIP_NATIVE") != "1":
            here = os.path.dirname(os.path.abspath(__file__))
            subprocess.run([sys.executable, os.path.join(here, "tools", "build_native.py")], check=True)
        super().run()


class NativeDistribution(Distribution):
    """The wheel carries compiled gfx950/x86-64 modules: tag it per platform, not py3-none-any."""

    def has_ext_modules(self):
        return True


setup(
    name="synapseml-amd",
    version="0.1.0",
    description="MI355X-native distributed ML: GBDT, Vowpal-Wabbit-style linear learners, ONNX / deep-learning "
                "inference, explainers and HTTP serving on PyTorch-ROCm + HIP",
    python_requires=">=3.10",
    packages=find_packages(include=["synapseml_amd", "synapseml_amd.*"]),
    package_data={"": ["*.so"]},
    install_requires=["numpy", "torch"],
    extras_require={"onnx": ["onnx"], "arrow": ["pyarrow"], "spark": ["pyspark"],
                    "test": ["pytest", "pytest-timeout", "scikit-learn", "hypothesis"]},
    cmdclass={"build_py": BuildWithNative},
    distclass=NativeDistribution,
)
