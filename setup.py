"""setuptools entry: compiles the gfx950 HIP kernels and the HDF5 layer in-tree
(cnmf_torch_amd/_build.py) before packaging, so wheels and editable installs carry the
same shared objects the repository uses.  ``pip install -e .`` or ``python setup.py
build_ext --inplace`` both work offline."""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.command.build_ext import build_ext

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


class NativeBuild(build_ext):
    def run(self):
        from cnmf_torch_amd import _build

        _build.build_all(force=False, jobs=int(os.environ.get("MAX_JOBS", "8")))


class BuildPy(build_py):
    def run(self):
        self.run_command("build_ext")
        super().run()


setup(cmdclass={"build_ext": NativeBuild, "build_py": BuildPy})
