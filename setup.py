"""Builds the native libraries in-tree (hipcc for gfx950 + g++), then packages.

    python setup.py build_ext --inplace     # or: python -m hipsnapshot._build
"""

from setuptools import setup
from setuptools.command.build_ext import build_ext


class BuildNative(build_ext):
    def run(self):
        from hipsnapshot import _build

        _build.build_all(force=True)


setup(cmdclass={"build_ext": BuildNative})
