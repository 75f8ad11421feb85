"""setuptools hook: compile the gfx950 extension in-tree before packaging.

``pip install -e .`` / ``python setup.py build_ext --inplace`` both run
``multigrad_amd.ops.build.build()`` (hipcc --offload-arch=gfx950, no hipify).
"""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildWithExtension(build_py):
    def run(self):
        from multigrad_amd.ops import build as b
        b.build()
        super().run()


try:
    from setuptools.command.build_ext import build_ext

    class BuildExt(build_ext):
        def run(self):
            from multigrad_amd.ops import build as b
            b.build()

    cmds = {"build_py": BuildWithExtension, "build_ext": BuildExt}
except ImportError:  # pragma: no cover
    cmds = {"build_py": BuildWithExtension}

setup(cmdclass=cmds)
