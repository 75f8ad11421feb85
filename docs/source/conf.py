"""Sphinx configuration (reference: docs/source/conf.py -- autodoc, napoleon, viewcode,
notebooks, the "nature" theme).

Build with ``make -C docs html`` where Sphinx is installed.  The notebook extension is
used when it is importable; without it the notebooks are left out of the build.  The
markdown design notes are included through ``myst_parser`` when that is importable.
"""
import importlib.util
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)


def _have(mod):
    return importlib.util.find_spec(mod) is not None


def _version():
    ns = {}
    with open(os.path.join(ROOT, "multigrad_amd", "_version.py")) as f:
        exec(f.read(), ns)
    return ns.get("__version__", "unknown version")


project = "multigrad_amd"
author = "multigrad_amd developers"
copyright = "2026, " + author
version = release = _version()

extensions = ["sphinx.ext.autodoc", "sphinx.ext.napoleon", "sphinx.ext.viewcode"]
exclude_patterns = [".ipynb_checkpoints/*", "_build"]
if _have("nbsphinx"):
    extensions.append("nbsphinx")
    nbsphinx_execute = "never"     # the notebook needs a GPU for its engine cells
else:
    exclude_patterns.append("notebooks/*")
if _have("myst_parser"):
    extensions.append("myst_parser")

source_suffix = {".rst": "restructuredtext"}
if _have("myst_parser"):
    source_suffix[".md"] = "markdown"
master_doc = "index"
templates_path = []
autodoc_member_order = "bysource"
autodoc_default_options = {"members": True, "show-inheritance": True}
napoleon_numpy_docstring = True

html_theme = "nature"
html_static_path = []
