"""Import alias for the framework package.

The framework's source tree lives in ``distributed-llm-training-benchmark-framework_amd/``
(a directory name that is not a valid Python identifier).  ``import dltb`` loads that
directory as the package ``dltb`` so that every submodule is importable as
``dltb.models``, ``dltb.ops``, ``dltb.parallel`` ... and relative imports inside the
package work unchanged.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "distributed-llm-training-benchmark-framework_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
