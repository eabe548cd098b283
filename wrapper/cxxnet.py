"""Drop-in module name of the reference's Python wrapper (wrapper/cxxnet.py):
``sys.path.append('wrapper'); import cxxnet`` keeps working.  The implementation is
cxxnet_amd.wrapper (no separate shared library is needed from Python; the CXN*
C ABI lives in cxxnet_amd/_native/libcxxnetwrapper.so for C/C++ callers)."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from cxxnet_amd.wrapper import DataIter, Net, train  # noqa: E402,F401
