"""trivy_amd: MI355X-native vulnerability matching for Trivy's detector hot path.

The product is the native library libtrivy_amd.so (C-ABI in include/trivy_amd.h):
a load-time flattener of trivy-db buckets into HBM tables plus gfx950 HIP kernels
that match batches of installed packages against them.  This Python package is a
thin ctypes mirror of the reference's Go surfaces (pkg/detector/ospkg, ...) used
by the tests and the benchmark.
"""
from .db import DB, Engine, load_fixture_files  # noqa: F401
from ._lib import lib, LIB_PATH, runtime_info  # noqa: F401

__version__ = "0.1.0"
