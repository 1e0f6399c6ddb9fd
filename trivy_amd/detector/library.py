"""Mirror of reference pkg/detector/library (driver.go:25-159, detect.go:11-42) over the C-ABI.

Packages and results use the reference's Go field names as dict keys (ftypes.Package,
types.DetectedVulnerability).  The matching itself (prefix-scanned advisories, the six
constraint grammars of compare/) runs in libtrivy_amd.so on the GPU.
"""
import ctypes

from .._lib import lib, s, errbuf, Result, TVM_EUNSUPPORTED_TYPE
from .ospkg import DetectError, _pkg_array, _convert


def ecosystem(lib_type):
    """NewDriver(libType).Type(), or None when the type is unsupported."""
    r = lib().tvm_library_type(lib_type.encode())
    return r.decode() if r else None


class Driver:
    """library.Driver (driver.go:96-100)."""

    def __init__(self, engine, lib_type):
        self.engine, self.lib_type = engine, lib_type
        self.ecosystem = ecosystem(lib_type)
        if self.ecosystem is None:
            raise ValueError(f"the {lib_type!r} library type is not supported for vulnerability scanning")

    def type(self):
        return self.ecosystem

    def detect_vulnerabilities(self, pkg_id, pkg_name, pkg_ver):
        """(*Driver).DetectVulnerabilities (driver.go:111-137)."""
        res = Result()
        e = errbuf()
        rc = lib().tvm_library_detect_vulnerabilities(self.engine.h, self.lib_type.encode(), s(pkg_id), s(pkg_name),
                                                      s(pkg_ver), ctypes.byref(res), e, len(e))
        if rc:
            raise DetectError(e.value.decode())
        try:
            return _convert(res, [{"ID": pkg_id, "Name": pkg_name, "Version": pkg_ver}])
        finally:
            lib().tvm_result_free(ctypes.byref(res))


def detect(engine, lib_type, pkgs):
    """library.Detect (detect.go:11-42): None for an unsupported type."""
    arr, keep = _pkg_array(pkgs)
    res = Result()
    e = errbuf()
    rc = lib().tvm_library_detect(engine.h, lib_type.encode(), arr, len(pkgs), ctypes.byref(res), e, len(e))
    if rc == TVM_EUNSUPPORTED_TYPE:
        return None
    if rc:
        raise DetectError(e.value.decode())
    try:
        return _convert(res, pkgs)
    finally:
        lib().tvm_result_free(ctypes.byref(res))
