import datetime
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def parse_now(s):
    return int(datetime.datetime.strptime(s, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=datetime.timezone.utc).timestamp())


def _drop_zero(v):
    """Go zero values are indistinguishable from absent fields in the reference's structs.
    The embedded types.Vulnerability (vulnerability.go:30) is flattened: detectors only set
    its Severity."""
    v = dict(v)
    emb = v.pop("Vulnerability", None)
    if isinstance(emb, dict):
        for k, x in emb.items():
            v.setdefault(k, x)
    return {k: x for k, x in v.items() if x not in ("", 0, None, {}, [])}


def canon(vulns):
    """Canonical multiset order (SURVEY.md §8c parity definition)."""
    vulns = [_drop_zero(v) for v in vulns]
    key = lambda v: (v.get("PkgID", ""), v.get("PkgName", ""), v.get("InstalledVersion", ""),
                     v.get("VulnerabilityID", ""), v.get("FixedVersion", ""), v.get("PkgPath", ""))
    return sorted(vulns, key=lambda v: (key(v), json.dumps(v, sort_keys=True)))


@pytest.fixture(scope="session")
def oracle_built():
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return True


@pytest.fixture(autouse=True)
def _device_drained(request):
    """After each GPU test, wait for the device and surface any asynchronous fault here, so
    the test whose launch faulted is the one that fails (not the next one's first copy)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    from trivy_amd import _lib
    if _lib._lib is None:  # the test never loaded the library: nothing of ours can be queued
        return
    # hipDeviceSynchronize + hipGetLastError inside libtrivy_amd's own HIP runtime instance,
    # so the library's streams (engine, pipeline, drop-in) are drained whatever torch loaded
    e = _lib.errbuf()
    if _lib._lib.tvm_device_sync(0, e, len(e)):
        pytest.fail(f"asynchronous device error after {request.node.nodeid}: {e.value.decode()}")
