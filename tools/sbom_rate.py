#!/usr/bin/env python3
"""Decode rate of the native CycloneDX decoder (trivy_amd/csrc/sbom.cpp) on a fleet-size
document: N dpkg components of one Debian image (tests/test_sbom_native.py fleet_document),
against the Python restatement (trivy_amd/sbom.py) on the same text.  Host only."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

from test_sbom_native import fleet_document  # noqa: E402
from trivy_amd import sbom as ts  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    text = fleet_document(n).encode()
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        d = ts.decode_cyclonedx_native(text)
        dt = time.perf_counter() - t0
        assert d.target(-1)[3] == n
        d.close()
        best = dt if best is None else min(best, dt)
    print(f"native: {n} components, {len(text) / 1e6:.1f} MB in {best * 1e3:.1f} ms = {n / best / 1e6:.2f} M components/s")
    if len(sys.argv) > 2:
        t0 = time.perf_counter()
        ts.decode_cyclonedx(text.decode())
        dt = time.perf_counter() - t0
        print(f"python: {dt * 1e3:.1f} ms = {n / dt / 1e6:.3f} M components/s")


if __name__ == "__main__":
    main()
