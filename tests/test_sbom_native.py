"""The native CycloneDX decoder (trivy_amd/csrc/sbom.cpp, tvm_sbom_*) against the Python
restatement trivy_amd/sbom.py, which the reference's integration SBOM goldens pin
(tests/test_sbom.py): the three CycloneDX goldens, then seeded synthetic documents that
exercise every rule of pkg/sbom/cyclonedx/unmarshal.go + pkg/sbom/io/decode.go the decoders
restate (component types, PURL forms and qualifiers, properties, dependencies, duplicate
bom-refs, malformed PURLs, escapes), field for field; the errors; and the decode rate at a
fleet-size document.  GPU: the native package arrays through the detectors give the same
findings as the Python path."""
import json
import os
import random
import time

import pytest

from trivy_amd import sbom as ts

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sbom")
CDX_GOLDENS = ["centos-7-cyclonedx.json", "fluentd-multiple-lockfiles-cyclonedx.json", "minikube-kbom.json"]


def _python(text):
    d = ts.decode_cyclonedx(text)
    d.pop("Root", None)
    return d


def _native(text):
    n = ts.decode_cyclonedx_native(text)
    try:
        return n.as_dict()
    finally:
        n.close()


@pytest.mark.parametrize("name", CDX_GOLDENS)
def test_goldens_equal_python_decode(name):
    text = open(os.path.join(HERE, name)).read()
    assert _native(text) == _python(text)


NAMES = ["bash", "openssl-libs", "libc6", "zlib", "lodash", "express", "Django", "requests", "log4j-core", "rails"]
VERS = ["1.0", "2.3.4-1", "1:1.0.2k-16.el7", "5.0-4+deb10u1", "0.9.8~rc1", "3.2", "v1.2.3", "4.17.21", ""]


def _purl(rng, name, ver, os_type):
    kind = rng.choice([os_type] * 4 + ["npm", "npm-scope", "maven", "pypi", "golang", "gem", "cocoapods", "k8s",
                                       "cargo", "conan", "unknown", "bad", "pct"])
    if rng.random() < 0.01:  # now and then a second OS package type: an aggregation error
        kind = rng.choice(["deb", "rpm", "apk"])
    q = []
    if rng.random() < 0.4:
        q.append("arch=" + rng.choice(["x86_64", "noarch", "amd64"]))
    if rng.random() < 0.2:
        q.append("epoch=" + rng.choice(["1", "2", "0", "+3", "x"]))
    if rng.random() < 0.1:
        q.append("modularitylabel=" + "nodejs:12:8030020201124152102:229f0a1c")
    if rng.random() < 0.2:
        q.append("distro=debian-10.2")
    qs = ("?" + "&".join(q)) if q else ""
    v = ("@" + ver) if ver else ""
    if kind == "deb":
        return f"pkg:deb/debian/{name}{v}{qs}"
    if kind == "rpm":
        return f"pkg:rpm/centos/{name}{v}{qs}"
    if kind == "apk":
        return f"pkg:apk/alpine/{name}{v}{qs}"
    if kind == "npm":
        return f"pkg:npm/{name}{v}"
    if kind == "npm-scope":
        return f"pkg:npm/%40babel/{name}{v}"
    if kind == "maven":
        return f"pkg:maven/org.apache.logging.log4j/{name}{v}"
    if kind == "pypi":
        return f"pkg:pypi/{name}{v}"
    if kind == "golang":
        return f"pkg:golang/github.com/x/{name}{v}"
    if kind == "gem":
        return f"pkg:gem/{name}{v}"
    if kind == "cocoapods":
        return f"pkg:cocoapods/{name}{v}#Core/Sub"
    if kind == "k8s":
        return f"pkg:k8s/{rng.choice(['eks', 'k8s.io', ''])}/{name}{v}"
    if kind == "cargo":
        return f"pkg:cargo/{name}{v}"
    if kind == "conan":
        return f"pkg:conan/{name}{v}"
    if kind == "unknown":
        return f"pkg:generic/{name}{v}"
    if kind == "pct":
        return f"pkg:npm/{name}%2Dx{v}"
    return rng.choice(["npm/x@1", "pkg:", "pkg:npm", "pkg:/"])


def _doc(seed, n=60):
    rng = random.Random(seed)
    comps, refs = [], []
    n_os = 1 if rng.random() < 0.8 else (0 if rng.random() < 0.8 else 2)
    os_type = rng.choice(["deb", "rpm", "apk"])
    for i in range(n_os):
        comps.append({"bom-ref": f"os-{i}", "type": "operating-system", "name": rng.choice(["debian", "centos", ""]),
                      "version": "10.2"})
    for i in range(n):
        name, ver = rng.choice(NAMES), rng.choice(VERS)
        ref = rng.choice([f"c{i}", f"c{i}", f"c{i}", f"c{max(0, i - 1)}", ""])  # some duplicate / empty refs
        typ = rng.choice(["library"] * 6 + ["application", "container", "platform", "file", "firmware"])
        c = {"bom-ref": ref, "type": typ, "name": name + rng.choice(["", "", "é", "\"q\""])}
        if rng.random() < 0.9:
            c["version"] = ver
        if rng.random() < 0.15:
            c["group"] = rng.choice(["org.example", "@scope", ""])
        if rng.random() < 0.95:
            c["purl"] = _purl(rng, name, ver, os_type)
        props = []
        if typ == "application" and rng.random() < 0.8:
            props.append({"name": "aquasecurity:trivy:Type",
                          "value": rng.choice(["npm", "pip", "jar", "node-pkg", "gemspec", "bundler", ""])})
        for k in ("PkgID", "FilePath", "SrcName", "SrcVersion", "SrcRelease", "SrcEpoch", "Modularitylabel",
                  "LayerDigest", "LayerDiffID", "Class"):
            if rng.random() < 0.15:
                val = {"SrcEpoch": rng.choice(["1", "0", "7"]), "FilePath": "app/package.json"}.get(k, f"{k.lower()}-{i}")
                props.append({"name": "aquasecurity:trivy:" + k if rng.random() < 0.9 else k, "value": val})
        if props:
            c["properties"] = props
        comps.append(c)
        refs.append(ref)
    deps = []
    for c in comps:
        if c["type"] in ("operating-system", "application") and rng.random() < 0.8:
            deps.append({"ref": c["bom-ref"], "dependsOn": rng.sample(refs, min(len(refs), rng.randint(0, 12)))
                         + ["missing-ref"]})
    doc = {"bomFormat": "CycloneDX", "specVersion": "1.5", "serialNumber": f"urn:uuid:{seed}", "version": 1,
           "metadata": {"component": {"bom-ref": "root", "type": "container", "name": "img"}},
           "components": comps, "dependencies": deps, "vulnerabilities": [{"id": "x", "ratings": [1.5e3, None, True]}]}
    return json.dumps(doc, ensure_ascii=rng.random() < 0.5)


@pytest.mark.parametrize("seed", range(40))
def test_synthetic_documents_equal_python_decode(seed):
    text = _doc(seed)
    try:
        want = _python(text)
    except ts.SBOMError as e:
        with pytest.raises(ts.SBOMError) as ei:
            _native(text)
        assert str(ei.value).split(":")[0] == str(e).split(":")[0]
        return
    assert _native(text) == want


def test_errors():
    for bad in ["{", "{\"components\": [1,]}", "{\"bomFormat\": \"CycloneDX\"} x", "[1, 2]", "{\"a\": tru}"]:
        with pytest.raises(ts.SBOMError):
            _native(bad)
    two_os = json.dumps({"components": [{"type": "operating-system", "name": "a"}, {"type": "operating-system"}]})
    with pytest.raises(ts.SBOMError, match="multiple OS components"):
        _native(two_os)
    mixed = json.dumps({"components": [{"type": "library", "name": "a", "purl": "pkg:deb/debian/a@1"},
                                       {"type": "library", "name": "b", "purl": "pkg:rpm/centos/b@1-1"}]})
    with pytest.raises(ts.SBOMError, match="multiple types of OS packages"):
        _native(mixed)
    with pytest.raises(ts.SBOMError, match="unsupported component type"):
        _native(json.dumps({"metadata": {"component": {"type": "file", "name": "x"}}}))


def fleet_document(n):
    """A fleet-size CycloneDX document: one OS (debian) and n dpkg components it depends on."""
    parts = []
    for i in range(n):
        parts.append('{"bom-ref":"pkg:deb/debian/p%d@1.%d-%d?distro=debian-12","type":"library","name":"p%d",'
                     '"version":"1.%d-%d","purl":"pkg:deb/debian/p%d@1.%d-%d?distro=debian-12","properties":'
                     '[{"name":"aquasecurity:trivy:SrcName","value":"s%d"},{"name":"aquasecurity:trivy:SrcVersion",'
                     '"value":"1.%d-%d"}]}' % (i, i % 97, i % 7, i, i % 97, i % 7, i, i % 97, i % 7, i // 3, i % 97, i % 7))
    refs = ",".join('"pkg:deb/debian/p%d@1.%d-%d?distro=debian-12"' % (i, i % 97, i % 7) for i in range(n))
    return ('{"bomFormat":"CycloneDX","specVersion":"1.5","version":1,"components":[{"bom-ref":"os","type":'
            '"operating-system","name":"debian","version":"12"},' + ",".join(parts) + '],"dependencies":[{"ref":"os",'
            '"dependsOn":[' + refs + ']}]}')


def test_fleet_document_rate():
    """200k components (the 1M-component rate is recorded by tools/sbom_rate.py): decoded
    natively, every package kept, in the OS's dependency order."""
    text = fleet_document(200_000)
    t0 = time.perf_counter()
    n = ts.decode_cyclonedx_native(text)
    dt = time.perf_counter() - t0
    _, _, _, count = n.target(-1)
    assert count == 200_000 and n.os == {"Family": "debian", "Name": "12"}
    n.close()
    assert dt < 2.0, dt


@pytest.mark.gpu
@pytest.mark.parametrize("name", CDX_GOLDENS)
def test_native_scan_equals_python_scan(name):
    import trivy_amd
    from test_sbom import FX, NOW
    eng = trivy_amd.Engine(trivy_amd.load_fixture_files(FX), 0)
    text = open(os.path.join(HERE, name)).read()
    want = ts.scan(eng, ts.decode(text), "img", now=NOW)
    n = ts.decode_cyclonedx_native(text)
    got = ts.scan_native(eng, n, "img", now=NOW)
    n.close()
    assert got == want and any(v for *_, v in got)


def _one(purl, props=()):
    return json.dumps({"bomFormat": "CycloneDX", "components": [
        {"bom-ref": "os", "type": "operating-system", "name": "centos", "version": "7"},
        {"bom-ref": "p", "type": "library", "name": "x", "purl": purl,
         "properties": [{"name": "aquasecurity:trivy:" + k, "value": v} for k, v in props]}],
        "dependencies": [{"ref": "os", "dependsOn": ["p"]}]})


@pytest.mark.parametrize("decode", [_python, _native], ids=["python", "native"])
def test_go_integer_and_rpm_semantics(decode):
    """Parity unpinned (no reference test covers these; restated from Go's strconv.Atoi and
    go-rpm-version): SrcEpoch is strconv.Atoi (decode.go:208-211: no whitespace, a sign, ASCII
    digits, int64 range; an error fails the decode); the purl epoch qualifier ignores an Atoi
    error (purl.go:229-233); an rpm purl's version splits at the FIRST '-' (purl.go:238-240, as
    the comparator does: oracle/rpm.c)."""
    pkg = lambda text: decode(text)["Packages"][0]  # noqa: E731
    assert pkg(_one("pkg:rpm/centos/x@1.2-3-4.el7"))["Version"] == "1.2"
    assert pkg(_one("pkg:rpm/centos/x@1.2-3-4.el7"))["Release"] == "3-4.el7"
    assert pkg(_one("pkg:rpm/centos/x@2:1.2-3.el7"))["Version"] == "1.2"
    for bad_epoch in ["+-1", "1 ", "0x1", "١", "9223372036854775808", ""]:
        assert pkg(_one(f"pkg:rpm/centos/x@1.0-1?epoch={urllib_quote(bad_epoch)}")).get("Epoch", 0) == 0, bad_epoch
    assert pkg(_one("pkg:rpm/centos/x@1.0-1?epoch=%2B3"))["Epoch"] == 3
    assert pkg(_one("pkg:rpm/centos/x@1.0-1?epoch=-2"))["Epoch"] == -2
    assert pkg(_one("pkg:rpm/centos/x@1.0-1", [("SrcEpoch", "9223372036854775807")]))["SrcEpoch"] == (1 << 63) - 1
    assert pkg(_one("pkg:rpm/centos/x@1.0-1", [("SrcEpoch", "-9223372036854775808")]))["SrcEpoch"] == -(1 << 63)
    assert pkg(_one("pkg:rpm/centos/x@1.0-1", [("SrcEpoch", "+7")]))["SrcEpoch"] == 7
    for bad in [" 1", "1 ", "\t1", "9223372036854775808", "1.0", "١", "+", ""]:
        with pytest.raises(ts.SBOMError, match="invalid src epoch"):
            decode(_one("pkg:rpm/centos/x@1.0-1", [("SrcEpoch", bad)]))


def urllib_quote(s):
    import urllib.parse
    return urllib.parse.quote(s, safe="")
