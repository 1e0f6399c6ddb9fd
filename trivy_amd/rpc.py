"""Twirp wire format of package batches and detected vulnerabilities (client/server mode;
SURVEY.md §8f rank 4: the transport of package batches into the detectors).

Restates the reference's protobuf schema for the messages on this path (field numbers are
the wire contract; rpc/common/service.proto:33-68 Package / PkgIdentifier / Location,
:116-154 Vulnerability / DataSource / Layer / CVSS / Severity, rpc/scanner/service.proto:
33-48 ScanResponse / Result) as descriptors built at import time, and the conversions of
pkg/rpc/convert.go:
  :51-77    ConvertToRPCPkgs        :205-231  ConvertFromRPCPkgs
  :79-92    ConvertToRPCPkgIdentifier (nil when empty)   :233-251 ConvertFromRPCPkgIdentifier
  :94-103   ConvertToRPCLocations   :253-263  ConvertFromRPCLocation
  :265-331  ConvertToRPCVulns (severity string -> enum, UNKNOWN when invalid; CVSS and vendor
            severity maps always present; timestamps; custom data as google.protobuf.Value)
  :562-619  ConvertFromRPCVulns (enum -> severity string)
  :364-370, :646-655 layers;  :397-407, :713-723 data sources;  :409-425 results (the
            vulnerability and package parts).
Packages and vulnerabilities are dicts with the Go field names (ftypes.Package,
types.DetectedVulnerability; zero values omitted), as everywhere else in this package.
`detect_scan_result` serves one twirp Result: its packages go through the GPU detector and
come back as the Result's vulnerabilities.  The twirp server itself is out of scope.
"""
import datetime

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory, struct_pb2, timestamp_pb2  # noqa: F401

SEVERITIES = ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]

_F = descriptor_pb2.FieldDescriptorProto
_T = {"string": _F.TYPE_STRING, "int32": _F.TYPE_INT32, "bool": _F.TYPE_BOOL, "double": _F.TYPE_DOUBLE,
      "enum": _F.TYPE_ENUM, "msg": _F.TYPE_MESSAGE}

# (message, [(field, number, type, label, type_name)])  label: "" single, "rep" repeated
_COMMON = [
    ("OS", [("family", 1, "string"), ("name", 2, "string"), ("eosl", 3, "bool"), ("extended", 4, "bool")]),
    ("Repository", [("family", 1, "string"), ("release", 2, "string")]),
    ("PkgIdentifier", [("purl", 1, "string"), ("bom_ref", 2, "string")]),
    ("Location", [("start_line", 1, "int32"), ("end_line", 2, "int32")]),
    ("Layer", [("digest", 1, "string"), ("diff_id", 2, "string"), ("created_by", 3, "string")]),
    ("DataSource", [("id", 1, "string"), ("name", 2, "string"), ("url", 3, "string")]),
    ("CVSS", [("v2_vector", 1, "string"), ("v3_vector", 2, "string"), ("v2_score", 3, "double"),
              ("v3_score", 4, "double")]),
    ("Package", [("id", 13, "string"), ("name", 1, "string"), ("version", 2, "string"), ("release", 3, "string"),
                 ("epoch", 4, "int32"), ("identifier", 19, "msg", "", ".trivy.common.PkgIdentifier"),
                 ("arch", 5, "string"), ("src_name", 6, "string"), ("src_version", 7, "string"),
                 ("src_release", 8, "string"), ("src_epoch", 9, "int32"), ("licenses", 15, "string", "rep"),
                 ("locations", 20, "msg", "rep", ".trivy.common.Location"),
                 ("layer", 11, "msg", "", ".trivy.common.Layer"), ("file_path", 12, "string"),
                 ("depends_on", 14, "string", "rep"), ("digest", 16, "string"), ("dev", 17, "bool"),
                 ("indirect", 18, "bool")]),
    ("Vulnerability", [("vulnerability_id", 1, "string"), ("pkg_name", 2, "string"),
                       ("installed_version", 3, "string"), ("fixed_version", 4, "string"), ("title", 5, "string"),
                       ("description", 6, "string"), ("severity", 7, "enum", "", ".trivy.common.Severity"),
                       ("references", 8, "string", "rep"),
                       ("pkg_identifier", 25, "msg", "", ".trivy.common.PkgIdentifier"),
                       ("layer", 10, "msg", "", ".trivy.common.Layer"), ("severity_source", 11, "string"),
                       ("cvss", 12, "msg", "rep", ".trivy.common.Vulnerability.CvssEntry"),
                       ("cwe_ids", 13, "string", "rep"), ("primary_url", 14, "string"),
                       ("published_date", 15, "msg", "", ".google.protobuf.Timestamp"),
                       ("last_modified_date", 16, "msg", "", ".google.protobuf.Timestamp"),
                       ("custom_advisory_data", 17, "msg", "", ".google.protobuf.Value"),
                       ("custom_vuln_data", 18, "msg", "", ".google.protobuf.Value"),
                       ("vendor_ids", 19, "string", "rep"),
                       ("data_source", 20, "msg", "", ".trivy.common.DataSource"),
                       ("vendor_severity", 21, "msg", "rep", ".trivy.common.Vulnerability.VendorSeverityEntry"),
                       ("pkg_path", 22, "string"), ("pkg_id", 23, "string"), ("status", 24, "int32")]),
]
_MAPS = {"Vulnerability": [("CvssEntry", "msg", ".trivy.common.CVSS"),
                           ("VendorSeverityEntry", "enum", ".trivy.common.Severity")]}
_SCANNER = [
    ("Result", [("target", 1, "string"), ("vulnerabilities", 2, "msg", "rep", ".trivy.common.Vulnerability"),
                ("class", 6, "string"), ("type", 3, "string"),
                ("packages", 5, "msg", "rep", ".trivy.common.Package")]),
    ("ScanResponse", [("os", 1, "msg", "", ".trivy.common.OS"),
                      ("results", 3, "msg", "rep", ".trivy.scanner.Result")]),
]


def _add_fields(m, fields):
    for f in fields:
        name, num, typ = f[:3]
        label = f[3] if len(f) > 3 else ""
        fd = m.field.add(name=name, number=num, type=_T[typ],
                         label=_F.LABEL_REPEATED if label == "rep" else _F.LABEL_OPTIONAL)
        if len(f) > 4:
            fd.type_name = f[4]


def _build():
    pool = descriptor_pool.Default()  # holds google/protobuf/{timestamp,struct}.proto (imported above)
    common = descriptor_pb2.FileDescriptorProto(name="trivy/common/service.proto", package="trivy.common",
                                                syntax="proto3",
                                                dependency=["google/protobuf/timestamp.proto",
                                                            "google/protobuf/struct.proto"])
    sev = common.enum_type.add(name="Severity")
    for i, s in enumerate(SEVERITIES):
        sev.value.add(name=s, number=i)
    for name, fields in _COMMON:
        m = common.message_type.add(name=name)
        _add_fields(m, fields)
        for entry, vt, vname in _MAPS.get(name, []):
            e = m.nested_type.add(name=entry)
            e.options.map_entry = True
            _add_fields(e, [("key", 1, "string"), ("value", 2, vt, "", vname)])
    pool.Add(common)
    scanner = descriptor_pb2.FileDescriptorProto(name="trivy/scanner/service.proto", package="trivy.scanner",
                                                 syntax="proto3", dependency=["trivy/common/service.proto"])
    for name, fields in _SCANNER:
        _add_fields(scanner.message_type.add(name=name), fields)
    pool.Add(scanner)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName(n))  # noqa: E731
    return {n: get("trivy.common." + n) for n, _ in _COMMON} | {n: get("trivy.scanner." + n) for n, _ in _SCANNER}


MSG = _build()
Package, Vulnerability, Result, ScanResponse = MSG["Package"], MSG["Vulnerability"], MSG["Result"], MSG["ScanResponse"]


# ---- packages ---------------------------------------------------------------------------------
def _to_identifier(ident):
    """ConvertToRPCPkgIdentifier: None for an empty identifier."""
    if not ident or (not ident.get("PURL") and not ident.get("BOMRef")):
        return None
    return MSG["PkgIdentifier"](purl=ident.get("PURL") or "", bom_ref=ident.get("BOMRef") or "")


def _from_identifier(msg, has):
    if not has:
        return {}
    out = {}
    if msg.bom_ref:
        out["BOMRef"] = msg.bom_ref
    if msg.purl:
        out["PURL"] = msg.purl
    return out


def _to_layer(layer):
    layer = layer or {}
    return MSG["Layer"](digest=layer.get("Digest", ""), diff_id=layer.get("DiffID", ""),
                        created_by=layer.get("CreatedBy", ""))


def _from_layer(msg, has):
    if not has:
        return {}
    return _nz({"Digest": msg.digest, "DiffID": msg.diff_id, "CreatedBy": msg.created_by})


def _nz(d):
    return {k: v for k, v in d.items() if v not in ("", None, 0, False, [], {})}


def to_rpc_pkgs(pkgs):
    """ConvertToRPCPkgs (convert.go:51-77)."""
    out = []
    for p in pkgs:
        m = Package(id=p.get("ID", ""), name=p.get("Name", ""), version=p.get("Version", ""),
                    release=p.get("Release", ""), epoch=int(p.get("Epoch", 0)), arch=p.get("Arch", ""),
                    dev=bool(p.get("Dev", False)), src_name=p.get("SrcName", ""), src_version=p.get("SrcVersion", ""),
                    src_release=p.get("SrcRelease", ""), src_epoch=int(p.get("SrcEpoch", 0)),
                    licenses=p.get("Licenses") or [], file_path=p.get("FilePath", ""),
                    depends_on=p.get("DependsOn") or [], digest=p.get("Digest", ""),
                    indirect=bool(p.get("Indirect", False)))
        ident = _to_identifier(p.get("Identifier"))
        if ident is not None:
            m.identifier.CopyFrom(ident)
        for loc in p.get("Locations") or []:
            m.locations.add(start_line=int(loc.get("StartLine", 0)), end_line=int(loc.get("EndLine", 0)))
        m.layer.CopyFrom(_to_layer(p.get("Layer")))  # always set: ConvertToRPCLayer returns a pointer
        out.append(m)
    return out


def from_rpc_pkgs(msgs):
    """ConvertFromRPCPkgs (convert.go:205-231)."""
    out = []
    for m in msgs:
        out.append(_nz({"ID": m.id, "Name": m.name, "Version": m.version, "Release": m.release, "Epoch": m.epoch,
                        "Arch": m.arch, "Identifier": _from_identifier(m.identifier, m.HasField("identifier")),
                        "Dev": m.dev, "SrcName": m.src_name, "SrcVersion": m.src_version,
                        "SrcRelease": m.src_release, "SrcEpoch": m.src_epoch, "Licenses": list(m.licenses),
                        "Locations": [_nz({"StartLine": x.start_line, "EndLine": x.end_line}) for x in m.locations],
                        "Layer": _from_layer(m.layer, m.HasField("layer")), "FilePath": m.file_path,
                        "DependsOn": list(m.depends_on), "Digest": m.digest, "Indirect": m.indirect}))
    return out


# ---- vulnerabilities ----------------------------------------------------------------------------
def _ts(value):
    """A Go time (RFC 3339 string or datetime) as google.protobuf.Timestamp."""
    t = timestamp_pb2.Timestamp()
    if isinstance(value, str):
        value = datetime.datetime.fromisoformat(value.replace("Z", "+00:00"))
    t.FromDatetime(value.astimezone(datetime.timezone.utc) if value.tzinfo else value)
    return t


def _ts_str(t):
    return t.ToDatetime(tzinfo=datetime.timezone.utc).isoformat().replace("+00:00", "Z")


def _value(x):
    v = struct_pb2.Value()
    if isinstance(x, dict):
        v.struct_value.update(x)
    elif isinstance(x, list):
        v.list_value.extend(x)
    elif isinstance(x, bool):
        v.bool_value = x
    elif isinstance(x, (int, float)):
        v.number_value = x
    elif x is None:
        v.null_value = 0
    else:
        v.string_value = str(x)
    return v


def _from_value(v):
    kind = v.WhichOneof("kind")
    if kind == "struct_value":
        return {k: _from_value(x) for k, x in v.struct_value.fields.items()}
    if kind == "list_value":
        return [_from_value(x) for x in v.list_value.values]
    if kind == "number_value":
        return v.number_value
    if kind == "bool_value":
        return v.bool_value
    if kind == "string_value":
        return v.string_value
    return None


def to_rpc_vulns(vulns):
    """ConvertToRPCVulns (convert.go:265-331)."""
    out = []
    for v in vulns:
        sev = v.get("Severity", "")
        m = Vulnerability(vulnerability_id=v.get("VulnerabilityID", ""), vendor_ids=v.get("VendorIDs") or [],
                          pkg_id=v.get("PkgID", ""), pkg_name=v.get("PkgName", ""), pkg_path=v.get("PkgPath", ""),
                          installed_version=v.get("InstalledVersion", ""), fixed_version=v.get("FixedVersion", ""),
                          status=int(v.get("Status", 0)), title=v.get("Title", ""),
                          description=v.get("Description", ""),
                          severity=SEVERITIES.index(sev) if sev in SEVERITIES else 0,  # NewSeverity error -> UNKNOWN
                          references=v.get("References") or [], severity_source=v.get("SeveritySource", ""),
                          cwe_ids=v.get("CweIDs") or [], primary_url=v.get("PrimaryURL", ""))
        ident = _to_identifier(v.get("PkgIdentifier"))
        if ident is not None:
            m.pkg_identifier.CopyFrom(ident)
        for vendor, s in (v.get("VendorSeverity") or {}).items():
            m.vendor_severity[vendor] = int(s)
        for vendor, c in (v.get("CVSS") or {}).items():
            m.cvss[vendor].CopyFrom(MSG["CVSS"](v2_vector=c.get("V2Vector", ""), v3_vector=c.get("V3Vector", ""),
                                                v2_score=float(c.get("V2Score", 0)),
                                                v3_score=float(c.get("V3Score", 0))))
        m.layer.CopyFrom(_to_layer(v.get("Layer")))
        if v.get("LastModifiedDate"):
            m.last_modified_date.CopyFrom(_ts(v["LastModifiedDate"]))
        if v.get("PublishedDate"):
            m.published_date.CopyFrom(_ts(v["PublishedDate"]))
        if v.get("Custom") is not None:
            m.custom_advisory_data.CopyFrom(_value(v["Custom"]))
        if v.get("VulnerabilityCustom") is not None:
            m.custom_vuln_data.CopyFrom(_value(v["VulnerabilityCustom"]))
        ds = v.get("DataSource")
        if ds is not None:
            m.data_source.CopyFrom(MSG["DataSource"](id=ds.get("ID", ""), name=ds.get("Name", ""),
                                                     url=ds.get("URL", "")))
        out.append(m)
    return out


def from_rpc_vulns(msgs):
    """ConvertFromRPCVulns (convert.go:562-619)."""
    out = []
    for m in msgs:
        d = {"VulnerabilityID": m.vulnerability_id, "VendorIDs": list(m.vendor_ids), "PkgID": m.pkg_id,
             "PkgName": m.pkg_name, "PkgPath": m.pkg_path, "InstalledVersion": m.installed_version,
             "FixedVersion": m.fixed_version,
             "PkgIdentifier": _from_identifier(m.pkg_identifier, m.HasField("pkg_identifier")),
             "Status": m.status, "Title": m.title, "Description": m.description,
             "Severity": SEVERITIES[m.severity] if m.severity < len(SEVERITIES) else "UNKNOWN",
             "CVSS": {k: _nz({"V2Vector": c.v2_vector, "V3Vector": c.v3_vector, "V2Score": c.v2_score,
                              "V3Score": c.v3_score}) for k, c in m.cvss.items()},
             "References": list(m.references), "CweIDs": list(m.cwe_ids),
             "VendorSeverity": dict(m.vendor_severity),
             "Layer": _from_layer(m.layer, m.HasField("layer")), "SeveritySource": m.severity_source,
             "PrimaryURL": m.primary_url}
        if m.HasField("last_modified_date"):
            d["LastModifiedDate"] = _ts_str(m.last_modified_date)
        if m.HasField("published_date"):
            d["PublishedDate"] = _ts_str(m.published_date)
        if m.HasField("custom_vuln_data"):
            d["VulnerabilityCustom"] = _from_value(m.custom_vuln_data)
        if m.HasField("custom_advisory_data"):
            d["Custom"] = _from_value(m.custom_advisory_data)
        if m.HasField("data_source"):
            d["DataSource"] = _nz({"ID": m.data_source.id, "Name": m.data_source.name, "URL": m.data_source.url})
        out.append(_nz(d))
    return out


# ---- results over the wire ----------------------------------------------------------------------
def encode_result(target, cls, typ, pkgs=(), vulns=()):
    r = Result(target=target, type=typ)
    setattr(r, "class", cls)
    r.packages.extend(to_rpc_pkgs(pkgs))
    r.vulnerabilities.extend(to_rpc_vulns(vulns))
    return r.SerializeToString()


def decode_result(raw):
    """ConvertFromRPCResults for one Result's target / class / type / packages / vulnerabilities."""
    r = Result.FromString(raw)
    return {"Target": r.target, "Class": getattr(r, "class"), "Type": r.type,
            "Packages": from_rpc_pkgs(r.packages), "Vulnerabilities": from_rpc_vulns(r.vulnerabilities)}


def detect_scan_result(engine, raw, family, os_ver, repo=None, now=None):
    """One twirp Result carrying an OS target's packages -> the same Result with the GPU
    detector's vulnerabilities (ospkg.Detect on the engine), serialized."""
    from .detector.ospkg import detect
    r = decode_result(raw)
    vulns, _eosl = detect(engine, family, os_ver, repo, r["Packages"], now=now)
    return encode_result(r["Target"], r["Class"] or "os-pkgs", r["Type"] or family, r["Packages"], vulns)
