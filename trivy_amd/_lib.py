"""ctypes binding of the trivy_amd C-ABI (include/trivy_amd.h).

The native library is the product: there is no Python or CPU fallback for any
matching step.  Loading fails loudly when libtrivy_amd.so has not been built.
"""
import atexit
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# TVM_LIB_PATH: another build of the same library - the sanitizer build (libtrivy_amd_san.so,
# `make -C trivy_amd/csrc san`) that tools/san/run.sh loads into the CPU tests
LIB_PATH = os.environ.get("TVM_LIB_PATH") or os.path.join(_HERE, "libtrivy_amd.so")

TVM_OK, TVM_EDETECT, TVM_EUNSUPPORTED_OS, TVM_EINVAL, TVM_EDEVICE, TVM_EUNSUPPORTED_TYPE = 0, 1, 2, 3, 4, 5
COPY_PKG_ID, COPY_PKG_NAME, COPY_IDENTIFIER, COPY_LAYER = 1, 2, 4, 8


class Str(ctypes.Structure):
    _fields_ = [("p", ctypes.c_char_p), ("n", ctypes.c_size_t)]


class Package(ctypes.Structure):
    _fields_ = [
        ("id", Str), ("name", Str), ("version", Str), ("release", Str), ("arch", Str),
        ("epoch", ctypes.c_int64),
        ("src_name", Str), ("src_version", Str), ("src_release", Str),
        ("src_epoch", ctypes.c_int64),
        ("modularitylabel", Str),
        ("has_build_info", ctypes.c_int32),
        ("content_sets", ctypes.POINTER(Str)), ("n_content_sets", ctypes.c_size_t),
        ("nvr", Str), ("build_arch", Str),
        ("file_path", Str),
    ]


class RawStr(ctypes.Structure):  # tvm_str read back from the library (not NUL-terminated)
    _fields_ = [("p", ctypes.c_void_p), ("n", ctypes.c_size_t)]

    def bytes(self):
        return ctypes.string_at(self.p, self.n) if self.n else b""


class RawPackage(ctypes.Structure):  # tvm_package read back (tvm_sbom_packages)
    _fields_ = [(n, RawStr if t is Str else t) for n, t in Package._fields_]


class SbomExtra(ctypes.Structure):
    _fields_ = [("purl", RawStr), ("bom_ref", RawStr), ("layer_digest", RawStr), ("layer_diff_id", RawStr),
                ("present", ctypes.c_uint32)]


class Repository(ctypes.Structure):
    _fields_ = [("family", Str), ("release", Str)]


class Vuln(ctypes.Structure):
    _fields_ = [
        ("pkg_index", ctypes.c_uint32), ("copy_flags", ctypes.c_uint32),
        ("vulnerability_id", ctypes.c_char_p),
        ("vendor_ids", ctypes.POINTER(ctypes.c_char_p)), ("n_vendor_ids", ctypes.c_size_t),
        ("pkg_id", ctypes.c_char_p), ("pkg_name", ctypes.c_char_p), ("pkg_path", ctypes.c_char_p),
        ("installed_version", ctypes.c_char_p), ("fixed_version", ctypes.c_char_p),
        ("status", ctypes.c_int32),
        ("severity_source", ctypes.c_char_p), ("severity", ctypes.c_char_p),
        ("has_data_source", ctypes.c_int32),
        ("data_source_id", ctypes.c_char_p), ("data_source_name", ctypes.c_char_p),
        ("data_source_url", ctypes.c_char_p),
        ("custom_json", ctypes.c_char_p),
    ]


class VulnSet(ctypes.Structure):
    _fields_ = [("row_end", ctypes.POINTER(ctypes.c_uint32)), ("n_pkgs", ctypes.c_size_t),
                ("first_pkg", ctypes.c_uint32), ("rec", ctypes.c_void_p), ("rec_width", ctypes.c_uint32),
                ("n", ctypes.c_size_t), ("adv_recs", ctypes.POINTER(Vuln)), ("n_adv_recs", ctypes.c_size_t),
                ("grp_recs", ctypes.POINTER(Vuln)), ("n_grp_recs", ctypes.c_size_t), ("priv", ctypes.c_void_p)]


class AttrCols(ctypes.Structure):
    _fields_ = [("arch_off", ctypes.c_void_p), ("arch_len", ctypes.c_void_p), ("cpe_set", ctypes.c_void_p)]


class Result(ctypes.Structure):
    _fields_ = [("vulns", ctypes.POINTER(Vuln)), ("n", ctypes.c_size_t), ("eosl", ctypes.c_int32),
                ("priv", ctypes.c_void_p)]


class FillIn(ctypes.Structure):
    _fields_ = [("vulnerability_id", Str), ("data_source_id", Str), ("severity_source", Str), ("severity", Str),
                ("status", ctypes.c_int32), ("has_fixed_version", ctypes.c_int32)]


class FillOut(ctypes.Structure):
    _fields_ = [("found", ctypes.c_int32), ("status", ctypes.c_int32), ("severity", ctypes.c_char_p),
                ("severity_source", ctypes.c_char_p), ("primary_url", ctypes.c_char_p),
                ("vulnerability_json", ctypes.c_char_p)]


class FillResult(ctypes.Structure):
    _fields_ = [("items", ctypes.POINTER(FillOut)), ("n", ctypes.c_size_t), ("priv", ctypes.c_void_p)]


class IgnoreRulesC(ctypes.Structure):
    _fields_ = [("ids", ctypes.POINTER(Str)), ("n_ids", ctypes.c_size_t), ("id_ranks", ctypes.c_void_p),
                ("all_id", ctypes.c_void_p), ("all_prec", ctypes.c_void_p), ("n_all", ctypes.c_size_t),
                ("pkg_pkg", ctypes.c_void_p), ("pkg_id", ctypes.c_void_p), ("pkg_prec", ctypes.c_void_p),
                ("n_pkg", ctypes.c_size_t), ("pkg_class", ctypes.c_void_p),
                ("cls_class", ctypes.c_void_p), ("cls_id", ctypes.c_void_p), ("cls_prec", ctypes.c_void_p),
                ("n_cls", ctypes.c_size_t)]


class FilterOpts(ctypes.Structure):
    _fields_ = [("severity_mask", ctypes.c_uint32), ("ignore_status_mask", ctypes.c_uint32),
                ("ignore", ctypes.POINTER(IgnoreRulesC)),
                ("vex_pkgs", ctypes.c_void_p), ("vex_id_index", ctypes.c_void_p), ("n_vex", ctypes.c_size_t),
                ("vex_ids", ctypes.POINTER(Str)), ("n_vex_ids", ctypes.c_size_t), ("vex_id_ranks", ctypes.c_void_p)]


# (name, restype, argtypes) for every exported symbol of include/trivy_amd.h
_P = ctypes.c_void_p
_SIG = [
    ("tvm_version", ctypes.c_char_p, []),
    ("tvm_abi_version", ctypes.c_int, []),
    ("tvm_db_new", _P, []),
    ("tvm_db_free", None, [_P]),
    ("tvm_db_put", ctypes.c_int, [_P, ctypes.POINTER(Str), ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_db_put_many", ctypes.c_int, [_P, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("tvm_db_put_bbolt", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_bbolt_walk", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_db_put_arena", ctypes.c_int, [_P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    ("tvm_db_finalize", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_db_stats", None, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_engine_open", _P, [_P, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_engine_close", None, [_P]),
    ("tvm_engine_swap", ctypes.c_int, [_P, _P, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_engine_table_bytes", ctypes.c_uint64, [_P]),
    ("tvm_engine_verify", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_engine_set_variant", ctypes.c_int, [_P, ctypes.c_int]),
    ("tvm_variant_name", ctypes.c_char_p, [ctypes.c_int]),
    ("tvm_variant_grammar_sets", ctypes.c_int, [ctypes.c_int]),
    ("tvm_engine_last_variant", ctypes.c_int, [_P]),
    ("tvm_ospkg_detect", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Repository),
                                        ctypes.POINTER(Package), ctypes.c_size_t, ctypes.c_int64,
                                        ctypes.POINTER(Result), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_ospkg_driver_detect", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Repository),
                                               ctypes.POINTER(Package), ctypes.c_size_t, ctypes.c_int64,
                                               ctypes.POINTER(Result), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_ospkg_is_supported", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64]),
    ("tvm_result_free", None, [ctypes.POINTER(Result)]),
    ("tvm_batch_new", _P, []),
    ("tvm_batch_free", None, [_P]),
    ("tvm_batch_add", ctypes.c_int64, [_P, _P, ctypes.c_char_p, Str, Str]),
    ("tvm_batch_add_many", ctypes.c_int64, [_P, _P, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("tvm_batch_add_many_ex", ctypes.c_int64, [_P, _P, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_uint32]),
    ("tvm_batch_size", ctypes.c_int64, [_P]),
    ("tvm_batch_add_targets", ctypes.c_int64, [_P, _P, ctypes.c_size_t, ctypes.POINTER(Str), ctypes.c_void_p,
                                               ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p]),
    ("tvm_batch_add_targets_attrs", ctypes.c_int64, [_P, _P, ctypes.c_size_t, ctypes.POINTER(Str), ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("tvm_batch_cpe_set", ctypes.c_int64, [_P, _P, ctypes.c_void_p, ctypes.c_size_t, Str]),
    ("tvm_batch_add_many_attrs", ctypes.c_int64, [_P, _P, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_uint32]),
    ("tvm_match_redhat_result", ctypes.c_int, [_P, _P, ctypes.POINTER(Result), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_match_redhat_merge", ctypes.c_int, [_P, _P, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_match_redhat_merge_time", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                   ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_match_redhat_vulns", ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, ctypes.POINTER(Result), ctypes.c_char_p,
                                              ctypes.c_size_t]),
    ("tvm_batch_upload", ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_match_launch", ctypes.c_int, [_P, _P, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_engine_sync", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_device_sync", ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_shutdown", None, []),
    ("tvm_pipeline_times", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_pool_stats", None, [ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_sbom_decode_cyclonedx", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_sbom_free", None, [ctypes.c_void_p]),
    ("tvm_sbom_info", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(RawStr),
                                     ctypes.POINTER(RawStr), ctypes.POINTER(RawStr), ctypes.POINTER(ctypes.c_int64),
                                     ctypes.POINTER(ctypes.c_size_t)]),
    ("tvm_sbom_packages", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(RawStr), ctypes.POINTER(RawStr),
                                         ctypes.POINTER(ctypes.POINTER(RawPackage)), ctypes.POINTER(ctypes.c_size_t)]),
    ("tvm_sbom_package_extra", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t,
                                              ctypes.POINTER(SbomExtra)]),
    ("tvm_wire_encode", ctypes.c_int, [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.POINTER(ctypes.c_uint32)]),
    ("tvm_pool_trim", None, []),
    ("tvm_match_status", ctypes.c_int, [_P, _P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_match_fetch", ctypes.c_int, [_P, _P, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_match_copy_device", ctypes.c_int, [_P, _P, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_match_order_into", ctypes.c_int, [_P, _P, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_match_time", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_char_p,
                                      ctypes.c_size_t]),
    ("tvm_match_algorithmic_bytes", ctypes.c_uint64, [_P, _P]),
    ("tvm_db_rows_many", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    ("tvm_batch_set_package_base", ctypes.c_int, [_P, ctypes.c_uint32]),
    ("tvm_batch_upload_into", ctypes.c_int, [_P, _P, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_pipeline_prepare", ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p,
                                            ctypes.c_size_t]),
    ("tvm_pipeline_run", ctypes.c_int, [_P, _P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_pipeline_result", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_pipeline_result_raw", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint32),
                                               ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_pipeline_stats", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_version_key", ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_size_t]),
    ("tvm_engine_dropin_stats", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_deb_fast_key_host", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p,
                                             ctypes.c_size_t]),
    ("tvm_db_advisory_vuln_id", ctypes.c_char_p, [_P, ctypes.c_uint32]),
    ("tvm_version_class", ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_lib_is_vulnerable_host", ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                                  ctypes.c_size_t]),
    ("tvm_library_type", ctypes.c_char_p, [ctypes.c_char_p]),
    ("tvm_library_detect", ctypes.c_int, [_P, ctypes.c_char_p, ctypes.POINTER(Package), ctypes.c_size_t,
                                          ctypes.POINTER(Result), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_library_detect_vulnerabilities", ctypes.c_int, [_P, ctypes.c_char_p, Str, Str, Str, ctypes.POINTER(Result),
                                                          ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_fill_info", ctypes.c_int, [_P, ctypes.POINTER(FillIn), ctypes.c_size_t, ctypes.POINTER(FillResult),
                                     ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_fill_result_free", None, [ctypes.POINTER(FillResult)]),
    ("tvm_match_fill", ctypes.c_int, [_P, _P, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_match_fill_fetch", ctypes.c_int, [_P, _P, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_match_fill_time", ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_char_p,
                                           ctypes.c_size_t]),
    ("tvm_match_fill_algorithmic_bytes", ctypes.c_uint64, [_P, _P]),
    ("tvm_fill_source_name", ctypes.c_char_p, [_P, ctypes.c_uint32]),
    ("tvm_match_filter", ctypes.c_int, [_P, _P, ctypes.POINTER(FilterOpts), ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_match_filter_fetch", ctypes.c_int, [_P, _P, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_match_filter_ignored", ctypes.c_int, [_P, _P, ctypes.c_void_p, ctypes.c_uint64,
                                                ctypes.POINTER(ctypes.c_uint64)]),
    ("tvm_vuln_rank_many", ctypes.c_int, [_P, ctypes.POINTER(Str), ctypes.c_size_t, ctypes.c_void_p]),
    ("tvm_batch_set_report", ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(Str),
                                            ctypes.POINTER(Str), ctypes.POINTER(Str)]),
    ("tvm_match_vulns", ctypes.c_int, [_P, _P, ctypes.POINTER(VulnSet), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_runtime_info", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_vuln_set_walk", ctypes.c_int, [ctypes.POINTER(VulnSet), _P, ctypes.c_void_p, ctypes.c_void_p]),
    ("tvm_pipeline_vulns", ctypes.c_int, [_P, _P, ctypes.POINTER(VulnSet), ctypes.c_char_p, ctypes.c_size_t]),
    ("tvm_vuln_set_free", None, [ctypes.POINTER(VulnSet)]),
    ("tvm_batch_report_get", ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(RawStr),
                                            ctypes.POINTER(RawStr), ctypes.POINTER(RawStr)]),
    ("tvm_match_filter_time", ctypes.c_int, [_P, _P, ctypes.POINTER(FilterOpts), ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_size_t]),
]

EXPORTED = [s[0] for s in _SIG]

_lib = None


def lib():
    """The loaded native library (raises if it is missing: no fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"trivy_amd native library not built: {LIB_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in _SIG:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        # drain the library's queues, join its worker threads and free its cached blocks while
        # the HIP runtime is still up (interpreter exit runs atexit before libraries unload)
        atexit.register(L.tvm_shutdown)
    return _lib


def s(x):
    """Python str/bytes -> tvm_str (keeps the bytes object alive on the struct)."""
    if x is None:
        return Str(None, 0)
    b = x.encode() if isinstance(x, str) else bytes(x)
    st = Str(b, len(b))
    st._keep = b
    return st


def errbuf():
    return ctypes.create_string_buffer(4096)


def runtime_info():
    """{"hip_runtime", "hip_driver", "libamdhip64"}: the HIP runtime libtrivy_amd's calls bind to
    (tvm_runtime_info; after `import torch` that is torch's bundled libamdhip64.so if torch
    loaded first - both carry the SONAME libamdhip64.so.7)."""
    rt, drv, path = ctypes.c_int(), ctypes.c_int(), ctypes.create_string_buffer(1024)
    lib().tvm_runtime_info(ctypes.byref(rt), ctypes.byref(drv), path, len(path))
    fmt = lambda v: f"{v // 10_000_000}.{v // 100_000 % 100}.{v % 100_000}"  # noqa: E731  HIP_VERSION encoding
    return {"hip_runtime": fmt(rt.value), "hip_driver": fmt(drv.value), "libamdhip64": path.value.decode()}

