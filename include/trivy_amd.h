/*
 * trivy_amd C-ABI: the drop-in boundary of the MI355X vulnerability-matching engine.
 *
 * This is the surface a cgo shim binds (INTEGRATION.md shows the Go side).  Plain
 * pointers and sizes only; no Go pointers are retained past a call (cgo rule); every
 * string/array returned is owned by the library and freed by the matching *_free call.
 *
 * Reference surfaces each entry point replaces (fwereade/trivy @ 2025-01-14):
 *   tvm_db_*                   trivy-db db.Init (pkg/commands/artifact/run.go:311) and the
 *                              per-call bucket reads behind <os>.VulnSrc.Get /
 *                              db.Config.GetAdvisories (used at pkg/detector/library/driver.go:114)
 *   tvm_engine_open/close      (new) device-resident tables, replaces the bbolt mmap
 *   tvm_engine_swap            server DB hot update (pkg/rpc/server/listen.go:154-190)
 *   tvm_ospkg_detect           ospkg.Detect            pkg/detector/ospkg/detect.go:63-82
 *   tvm_ospkg_driver_detect    ospkg.Driver.Detect     pkg/detector/ospkg/detect.go:57-60
 *   tvm_ospkg_is_supported     ospkg.Driver.IsSupportedVersion  detect.go:59
 *   tvm_batch_* / tvm_match_*  (new) many-target batching behind concurrent Detect calls
 *                              (pkg/k8s/scanner/scanner.go:141, pkg/rpc/server/server.go:45)
 *   tvm_fill_info              vulnerability.Client.FillInfo  pkg/vulnerability/vulnerability.go:60-109
 *                              (with getVendorSeverity :111-134 and getPrimaryURL :136-157)
 *   tvm_match_fill*            (new) FillInfo fused behind a batch's device-resident match list
 *   tvm_match_filter*          result.FilterResult's vulnerability part (pkg/result/filter.go:60-139:
 *                              severity / status / ignore-file IDs, dedup, BySeverity order) per
 *                              result of a batch
 *
 * Error convention: functions return 0 on success and a non-zero TVM_E* code on failure,
 * with a NUL-terminated message written to (err, errlen).  Messages carry the same text
 * the reference's errors do (e.g. "failed to get debian advisories: failed to unmarshal
 * advisory JSON: ...", wrapped "failed detection: ..." by tvm_ospkg_detect).
 */
#ifndef TRIVY_AMD_H
#define TRIVY_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TVM_ABI_VERSION 1

enum {
  TVM_OK = 0,
  TVM_EDETECT = 1,          /* detection failed (message in err) */
  TVM_EUNSUPPORTED_OS = 2,  /* ospkg.ErrUnsupportedOS (detect.go:30) */
  TVM_EINVAL = 3,
  TVM_EDEVICE = 4,          /* HIP / device failure; no CPU fallback exists */
  TVM_EUNSUPPORTED_TYPE = 5,/* library.NewDriver returned false (detect.go:12-15: nil, nil) */
};

typedef struct tvm_db tvm_db;
typedef struct tvm_engine tvm_engine;
typedef struct tvm_batch tvm_batch;

typedef struct {
  const char* p;
  size_t n;
} tvm_str;

/* ftypes.Package fields read by the detectors (pkg/fanal/types/artifact.go:68-105). */
typedef struct {
  tvm_str id, name, version, release, arch;
  int64_t epoch;
  tvm_str src_name, src_version, src_release;
  int64_t src_epoch;
  tvm_str modularitylabel;
  int32_t has_build_info;           /* BuildInfo != nil */
  const tvm_str* content_sets;      /* BuildInfo.ContentSets */
  size_t n_content_sets;
  tvm_str nvr, build_arch;          /* BuildInfo.Nvr, BuildInfo.Arch */
  tvm_str file_path;
} tvm_package;

/* ftypes.Repository (artifact.go:57-60); pass NULL for a nil *Repository. */
typedef struct {
  tvm_str family, release;
} tvm_repository;

/* copy_flags: which fields of input package pkg_index the driver copies verbatim. */
enum {
  TVM_COPY_PKG_ID = 1,
  TVM_COPY_PKG_NAME = 2,
  TVM_COPY_IDENTIFIER = 4, /* PkgIdentifier */
  TVM_COPY_LAYER = 8,      /* Layer */
};

/* types.DetectedVulnerability (pkg/types/vulnerability.go:9-31). Empty string = unset. */
typedef struct {
  uint32_t pkg_index;
  uint32_t copy_flags;
  const char* vulnerability_id;
  const char* const* vendor_ids;    /* NULL when nil */
  size_t n_vendor_ids;
  const char* pkg_id;
  const char* pkg_name;
  const char* pkg_path;
  const char* installed_version;
  const char* fixed_version;
  int32_t status;                   /* dbTypes.Status */
  const char* severity_source;      /* SeveritySource */
  const char* severity;             /* Vulnerability.Severity */
  int32_t has_data_source;          /* DataSource != nil */
  const char* data_source_id;
  const char* data_source_name;
  const char* data_source_url;
  const char* custom_json;          /* Custom as JSON text; NULL when nil */
} tvm_vuln;

typedef struct {
  tvm_vuln* vulns;
  size_t n;
  int32_t eosl;                     /* ospkg.Detect's second return value */
  void* priv;
} tvm_result;

/* ---- library ------------------------------------------------------------------------ */
const char* tvm_version(void);
int tvm_abi_version(void);

/* ---- advisory DB (host side) -------------------------------------------------------- */
tvm_db* tvm_db_new(void);
void tvm_db_free(tvm_db* db);
/* One bbolt record: bucket path (root bucket, nested buckets...) + key -> JSON value.
 * path has `depth` elements, the last being the key. */
int tvm_db_put(tvm_db* db, const tvm_str* path, size_t depth, const char* value, size_t vlen);
/* n records at once: paths is n*depth elements (row-major), values has n elements. */
int tvm_db_put_many(tvm_db* db, size_t n, const tvm_str* paths, size_t depth, const tvm_str* values);
/* n records from one byte arena: record r's path items and value are the (depth + 1)
 * slices off[r*(depth+1) + j], len[...] (j = depth is the value). */
int tvm_db_put_arena(tvm_db* db, size_t n, size_t depth, const char* arena, const uint64_t* off,
                     const uint32_t* len);
/* A bbolt file image (trivy.db as downloaded; the reference opens it with go.etcd.io/bbolt,
 * pkg/db/db.go:89-110): every record, (bucket path..., key) -> value, goes through
 * tvm_db_put.  Read-only walk of the current meta page's tree; a malformed file fails with
 * TVM_EINVAL and a message (records put before the failure stay). */
int tvm_db_put_bbolt(tvm_db* db, const void* bytes, size_t len, char* err, size_t errlen);
/* The same walk, reporting each record to `visit` (path = buckets + key, `depth` items);
 * a nonzero return from visit stops the walk (TVM_EINVAL). */
typedef int (*tvm_bbolt_visit)(void* ctx, const tvm_str* path, size_t depth, const char* value, size_t vlen);
int tvm_bbolt_walk(const void* bytes, size_t len, tvm_bbolt_visit visit, void* ctx, char* err, size_t errlen);
/* Decode + flatten into device images. Must be called once, before tvm_engine_open. */
int tvm_db_finalize(tvm_db* db, char* err, size_t errlen);
/* Statistics: [0] platforms [1] keys [2] advisories [3] interval rows [4] key-arena bytes */
void tvm_db_stats(const tvm_db* db, uint64_t out[5]);

/* ---- device engine -------------------------------------------------------------------- */
/* Uploads the finalized tables to HIP device `device`.  `db` must outlive the engine. */
tvm_engine* tvm_engine_open(tvm_db* db, int device, char* err, size_t errlen);
void tvm_engine_close(tvm_engine* e);
/* Atomically replaces the engine's tables (waits for in-flight calls; server hot update). */
int tvm_engine_swap(tvm_engine* e, tvm_db* db, char* err, size_t errlen);
uint64_t tvm_engine_table_bytes(const tvm_engine* e);
/* Drop-in path counters since open/swap: out3 = {launches, calls served, calls that shared
 * a launch with others}.  Concurrent driver calls (ospkg / library Detect) are coalesced
 * into one launch per batch of queued calls (twirp server.go:45, k8s scanner.go:141). */
int tvm_engine_dropin_stats(tvm_engine* e, uint64_t* out3);
/* Integrity check: re-reads every device table and compares it with the host image. */
int tvm_engine_verify(tvm_engine* e, char* err, size_t errlen);
/* Tuning knob: selects the match-kernel variant (tile size / LDS budget); returns the
 * previous one.  v < 0 only queries.  Names via tvm_variant_name (NULL past the last);
 * variant 0 = "auto" (default): the tuned variant for the batch's grammar set. */
int tvm_engine_set_variant(tvm_engine* e, int v);
const char* tvm_variant_name(int v);
/* Batches variant v runs: bit 0 dpkg-only, bit 1 OS grammars (dpkg / apk / rpm), bit 2 any
 * grammar; a launch of a variant not built for the batch fails with TVM_EDEVICE. */
int tvm_variant_grammar_sets(int v);
/* Variant index the engine's most recent launch ran (auto resolved); -1 before any. */
int tvm_engine_last_variant(tvm_engine* e);

/* ---- ospkg ------------------------------------------------------------------------------ */
/* ospkg.Detect: family = ftypes.OSType ("debian", "ubuntu", ...); now_unix = clock.Now(ctx).
 * Returns TVM_EUNSUPPORTED_OS for an unknown family. */
int tvm_ospkg_detect(tvm_engine* e, const char* os_family, const char* os_name, const tvm_repository* repo,
                     const tvm_package* pkgs, size_t n, int64_t now_unix, tvm_result* out, char* err,
                     size_t errlen);
/* Driver.Detect of drivers[os_family] (no gpg-pubkey filter, no EOSL, no wrapping). */
int tvm_ospkg_driver_detect(tvm_engine* e, const char* os_family, const char* os_ver, const tvm_repository* repo,
                            const tvm_package* pkgs, size_t n, int64_t now_unix, tvm_result* out, char* err,
                            size_t errlen);
/* Driver.IsSupportedVersion: 1 / 0, or -1 for an unsupported family. */
int tvm_ospkg_is_supported(const char* os_family, const char* os_ver, int64_t now_unix);
void tvm_result_free(tvm_result* r);

/* ---- library (language packages) ---------------------------------------------------------
 * pkg/detector/library: NewDriver (driver.go:25-93), (*Driver).DetectVulnerabilities
 * (driver.go:111-137) and Detect (detect.go:11-42).  lib_type is an ftypes.LangType
 * ("npm", "pip", "gomod", "jar", ...).  Unsupported types return TVM_EUNSUPPORTED_TYPE. */
/* Driver.Type(): the trivy-db ecosystem of lib_type, or NULL when NewDriver fails. */
const char* tvm_library_type(const char* lib_type);
/* library.Detect: packages use id, name, version, file_path (-> PkgPath); results carry
 * COPY_LAYER | COPY_IDENTIFIER.  Errors: "failed to scan <eco> vulnerabilities: ...". */
int tvm_library_detect(tvm_engine* e, const char* lib_type, const tvm_package* pkgs, size_t n, tvm_result* out,
                       char* err, size_t errlen);
/* Driver.DetectVulnerabilities(pkgID, pkgName, pkgVer): errors "failed to get <eco> advisories: ...". */
int tvm_library_detect_vulnerabilities(tvm_engine* e, const char* lib_type, tvm_str pkg_id, tvm_str pkg_name,
                                       tvm_str pkg_ver, tvm_result* out, char* err, size_t errlen);

/* ---- many-target batches (device-resident; bench + request coalescing) ---------------- */
tvm_batch* tvm_batch_new(void);
void tvm_batch_free(tvm_batch* b);
/* Adds one package under an explicit root bucket (e.g. "debian 12"), lookup name and the
 * formatted version the driver compares.  Returns the package's batch index. */
int64_t tvm_batch_add(tvm_batch* b, tvm_engine* e, const char* bucket, tvm_str name, tvm_str version);
/* tvm_batch_add_many plus the per-package attributes the rpm drivers filter on (the batch
 * form of what tvm_ospkg_detect derives from tvm_package): TVM_ATTR_ARCH takes one arch
 * string per package (rocky.go arch entries, redhat.go arch filter), TVM_ATTR_KSPLICE tags
 * each package with the ksplice token of its release (oracle.go:46-53, 77). */
enum { TVM_ATTR_ARCH = 1, TVM_ATTR_KSPLICE = 2, TVM_ATTR_CPESET = 4 };
int64_t tvm_batch_add_many_ex(tvm_batch* b, tvm_engine* e, const char* bucket, size_t n, const char* arena,
                              const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                              const uint32_t* ver_len, const uint64_t* arch_off, const uint32_t* arch_len,
                              uint32_t flags);
/* Red Hat: registers the CPE set of one (content sets, NVR) combination - redhat.go:112-120:
 * BuildInfo.ContentSets and "Nvr-Arch", or the release's default content sets and "" without
 * BuildInfo - resolved through the "Red Hat CPE" buckets; returns its id for TVM_ATTR_CPESET
 * (one per distinct combination, typically one per image), or -1. */
int64_t tvm_batch_cpe_set(tvm_batch* b, tvm_engine* e, const tvm_str* content_sets, size_t n, tvm_str nvr);
/* Optional per-package attribute columns of tvm_batch_add_many_attrs. */
typedef struct {
  const uint64_t* arch_off; /* TVM_ATTR_ARCH: arch string per package in the arena */
  const uint32_t* arch_len;
  const uint32_t* cpe_set;  /* TVM_ATTR_CPESET: tvm_batch_cpe_set id per package (Red Hat) */
} tvm_attr_cols;
/* tvm_batch_add_many plus attributes (the batch form of what tvm_ospkg_detect derives from
 * tvm_package): TVM_ATTR_ARCH (redhat.go:129-135 arch filter, rocky arch entries),
 * TVM_ATTR_KSPLICE (oracle.go:46-53, 77), TVM_ATTR_CPESET (the Red Hat CPE-set intersection of
 * trivy-db's redhat-oval Get).  The name is the lookup name the driver uses (Red Hat:
 * addModularNamespace, redhat.go:207-220). */
int64_t tvm_batch_add_many_attrs(tvm_batch* b, tvm_engine* e, const char* bucket, size_t n, const char* arena,
                                 const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                                 const uint32_t* ver_len, const tvm_attr_cols* attrs, uint32_t flags);
/* n packages of one bucket from a byte arena; returns the batch index of the first. */
int64_t tvm_batch_add_many(tvm_batch* b, tvm_engine* e, const char* bucket, size_t n, const char* arena,
                           const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                           const uint32_t* ver_len);
/* Many targets at once (a fleet's images / lockfiles, one Result each, as one
 * tvm_batch_add_many per target would add them): target t is packages [target_end[t-1],
 * target_end[t]) of the columns (target_end[-1] = 0), under root bucket buckets[t].  Returns
 * the batch index of the first package, -1 on bad arguments. */
int64_t tvm_batch_add_targets(tvm_batch* b, tvm_engine* e, size_t n_targets, const tvm_str* buckets,
                              const uint64_t* target_end, const char* arena, const uint64_t* name_off,
                              const uint32_t* name_len, const uint64_t* ver_off, const uint32_t* ver_len);
/* tvm_batch_add_targets with the rpm drivers' attributes (what tvm_batch_add_many_attrs adds
 * for one target): target_flags[t] = the TVM_ATTR_* bits of target t (NULL = none; KSPLICE
 * and CPESET exclusive), and the attribute columns per package (arch strings in the arena,
 * tvm_batch_cpe_set ids), read only for the packages of targets whose flags name them.  Both
 * calls fill the batch on the host threads (the package scanners of pkg/scanner/local/scan.go:
 * 170-194 hand packages over per target; here a fleet's targets arrive in one call). */
int64_t tvm_batch_add_targets_attrs(tvm_batch* b, tvm_engine* e, size_t n_targets, const tvm_str* buckets,
                                    const uint32_t* target_flags, const uint64_t* target_end, const char* arena,
                                    const uint64_t* name_off, const uint32_t* name_len, const uint64_t* ver_off,
                                    const uint32_t* ver_len, const tvm_attr_cols* attrs);
int64_t tvm_batch_size(const tvm_batch* b);
/* Copies the batch to the device and sizes the match buffer. */
int tvm_batch_upload(tvm_engine* e, tvm_batch* b, uint64_t match_cap, char* err, size_t errlen);
/* Enqueues one match pass on the engine stream (async). */
int tvm_match_launch(tvm_engine* e, tvm_batch* b, char* err, size_t errlen);
int tvm_engine_sync(tvm_engine* e, char* err, size_t errlen);
/* Waits for every stream of the library on `device` (hipDeviceSynchronize inside the library's
 * own HIP runtime instance) and reports any pending asynchronous error.  Test and health-check
 * hook; no reference counterpart. */
int tvm_device_sync(int device, char* err, size_t errlen);
/* Process teardown: drains the queues of every device an engine was opened on (a process that
 * opened none starts no HIP work here), joins the library's host worker threads and
 * frees its cached device / pinned blocks, so that nothing of the library's is left for the
 * HIP runtime's own teardown at exit.  Call once before the process exits (the Python
 * binding registers it with atexit); the library stays usable (later calls run without the
 * worker threads and without block caching).  No reference counterpart. */
void tvm_shutdown(void);
/* Total matches, first poisoned package (-1 none), internal error bits (read on the engine
 * stream, behind the batch's launches). */
int tvm_match_status(tvm_engine* e, tvm_batch* b, uint64_t* n_matches, int64_t* err_pkg, uint64_t* err_bits);
/* Copies up to cap pairs {pkg_index, advisory_index} (uint32 x2) to host in (package,
 * advisory) order.  TVM_EINVAL when the device match buffer overflowed (n_matches > the
 * upload's match_cap): re-upload with match_cap >= n_matches. */
int tvm_match_fetch(tvm_engine* e, tvm_batch* b, uint32_t* pairs, uint64_t cap, uint64_t* n_out);
/* Copies up to cap raw pairs device-to-device into dst (device memory on the engine's GPU):
 * package order within a tile, tiles in completion order (sort by (pkg, adv) to canonicalise).
 * For multi-GPU gathers that keep the match list off the host. */
int tvm_match_copy_device(tvm_engine* e, tvm_batch* b, void* dst, uint64_t cap, uint64_t* n_out);
/* The last pass's per-package advisory lists (CSR, (package, advisory) order) written into
 * caller-owned device buffers on the engine's GPU, then synchronised: package p's advisories
 * are csr_adv[row_end[p-1] .. row_end[p]) (row_end[-1] = 0; p counted from the batch's first
 * package, so a shard's offsets start at 0).  The ordered form a multi-GPU gather sends to the
 * root (4 B per match + 4 B per package), replacing the reference's per-target result slices
 * (pkg/scanner/local/scan.go:170-194 scanVulnerabilities collects them per target).  TVM_EINVAL when the pass
 * overflowed its match buffer or cap is below the match count (*n_out = the count). */
int tvm_match_order_into(tvm_engine* e, tvm_batch* b, void* csr_adv_dev, void* row_end_dev, uint64_t cap,
                         uint64_t* n_out, char* err, size_t errlen);
/* Times `steps` back-to-back launches with HIP events on the engine stream (ms total). */
int tvm_match_time(tvm_engine* e, tvm_batch* b, int steps, double* ms, char* err, size_t errlen);
/* Algorithmic bytes of one pass (DESIGN.md "roofline"), computed on the host from the batch. */
uint64_t tvm_match_algorithmic_bytes(tvm_engine* e, tvm_batch* b);
/* Host-side sort key of a version string (diagnostics/tests).  Grammars: 1 dpkg, 2 apk,
 * 3 rpm, 4 go-version, 5 npm, 6 PEP 440, 7 Maven, 8 RubyGems, 9 Bitnami.
 * Maven: the key the product compares, the version's numeric projection (only ever compared
 * with numeric bounds).
 * Returns the key length (<= cap bytes written) or -1 when the version does not parse. */
int tvm_version_key(int grammar, const char* s, size_t n, uint8_t* out, size_t cap);
/* Version class of a library grammar (npm: 1 pre-release; PEP 440: bits local/pre/post), -1 on error. */
int tvm_version_class(int grammar, const char* s, size_t n);
/* Host run of the match kernel's lane-serial dpkg key builder (verkey.h deb_fast_key) on
 * s placed `shift` (0..3) bytes past a dword boundary (tests: it must equal tvm_version_key
 * for the dpkg grammar).  Key length, -1 when the version does not parse, -2 when the
 * kernel hands the version to the generic encoder. */
int tvm_deb_fast_key_host(const char* s, size_t n, uint32_t shift, uint8_t* out, size_t cap);
/* Host-side compare.IsVulnerable through the load-time interval compiler (tests): 1/0, -1
 * when the advisory JSON does not decode.  Maven: the rows the product builds - intervals for
 * an advisory whose bounds are all numeric, else the pairwise program - so it mirrors the
 * device rows and is not ground truth for numeric-bound advisories; grammar |
 * TVM_ISVULN_PAIRWISE evaluates every Maven advisory with the pairwise ComparableVersion
 * program instead (tests check the two against each other and against the oracle). */
enum { TVM_ISVULN_PAIRWISE = 0x100 };
int tvm_lib_is_vulnerable_host(int grammar, const char* ver, size_t ver_len, const char* advisory_json,
                               size_t json_len);
/* Advisory fields for host-side inspection of batch results. */
const char* tvm_db_advisory_vuln_id(const tvm_db* db, uint32_t adv);

/* ---- multi-GPU sharding support ----------------------------------------------------------
 * Row counts (advisory intervals) of n packages of one bucket from the host index - the
 * pre-probe that balances a batch's shards by predicted work rather than by package count. */
int tvm_db_rows_many(const tvm_db* db, const char* bucket, size_t n, const char* arena, const uint64_t* name_off,
                     const uint32_t* name_len, uint32_t* out);
/* Adds `base` to the package index of every match the batch reports (a shard of a global
 * batch reports global indices); default 0. */
int tvm_batch_set_package_base(tvm_batch* b, uint32_t base);
/* tvm_batch_upload, but the match columns (package, advisory; uint32 each, cap entries) are
 * written into caller-owned device buffers on the engine's GPU (e.g. tensors a collective
 * then gathers); the batch never frees them. */
int tvm_batch_upload_into(tvm_engine* e, tvm_batch* b, void* pkg_dev, void* adv_dev, uint64_t cap, char* err,
                          size_t errlen);

/* ---- end-to-end pipelined pass ---------------------------------------------------------
 * The whole detector path for a host-side batch in one call: the batch goes to the GPU in
 * chunks (DMA from a pinned copy prepare builds on the host threads), each chunk is
 * matched as soon as it lands, and its per-package advisory lists come back (CSR) while
 * the next chunk is matched.  This is what a cgo caller pays per batch of targets
 * (detect.go:63 / library/detect.go:11 called for every target of a scan). */
/* Freezes the batch (no more adds afterwards) and sizes every device / pinned buffer (taken
 * from a process-wide block cache, so a fresh batch allocates nothing once one of its size has
 * run; host threads: TVM_HOST_THREADS, else OMP_NUM_THREADS, else all).  Unless
 * flags has TVM_PIPE_RAW, the batch travels in its transport form when it has one (every
 * name and version under 256 bytes, at most 255 platforms): each distinct name and each
 * distinct version string crosses the link once, packages carry references to them, and
 * the GPU rebuilds the batch's arrays chunk by chunk (one DMA per chunk). */
enum { TVM_PIPE_RAW = 1, TVM_PIPE_ADV32 = 2 };
int tvm_pipeline_prepare(tvm_engine* e, tvm_batch* b, uint64_t match_cap, uint32_t chunk_packages, uint32_t flags,
                         char* err, size_t errlen);
/* One pass; ms = wall time of the call.  TVM_EINVAL with *n_matches set when the matches do
 * not fit match_cap (prepare again with a larger one). */
int tvm_pipeline_run(tvm_engine* e, tvm_batch* b, uint64_t* n_matches, int64_t* err_pkg, double* ms, char* err,
                     size_t errlen);
/* The last pass's result (library-owned memory, valid until the next pass or
 * tvm_batch_free): package p's advisory indices are adv[row_end[p-1] .. row_end[p])
 * (row_end[-1] = 0), in (package, advisory) order.  When the DB has fewer than 2^24
 * advisories (and prepare had no TVM_PIPE_ADV32) the indices cross the link as 3 bytes
 * each; this call then widens them into a 4-byte array on the host once per pass. */
int tvm_pipeline_result(tvm_batch* b, const uint32_t** adv, const uint32_t** row_end, uint64_t* n_matches);
/* The result as it arrived in pinned host memory: index i is the `width`-byte (3 or 4)
 * little-endian integer at adv + width * i. */
int tvm_pipeline_result_raw(tvm_batch* b, const void** adv, uint32_t* width, const uint32_t** row_end,
                            uint64_t* n_matches);
/* [0] bytes the last pass copied host to device, [1] device to host, [2] chunks, [3] 1 when
 * the batch travels in its transport form, [4] prepare's host time building it (us). */
int tvm_pipeline_stats(tvm_batch* b, uint64_t out[5]);
/* The transport form prepare would build for n packages (platform ids as the batch holds
 * them, 0xFFFFFFFF = absent bucket), on the host alone (no device; test and inspection hook).
 * With out = NULL only the sizes are returned.  chunks: 10 values per
 * chunk {offset, bytes, name-ref / version-ref / lengths / platform / group-offset / attribute
 * section offsets, packages, groups}; plats: platform index -> platform id.  *bytes = 0:
 * the batch has no transport form. */
int tvm_wire_encode(size_t n, const uint32_t* plat, const char* arena, const uint64_t* name_off, const uint32_t* name_len,
                    const uint64_t* ver_off, const uint32_t* ver_len, uint32_t chunk_packages, int threads, void* out,
                    uint64_t cap, uint64_t* bytes,
                    uint64_t* chunks, uint64_t chunks_cap, uint64_t* n_chunks, uint32_t* plats, uint32_t plats_cap,
                    uint32_t* n_plats);
/* Host time of the last prepare (us): building the transport form, and the whole call. */
int tvm_pipeline_times(tvm_batch* b, uint64_t* encode_us, uint64_t* prepare_us);
/* The block cache behind batch buffers: {cached device bytes, cached pinned host bytes, hits,
 * misses}; tvm_pool_trim frees every cached block. */
void tvm_pool_stats(uint64_t out[4]);
void tvm_pool_trim(void);
/* The HIP runtime this library's calls bind to: hipRuntimeGetVersion / hipDriverGetVersion
 * and the path of the libamdhip64 that provides them (a host process that loaded another
 * libamdhip64.so.7 first - torch's bundled runtime - binds this library to that one). */
int tvm_runtime_info(int* hip_runtime, int* hip_driver, char* path, size_t pathlen);

/* ---- SBOM decode (the detector input of `trivy sbom`) ------------------------------------
 * Native CycloneDX JSON decode: pkg/sbom/cyclonedx/unmarshal.go:63-230 + pkg/sbom/io/decode.go:
 * 47-380 (the OS component, OS packages by the OS's dependencies or else of one PURL type,
 * applications by their Type property or one per language type, sorted).  The result holds
 * the detector input as tvm_package records (valid until tvm_sbom_free), ready for
 * tvm_ospkg_detect (app = -1) and tvm_library_detect (app = 0..n_apps-1). */
typedef struct tvm_sbom tvm_sbom;
/* flags: TVM_SBOM_BORROW = the result points into `text`, which must stay valid until
 * tvm_sbom_free (no copy of the document); else the document is copied. */
enum { TVM_SBOM_BORROW = 1 };
int tvm_sbom_decode_cyclonedx(const char* text, size_t len, uint32_t flags, tvm_sbom** out, char* err, size_t errlen);
void tvm_sbom_free(tvm_sbom* s);
int tvm_sbom_info(const tvm_sbom* s, int32_t* has_os, tvm_str* os_family, tvm_str* os_name, tvm_str* serial,
                  int64_t* version, size_t* n_apps);
/* app = -1: the OS packages (type / file_path empty); else application app's Type, FilePath
 * and libraries. */
int tvm_sbom_packages(const tvm_sbom* s, int64_t app, tvm_str* type, tvm_str* file_path, const tvm_package** pkgs,
                      size_t* n);
/* Fields of package i beyond tvm_package: PkgIdentifier (PURL, BOMRef), Layer (Digest, DiffID),
 * and which optional fields the SBOM set (bits: 1 Arch, 2 Epoch, 4 Release, 8 Modularitylabel,
 * 16 FilePath, 32 SrcName, 64 SrcVersion, 128 SrcRelease, 256 SrcEpoch, 512 Layer.Digest,
 * 1024 Layer.DiffID). */
typedef struct {
  tvm_str purl, bom_ref, layer_digest, layer_diff_id;
  uint32_t present;
} tvm_sbom_extra;
int tvm_sbom_package_extra(const tvm_sbom* s, int64_t app, size_t i, tvm_sbom_extra* out);

/* ---- Red Hat on the batch path ----------------------------------------------------------
 * After tvm_match_launch (+ sync): the Red Hat driver's epilogue for every package of the
 * batch's "Red Hat"-bucket targets at once - the per-CVE merge of redhat.go:146-187 (first
 * advisory of a VulnerabilityID gives Status / Severity; fixed advisories union their
 * VendorIDs and raise FixedVersion to the greatest rpm version; sorted by VulnerabilityID per
 * package) grouped on the GPU.  Vulns carry pkg_index = batch index, InstalledVersion = the
 * batch version, copy flags PKG_ID | PKG_NAME | IDENTIFIER | LAYER (the caller copies them from
 * its package, whose Name is the plain name, not the modular lookup name). */
int tvm_match_redhat_result(tvm_engine* e, tvm_batch* b, tvm_result* out, char* err, size_t errlen);
/* Enqueues the same per-CVE merge on the engine stream (no host round trip) and makes the
 * MERGED list the batch's match list: from here until the next tvm_match_launch, the pairs
 * of tvm_match_status / _fetch / _fill / _fill_fetch / _filter are, for Red Hat packages,
 * one {package, advisory} per (package, VulnerabilityID) in VulnerabilityID order, where the
 * advisory is the representative member (the one with the greatest FixedVersion when any
 * member is fixed - its FixedVersion is the merged one - else the first); the first member
 * still supplies Status and Severity to FillInfo (redhat.go:140-171 -> vulnerability.go:60).
 * Pairs of other drivers' packages are unchanged.  This is the reference's order of work:
 * DetectVulnerabilities (merged) -> FillInfo -> result.Filter, all on the device. */
int tvm_match_redhat_merge(tvm_engine* e, tvm_batch* b, char* err, size_t errlen);
/* After tvm_match_redhat_merge (+ sync): the merged Red Hat vulnerabilities of the listed
 * {package, advisory} pairs (e.g. tvm_match_filter_fetch's survivors), as
 * tvm_match_redhat_result builds them; pairs of other drivers are skipped. */
int tvm_match_redhat_vulns(tvm_engine* e, tvm_batch* b, const uint32_t* pairs, uint64_t n, tvm_result* out,
                           char* err, size_t errlen);
/* Times `steps` back-to-back merges on the engine stream with HIP events (ms total); leaves
 * the batch on its merged list. */
int tvm_match_redhat_merge_time(tvm_engine* e, tvm_batch* b, int steps, double* ms, char* err, size_t errlen);

/* ---- DetectedVulnerability sets of a batch ----------------------------------------------
 * The drivers' epilogues on the batch path: what Driver.Detect returns per target
 * (debian.go:78-98, ubuntu.go:99-108, alpine.go:94-101, alma.go:64-71, rocky.go:69-76,
 * oracle.go:70-80, redhat.go:140-187, mariner.go:50-70, ..., library/driver.go:125-132 +
 * detect.go:33-37), for every match of a batch at once.  A DetectedVulnerability is split in
 * two parts:
 *   - its record (tvm_vuln without the package fields): VulnerabilityID, VendorIDs,
 *     FixedVersion (rpm Version.String() for the drivers that print it, createFixedVersions for
 *     libraries), Status, SeveritySource / Severity, DataSource, Custom, and copy_flags (which
 *     fields the caller copies from its package: PkgID, PkgName, PkgIdentifier, Layer).  Record
 *     r < n_adv_recs is advisory r's, as its driver populates it (shared by every package that
 *     matches it, built once per DB); r >= n_adv_recs is grp_recs[r - n_adv_recs], a Red Hat
 *     group of several advisories of one VulnerabilityID merged per redhat.go:146-187;
 *   - its package: InstalledVersion and PkgPath of the batch package (tvm_batch_report_get),
 *     PkgID / PkgName / PkgIdentifier / Layer from the caller's own package per copy_flags.
 * The set is per-package lists (CSR) of record indices, in pinned memory as the device wrote
 * them (3-byte indices while the records number below 2^24), so no per-match host pass is
 * needed to hand it on.  Order: by package, then as the driver reports them (advisory order;
 * Red Hat: VulnerabilityID order).  Library-owned; free with tvm_vuln_set_free. */
typedef struct {
  const uint32_t* row_end;       /* package first_pkg + p has DetectedVulnerabilities [row_end[p-1], row_end[p])
                                    (row_end[-1] = 0), p < n_pkgs */
  size_t n_pkgs;
  uint32_t first_pkg;            /* batch index of row_end's package 0 (tvm_batch_set_package_base) */
  const uint8_t* rec;            /* n record indices, rec_width (3 or 4) little-endian bytes each */
  uint32_t rec_width;
  size_t n;
  const tvm_vuln* adv_recs;      /* one per DB advisory (pkg_index 0; package fields "") */
  size_t n_adv_recs;
  const tvm_vuln* grp_recs;      /* merged Red Hat groups: record n_adv_recs + k */
  size_t n_grp_recs;
  void* priv;
} tvm_vuln_set;
/* After tvm_match_launch: the batch's DetectedVulnerability set.  Batches with Red Hat packages
 * are merged on the device first (tvm_match_redhat_merge, if it has not run).  TVM_EINVAL when
 * the pass overflowed its match buffer, met an undecodable advisory or flagged an error. */
int tvm_match_vulns(tvm_engine* e, tvm_batch* b, tvm_vuln_set* out, char* err, size_t errlen);
/* The same from the last completed tvm_pipeline_run (TVM_EINVAL before one).  Batches without
 * Red Hat packages: the lists that pass left in pinned memory, no copy - the set is invalidated
 * by the next tvm_pipeline_prepare / tvm_pipeline_run / tvm_batch_free of the batch.  Batches
 * with Red Hat packages: the per-CVE merge (redhat.go:146-187) and the export run on the device
 * over the pass's match list (still in HBM), and the set owns its lists (valid until
 * tvm_vuln_set_free). */
int tvm_pipeline_vulns(tvm_engine* e, tvm_batch* b, tvm_vuln_set* out, char* err, size_t errlen);
void tvm_vuln_set_free(tvm_vuln_set* s);
/* A consumer of a set, natively (INTEGRATION.md §3's loop on the host threads): every
 * DetectedVulnerability's record index decoded, its record resolved (adv_recs / grp_recs) and
 * its value fields read (the string pointers are handed on, as the loop copies the record), its
 * package's InstalledVersion located in the batch (tvm_batch_report_get).  n_out =
 * DetectedVulnerabilities walked; digest = the wrapping sum over them of fmix64(p *
 * 0x9E3779B97F4A7C15 + r * 0xC2B2AE3D27D4EB4F + (|InstalledVersion| << 40) + (status << 32) +
 * (n_vendor_ids << 24) + (has_data_source << 8) + copy_flags), each field's low byte, p =
 * first_pkg + the package's batch index, r = the record index - what a caller's own loop over
 * the set costs, and a check that it saw every entry (bench.py end_to_end consume_ms). */
int tvm_vuln_set_walk(const tvm_vuln_set* s, const tvm_batch* b, uint64_t* n_out, uint64_t* digest);
/* The package side of packages [first, first + n): names = the tvm_batch_set_report PkgName
 * (p = NULL: the caller's package Name), versions = InstalledVersion (the report's, else the
 * batch version, which is FormatVersion of the package for every driver comparing the binary
 * version), paths = PkgPath (report, else empty).  Views into the batch (valid until it changes);
 * NULL arrays are skipped. */
int tvm_batch_report_get(const tvm_batch* b, uint64_t first, uint64_t n, tvm_str* names, tvm_str* versions,
                         tvm_str* paths);

/* ---- vulnerability detail: FillInfo ------------------------------------------------ */
/* One detected vulnerability as FillInfo reads it (vulnerability.go:60-109). */
typedef struct {
  tvm_str vulnerability_id;
  tvm_str data_source_id;       /* DataSource.ID; empty when DataSource is nil */
  tvm_str severity_source;      /* SeveritySource the detector set; empty = none */
  tvm_str severity;             /* Vulnerability.Severity the detector set (read with severity_source) */
  int32_t status;               /* Status the detector set (dbTypes.Status) */
  int32_t has_fixed_version;    /* FixedVersion != "" */
} tvm_fill_in;
/* What FillInfo writes back.  When !found (trivy-db GetVulnerability failed: unknown ID or
 * undecodable record; the reference logs and skips, :72-76) only status changed and the
 * other fields are "" / NULL. */
typedef struct {
  int32_t found;
  int32_t status;                    /* Status */
  const char* severity;              /* Vulnerability.Severity */
  const char* severity_source;       /* SeveritySource */
  const char* primary_url;           /* PrimaryURL */
  const char* vulnerability_json;    /* the Vulnerability as JSON (trivy-db types.Vulnerability
                                        fields, omitempty; VendorSeverity includes the detector's
                                        package-specific entry, :95-101); NULL when !found */
} tvm_fill_out;
typedef struct {
  tvm_fill_out* items;
  size_t n;
  void* priv;
} tvm_fill_result;
/* Client.FillInfo over n detected vulnerabilities: decisions on the GPU (one launch), the
 * strings rebuilt on the host.  Thread-safe. */
int tvm_fill_info(tvm_engine* e, const tvm_fill_in* in, size_t n, tvm_fill_result* out, char* err, size_t errlen);
void tvm_fill_result_free(tvm_fill_result* r);
/* Batch path: enqueue FillInfo over the batch's device match list right behind
 * tvm_match_launch (same stream, no host round trip); each (package, advisory) pair is
 * filled as its driver's Detect would have populated it - after tvm_match_redhat_merge, a
 * Red Hat pair as its merged DetectedVulnerability (Status / Severity of the first member,
 * FixedVersion of the representative). */
int tvm_match_fill(tvm_engine* e, tvm_batch* b, char* err, size_t errlen);
/* After sync: per pair, in tvm_match_fetch order, 4 uint32: {vulnerability record
 * (0xFFFFFFFF = not found), status, severity code
 * (0..4 SeverityNames; 0xFFFD detector's; 0xFFFE DB string; 0xFFFF out of range) |
 * severity-source id << 16 (0xFFFF = none), primary URL kind << 28 | reference index}. */
int tvm_match_fill_fetch(tvm_engine* e, tvm_batch* b, uint32_t* out4, uint64_t cap, uint64_t* n_out);
/* Times `steps` back-to-back tvm_match_fill launches (ms total); needs a completed match. */
int tvm_match_fill_time(tvm_engine* e, tvm_batch* b, int steps, double* ms, char* err, size_t errlen);
/* Algorithmic bytes of one tvm_match_fill pass over the batch's current match list. */
uint64_t tvm_match_fill_algorithmic_bytes(tvm_engine* e, tvm_batch* b);
/* Name of a severity-source id from tvm_match_fill_fetch ("" for 0xFFFF / unknown). */
const char* tvm_fill_source_name(tvm_engine* e, uint32_t id);

/* ---- result.Filter over a batch -------------------------------------------------------- */
/* One tvm_batch_add* call = one Result.  A package's DetectedVulnerability PkgName /
 * InstalledVersion / PkgPath are its batch (name, version) and "" unless
 * tvm_batch_set_report names others for packages [first, first + n): Debian / Ubuntu report
 * the binary package and FormatVersion while they match on the source package
 * (debian.go:66-83), library packages carry a PkgPath (filter.go:124 dedup key, BySeverity's
 * last key).  NULL arrays keep the defaults.  Replaces the filter's package layout. */
int tvm_batch_set_report(tvm_batch* b, uint64_t first, uint64_t n, const tvm_str* names, const tvm_str* versions,
                         const tvm_str* paths);

/* Ignore-file findings compiled against the batch by the host (trivy_amd/ignore.py; the
 * reference's IgnoreConfig.MatchVulnerability, ignore.go:86-161).  Rules name a
 * vulnerability by index into ids and carry the precedence of the finding they came from,
 * pass << 31 | finding index (pass 0: the finding has no paths or one matched the result's
 * Target; pass 1: one matched the package's PkgPath): a pair several rules hit is ignored by
 * the smallest, which is the finding MatchVulnerability returns. */
typedef struct {
  const tvm_str* ids;            /* distinct vulnerability IDs */
  size_t n_ids;
  const uint32_t* id_ranks;      /* optional: tvm_vuln_rank_many of ids (same engine, no swap
                                    since), so a call ranks no strings */
  const uint32_t* all_id;        /* rules for every package */
  const uint32_t* all_prec;
  size_t n_all;
  const uint32_t* pkg_pkg;       /* rules for one package (PURL-scoped findings whose PURL */
  const uint32_t* pkg_id;        /* matches that package's) */
  const uint32_t* pkg_prec;
  size_t n_pkg;
  const uint32_t* pkg_class;     /* per batch package: its class (NULL: no class rules) */
  const uint32_t* cls_class;     /* rules for every package of one class (PURL-scoped */
  const uint32_t* cls_id;        /* findings on packages without a PURL, matchPURL */
  const uint32_t* cls_prec;      /* ignore.go:116-126; path-scoped findings by Target / */
  size_t n_cls;                  /* PkgPath) */
} tvm_ignore_rules;

typedef struct {
  uint32_t severity_mask;        /* bit i: SeverityNames[i] is in FilterOption.Severities (i <= 4) */
  uint32_t ignore_status_mask;   /* bit s: dbTypes.Status s is in FilterOption.IgnoreStatuses */
  const tvm_ignore_rules* ignore;  /* NULL: no ignore file */
  /* VEX suppressions (pkg/vex, applied after the dedup as filter.go:51-53 filterByVEX does):
   * entry k drops package vex_pkgs[k]'s finding of vulnerability vex_ids[vex_id_index[k]].
   * The host compiles a VEX document against the batch's package PURLs into these entries
   * (trivy_amd/vex.py: OpenVEX openvex.go:21-54, CycloneDX cyclonedx.go:48-84, CSAF
   * csaf.go:27-83); the per-finding test runs on the GPU.  n_vex = 0: no VEX document. */
  const uint32_t* vex_pkgs;
  const uint32_t* vex_id_index;
  size_t n_vex;
  const tvm_str* vex_ids;        /* distinct vulnerability IDs */
  size_t n_vex_ids;
  const uint32_t* vex_id_ranks;  /* optional: tvm_vuln_rank_many of vex_ids */
} tvm_filter_opts;
/* The filter's rank of each vulnerability ID (byte order among the DB's advisory IDs;
 * 0xFFFFFFFF: no advisory has it), computed once when a VEX document or ignore file is
 * compiled for a batch.  Ranks belong to the engine's current DB. */
int tvm_vuln_rank_many(tvm_engine* e, const tvm_str* ids, size_t n, uint32_t* ranks);
/* filterVulnerabilities + sort.Sort(BySeverity) (+ the VEX filter) for every result of the
 * batch, on the GPU, after tvm_match_launch + tvm_match_fill.  n_kept = surviving
 * vulnerabilities, n_ignored = findings the ignore file dropped (ModifiedFindings).
 * Not for a batch with a package base (a shard): results must be whole. */
int tvm_match_filter(tvm_engine* e, tvm_batch* b, const tvm_filter_opts* o, uint64_t* n_kept, uint64_t* n_ignored,
                     char* err, size_t errlen);
/* The surviving {package, advisory} pairs (uint32 x2) in report order: results in add
 * order, each in BySeverity order. */
int tvm_match_filter_fetch(tvm_engine* e, tvm_batch* b, uint32_t* pairs, uint64_t cap, uint64_t* n_out);
/* The ignored findings as {package, advisory, finding index} (uint32 x3) in detection
 * order (results in add order, each in its Vulnerabilities order): result.ModifiedFindings
 * with status "ignored" and the finding's Statement (filter.go:117-122). */
int tvm_match_filter_ignored(tvm_engine* e, tvm_batch* b, uint32_t* triples, uint64_t cap, uint64_t* n_out);
/* Wall time of `steps` tvm_match_filter calls (ms total; each call synchronises once). */
int tvm_match_filter_time(tvm_engine* e, tvm_batch* b, const tvm_filter_opts* o, int steps, double* ms, char* err,
                          size_t errlen);

#ifdef __cplusplus
}
#endif
#endif /* TRIVY_AMD_H */
