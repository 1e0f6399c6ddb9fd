// Load-time compilation of library advisories into interval rows (host only).
//
// compare.IsVulnerable (reference pkg/detector/library/compare/compare.go:21-55) over one
// advisory is, for a fixed grammar, a set of installed versions.  Every constraint
// primitive of the six grammars is an interval of that grammar's sort-key order (libver.h)
// within a version class, so the set is computed once here as a union of disjoint
// intervals per class - (Vulnerable) minus (Patched or Unaffected) - and each interval
// becomes one row.  The kernel then tests an installed key against rows exactly as for
// the OS drivers; disjointness guarantees at most one match per advisory.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace tvm {

// One interval of the key order: lo/hi bounds (inf = unbounded) with inclusivity.
struct KBound {
  bool inf = true;
  std::string k;
  bool incl = false;
};
struct KInterval {
  KBound lo, hi;
};
using KSet = std::vector<KInterval>;  // sorted, disjoint, non-empty intervals

// A compiled advisory: either "always" (an empty constraint string: reported even for an
// unparsable installed version, compare.go:23-28) or per-class interval sets.
struct LibRows {
  bool ok = false;      // the constraints compiled (false: cls holds nothing)
  bool always = false;
  int ncls = 1;
  std::vector<KSet> cls;  // ncls entries
};

// Maven advisories as IsVulnerable programs (libver.h mvn_program_eval): ALWAYS (an empty
// constraint string), NEVER (unparsable / nothing to match) or a program in `words`.
enum MvnProgState { MVN_NEVER = 0, MVN_ALWAYS = 1, MVN_PROGRAM = 2 };
// Every bound text of the advisory's constraints is numeric (libver.h mvn_numeric).
bool mvn_bounds_numeric(const std::vector<std::string>& vulnerable, const std::vector<std::string>& patched,
                        const std::vector<std::string>& unaffected);
MvnProgState mvn_program(const std::vector<std::string>& vulnerable, const std::vector<std::string>& patched,
                         const std::vector<std::string>& unaffected, std::vector<uint32_t>& words);
// The advisory is a program whose bounds are all numeric and compile: it is matched as
// key-order intervals over the installed version's numeric projection (libver.h
// mvn_numeric_projection), exact for every installed version; DB::compile_rows builds no
// program row for it.
bool mvn_hybrid(const std::vector<std::string>& vulnerable, const std::vector<std::string>& patched,
                const std::vector<std::string>& unaffected);
// compare.IsVulnerable for the Maven grammar, pairwise (host): 1 / 0.
int mvn_is_vulnerable(const std::vector<std::string>& vulnerable, const std::vector<std::string>& patched,
                      const std::vector<std::string>& unaffected, const std::string& installed);

// Number of version classes of a grammar (libver.h class bits).
int lib_classes(uint8_t cmp);

// matchVersion's constraint parse + evaluation as a set; false on a parse error.
bool lib_compile_constraint(uint8_t cmp, const std::string& constraint, std::vector<KSet>& out);

// compare.IsVulnerable as a set (parse errors -> the empty set).
LibRows lib_compile_advisory(uint8_t cmp, const std::vector<std::string>& vulnerable,
                             const std::vector<std::string>& patched, const std::vector<std::string>& unaffected);

// Host evaluation (tests and diagnostics): does the installed version fall in the rows?
bool lib_rows_contain(uint8_t cmp, const LibRows& r, const std::string& installed);

}  // namespace tvm
