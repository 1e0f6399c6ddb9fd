// ThreadSanitizer harness (tools/san/run.sh): the host threads of the library's batch
// preparation, without a GPU - (1) the parallel wire encoder (wire.cpp) at 8 threads against
// 1 thread, byte for byte; (2) the process-wide WorkerPool (host_par.h) driven by two caller
// threads at once (jobs serialise on the pool), then shut down (tvm_shutdown's path) with a job
// after it running inline; (3) the CycloneDX decoder's parallel pieces (sbom.cpp) at 8 threads
// against 1.  Exit 0 = every comparison equal (TSan halts on the first race).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "host_par.h"
#include "sbom.h"
#include "wire.h"

using namespace tvm;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

static std::vector<uint8_t> encode(const HostBatch& hb, int threads) {
  std::vector<uint64_t> toff(hb.tile_off.begin(), hb.tile_off.end());
  toff.resize(size_t(hb.n_tiles()) * kGroupsPerTile + 1, hb.arena.size());
  std::vector<uint32_t> bounds;
  for (uint32_t t = 0; t < hb.n_tiles(); t += 37) bounds.push_back(t);  // chunks of 37 tiles
  bounds.push_back(hb.n_tiles());
  WireEncoder enc;
  std::string err;
  if (!enc.plan(hb, toff, bounds, threads, err)) return {};
  std::vector<uint8_t> out(enc.bytes());
  enc.emit(out.data());
  return out;
}

int main() {
  // (1) wire encoder
  std::mt19937_64 rng(7);
  HostBatch hb;
  std::vector<std::string> names, vers;
  for (int i = 0; i < 5000; i++) names.push_back("pkg-" + std::to_string(rng() % 100000));
  for (int i = 0; i < 3000; i++) vers.push_back(std::to_string(rng() % 9) + "." + std::to_string(rng() % 50) + "-" + std::to_string(rng() % 7));
  for (int i = 0; i < 300000; i++)
    hb.add(uint32_t(rng() % 5), names[rng() % names.size()], vers[rng() % vers.size()]);
  const std::vector<uint8_t> w1 = encode(hb, 1), w8 = encode(hb, 8);
  if (w1.empty() || w1 != w8) return fail("wire encoder: 8 threads differ from 1");
  std::printf("wire encoder: %zu packages, %zu bytes, 1 == 8 threads\n", hb.size(), w1.size());

  // (2) the worker pool from two callers at once, then shutdown
  std::atomic<int> bad{0};
  auto caller = [&](int seed) {
    for (int job = 0; job < 200; job++) {
      std::vector<uint64_t> v(1000 + seed * 7 + job, 0);
      WorkerPool::get().parallel_for(v.size(), [&](size_t i) { v[i] = i * i + uint64_t(seed); });
      for (size_t i = 0; i < v.size(); i++)
        if (v[i] != i * i + uint64_t(seed)) bad++;
    }
  };
  std::thread a(caller, 1), b(caller, 2);
  a.join();
  b.join();
  if (bad) return fail("worker pool: wrong results");
  std::vector<uint64_t> s(64, 0);
  pool_range_for(s.size(), 1, [&](size_t x, size_t y) {
    for (size_t i = x; i < y; i++) s[i] = i + 1;
  });
  WorkerPool::shutdown_all();
  std::vector<int> after(100, 0);
  WorkerPool::get().parallel_for(after.size(), [&](size_t i) { after[i] = int(i); });  // runs inline
  for (size_t i = 0; i < after.size(); i++)
    if (after[i] != int(i) || s[i % 64] != i % 64 + 1) return fail("worker pool after shutdown");
  std::printf("worker pool: 2 callers x 200 jobs, shutdown, inline job: ok\n");

  // (3) CycloneDX decode in parallel pieces
  std::string doc = R"({"bomFormat":"CycloneDX","specVersion":"1.5","serialNumber":"urn:uuid:1","version":1,)"
                    R"("metadata":{"component":{"bom-ref":"root","type":"container","name":"img"}},"components":[)";
  doc += R"({"bom-ref":"os","type":"operating-system","name":"debian","version":"12.4"})";
  for (int i = 0; i < 40000; i++) {
    const std::string n = "lib" + std::to_string(i % 9000), v = "1." + std::to_string(i % 31) + "-" + std::to_string(i % 5);
    doc += R"(,{"bom-ref":"pkg:deb/debian/)" + n + "@" + v + "?arch=amd64&distro=debian-12.4\",\"type\":\"library\",\"name\":\"" +
           n + "\",\"version\":\"" + v + R"(","purl":"pkg:deb/debian/)" + n + "@" + v +
           R"(?arch=amd64&distro=debian-12.4","properties":[{"name":"aquasecurity:trivy:SrcName","value":")" + n +
           R"("},{"name":"aquasecurity:trivy:PkgType","value":"debian"}]})";
  }
  doc += R"(],"dependencies":[{"ref":"root","dependsOn":["os"]}]})";
  std::vector<std::string> dumps;
  for (const char* t : {"1", "8"}) {
    setenv("TVM_HOST_THREADS", t, 1);
    Sbom sb;
    std::string err;
    if (!decode_cyclonedx(doc, sb, err)) return fail(("sbom decode: " + err).c_str());
    std::string d;
    for (size_t i = 0; i < sb.view.size(); i++) {
      const tvm_package& p = sb.view[i];
      d.append(p.name.p, p.name.n).append("|").append(p.version.p, p.version.n).append("|");
      d.append(p.src_name.p ? p.src_name.p : "", p.src_name.n).append("\n");
    }
    dumps.push_back(d);
  }
  if (dumps[0].empty() || dumps[0] != dumps[1]) return fail("sbom decode: 8 threads differ from 1");
  std::printf("sbom decode: %zu bytes of text, 1 == 8 threads\n", doc.size());
  std::printf("tsan harness: ok\n");
  return 0;
}
