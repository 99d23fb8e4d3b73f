// Host-only robustness harness for the GraphDef wire codec, meant to be built
// with AddressSanitizer + UndefinedBehaviorSanitizer (scripts/sanitize_host.sh).
//
// GraphDefs are untrusted input (files, bytes from users), so the decoder
// must reject malformed data with a GraphError, never read out of bounds.
// The harness (1) round-trips the fixture GraphDefs and checks the bytes are
// stable, (2) decodes deterministic mutations of them: bit flips, truncations,
// random byte runs, varint-length corruption.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../proto/graphdef.h"

using namespace tfa;

static std::string read_file(const char* path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", path);
    std::exit(2);
  }
  std::ostringstream os;
  os << f.rdbuf();
  return os.str();
}

static int decode(const std::string& b, int64_t& ok, int64_t& rejected) {
  try {
    GraphDef g = parse_graphdef(b);
    // touch everything the importer reads
    size_t n = 0;
    for (auto& nd : g.nodes) n += nd.name.size() + nd.op.size() + nd.inputs.size() + nd.attr.size();
    std::string again = serialize_graphdef(g);
    GraphDef g2 = parse_graphdef(again);  // re-encoded output must decode
    if (g2.nodes.size() != g.nodes.size()) {
      std::fprintf(stderr, "re-encode changed the node count\n");
      return 1;
    }
    (void)n;
    ++ok;
  } catch (const GraphError&) {
    ++rejected;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s ITERATIONS graph.pb [graph.pb...]\n", argv[0]);
    return 2;
  }
  const long iters = std::atol(argv[1]);
  std::mt19937_64 rng(12345);
  int64_t ok = 0, rejected = 0;
  for (int a = 2; a < argc; ++a) {
    std::string base = read_file(argv[a]);
    GraphDef g = parse_graphdef(base);
    std::string rt = serialize_graphdef(g);
    if (serialize_graphdef(parse_graphdef(rt)) != rt) {
      std::fprintf(stderr, "%s: round trip is not stable\n", argv[a]);
      return 1;
    }
    for (long i = 0; i < iters; ++i) {
      std::string m = base;
      switch (i % 4) {
        case 0: {  // bit flips
          int flips = 1 + static_cast<int>(rng() % 4);
          for (int k = 0; k < flips && !m.empty(); ++k) m[rng() % m.size()] ^= static_cast<char>(1u << (rng() % 8));
          break;
        }
        case 1:  // truncation
          m.resize(rng() % (m.size() + 1));
          break;
        case 2: {  // random run
          size_t at = m.empty() ? 0 : rng() % m.size();
          size_t len = 1 + rng() % 16;
          for (size_t k = 0; k < len && at + k < m.size(); ++k) m[at + k] = static_cast<char>(rng());
          break;
        }
        default: {  // huge varint lengths
          size_t at = m.empty() ? 0 : rng() % m.size();
          std::string v = "\xff\xff\xff\xff\x0f";
          m.insert(at, v);
          break;
        }
      }
      if (decode(m, ok, rejected)) return 1;
    }
  }
  std::printf("proto_fuzz: %lld decoded, %lld rejected, no sanitizer findings\n", (long long)ok,
              (long long)rejected);
  return 0;
}
