// Host-sanitizer driver for the native CSV parser (csrc/host/csv_parser.cpp).
// Built with -fsanitize=address,undefined by tools/sanitize/run.sh; parses every
// file given on the command line with 1 and N threads, then a few thousand
// random / truncated / quote-heavy buffers, and checks that the threaded result
// equals the single-threaded one.  GPU-side ASan is not available on the pool.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <string>

#include "../../csrc/host/csv_parser.h"

static int g_fail = 0;

static void check_same(const har::CsvResult& a, const har::CsvResult& b, const char* what) {
  bool ok = a.nrows == b.nrows && a.ncols == b.ncols && a.kinds == b.kinds && a.names == b.names;
  for (int c = 0; ok && c < a.ncols; ++c)
    for (int64_t r = 0; ok && r < a.nrows; ++r) {
      ok = a.field(c, r) == b.field(c, r) && a.missing[c][r] == b.missing[c][r];
      if (ok && a.kinds[c] == "double") {
        double x = a.doubles[c][r], y = b.doubles[c][r];
        ok = (x == y) || (x != x && y != y);
      }
    }
  if (!ok) {
    std::fprintf(stderr, "MISMATCH threads=1 vs threads=N on %s\n", what);
    ++g_fail;
  }
}

static void run(const std::string& buf, const char* what) {
  for (bool header : {true, false}) {
    auto a = har::parse_csv(buf.data(), buf.size(), header, 1);
    auto b = har::parse_csv(buf.data(), buf.size(), header, 7);
    check_same(a, b, what);
  }
}

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    std::string s = ss.str();
    run(s, argv[i]);
    for (size_t cut : {size_t(1), s.size() / 3, s.size() / 2, s.size() - 1})  // truncated inputs
      if (cut < s.size()) run(s.substr(0, cut), "truncated");
  }
  std::mt19937 rng(1234);
  const char alphabet[] = "0123456789.,-+eE\"\n\r abcNaN?";
  for (int it = 0; it < 3000; ++it) {
    size_t n = rng() % 600;
    std::string s = "a,b,c\n";
    for (size_t k = 0; k < n; ++k) s.push_back(alphabet[rng() % (sizeof(alphabet) - 1)]);
    run(s, "random");
  }
  std::printf("csv sanitizer run: %s\n", g_fail ? "FAIL" : "OK");
  return g_fail ? 1 : 0;
}
