// Multi-threaded CSV tokenizer + number parser + Spark-style type votes.
//
// Host half of the columnar ETL that replaces Spark's CSV data source
// (reference: Main/main.py:18-20).  Three passes:
//   1. line index: each thread scans a byte range for '\n' (CRLF tolerated),
//   2. field split + parse: rows are distributed over threads; every field is
//      classified (empty / int literal / float literal / other) and parsed,
//   3. per-column votes are merged -> int | long | double | string.
// Quoted fields ("a,b" and "" escapes) are supported.
#include "csv_parser.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace har {
namespace {

inline bool is_int_literal(const char* s, size_t n) {
  size_t i = 0;
  if (n == 0) return false;
  if (s[0] == '+' || s[0] == '-') i = 1;
  if (i == n) return false;
  for (; i < n; ++i)
    if (s[i] < '0' || s[i] > '9') return false;
  return true;
}

// Decimal/float literal: [+-]? (digits [. digits?] | . digits) ([eE][+-]?digits)?  or NaN/Infinity
inline bool is_float_literal(const char* s, size_t n) {
  if (n == 0) return false;
  size_t i = 0;
  if (s[0] == '+' || s[0] == '-') i = 1;
  if (n - i == 3 && std::memcmp(s + i, "NaN", 3) == 0) return true;
  if (n - i == 8 && std::memcmp(s + i, "Infinity", 8) == 0) return true;
  size_t digits = 0;
  while (i < n && s[i] >= '0' && s[i] <= '9') { ++i; ++digits; }
  if (i < n && s[i] == '.') {
    ++i;
    while (i < n && s[i] >= '0' && s[i] <= '9') { ++i; ++digits; }
  }
  if (digits == 0) return false;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
    size_t ed = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') { ++i; ++ed; }
    if (ed == 0) return false;
  }
  return i == n;
}

struct Span {
  int64_t off;
  int32_t len;
  int32_t quoted;
};

// Split one line [b, e) into fields; returns number of fields written.
int split_line(const char* base, int64_t b, int64_t e, std::vector<Span>& out) {
  out.clear();
  int64_t i = b;
  while (true) {
    if (i < e && base[i] == '"') {
      int64_t s = i + 1, j = s;
      while (j < e) {
        if (base[j] == '"') {
          if (j + 1 < e && base[j + 1] == '"') { j += 2; continue; }
          break;
        }
        ++j;
      }
      out.push_back({s, (int32_t)(j - s), 1});
      i = j + 1;
      while (i < e && base[i] != ',') ++i;
    } else {
      int64_t s = i;
      while (i < e && base[i] != ',') ++i;
      out.push_back({s, (int32_t)(i - s), 0});
    }
    if (i >= e) break;
    ++i;  // skip ','
    if (i == e) { out.push_back({e, 0, 0}); break; }
  }
  return (int)out.size();
}

std::string unquote(const char* p, int32_t n, bool quoted) {
  if (!quoted) return std::string(p, p + n);
  std::string s;
  s.reserve(n);
  for (int32_t i = 0; i < n; ++i) {
    s.push_back(p[i]);
    if (p[i] == '"' && i + 1 < n && p[i + 1] == '"') ++i;
  }
  return s;
}

}  // namespace

CsvResult parse_csv(const char* data, size_t size, bool header, int num_threads) {
  CsvResult res;
  if (num_threads <= 0) num_threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // strip UTF-8 BOM
  size_t start = 0;
  if (size >= 3 && (unsigned char)data[0] == 0xEF && (unsigned char)data[1] == 0xBB && (unsigned char)data[2] == 0xBF)
    start = 3;

  // ---- pass 1: line index (parallel newline scan) ----
  const int T = (size - start) < (1u << 20) ? 1 : num_threads;
  std::vector<std::vector<int64_t>> nl(T);
  {
    std::vector<std::thread> th;
    size_t chunk = (size - start + T - 1) / T;
    for (int t = 0; t < T; ++t) {
      th.emplace_back([&, t] {
        size_t b = start + t * chunk, e = std::min(size, b + chunk);
        for (size_t i = b; i < e; ++i)
          if (data[i] == '\n') nl[t].push_back((int64_t)i);
      });
    }
    for (auto& x : th) x.join();
  }
  std::vector<std::pair<int64_t, int64_t>> lines;  // [b, e) without CR/LF
  {
    int64_t prev = (int64_t)start;
    auto push = [&](int64_t b, int64_t e) {
      if (e > b && data[e - 1] == '\r') --e;
      if (e > b) lines.emplace_back(b, e);  // skip empty lines
    };
    for (auto& v : nl)
      for (int64_t p : v) { push(prev, p); prev = p + 1; }
    if (prev < (int64_t)size) push(prev, (int64_t)size);
  }
  if (lines.empty()) return res;

  std::vector<Span> tmp;
  size_t first = 0;
  int ncol;
  if (header) {
    ncol = split_line(data, lines[0].first, lines[0].second, tmp);
    for (auto& s : tmp) {
      std::string name = unquote(data + s.off, s.len, s.quoted);
      // trim spaces
      size_t a = name.find_first_not_of(' '), z = name.find_last_not_of(' ');
      res.names.push_back(a == std::string::npos ? "" : name.substr(a, z - a + 1));
    }
    first = 1;
  } else {
    ncol = split_line(data, lines[0].first, lines[0].second, tmp);
    for (int j = 0; j < ncol; ++j) res.names.push_back("_c" + std::to_string(j));
  }
  const int64_t nrows = (int64_t)lines.size() - (int64_t)first;
  res.nrows = nrows;
  res.ncols = ncol;
  res.doubles.assign((size_t)ncol, std::vector<double>(nrows, NAN));
  res.ints.assign((size_t)ncol, std::vector<int64_t>(nrows, 0));
  res.missing.assign((size_t)ncol, std::vector<uint8_t>(nrows, 0));
  res.spans.assign((size_t)ncol * nrows, {0, 0});
  std::vector<uint8_t> quoted((size_t)ncol * nrows, 0);

  // ---- pass 2: split + classify + parse (parallel over rows) ----
  const int RT = nrows < 4096 ? 1 : num_threads;
  // votes[t][j]: bit0 = saw non-int, bit1 = saw non-float, bit2 = saw int overflow(int32)
  std::vector<std::vector<uint8_t>> votes(RT, std::vector<uint8_t>(ncol, 0));
  std::vector<std::vector<uint8_t>> any_nonempty(RT, std::vector<uint8_t>(ncol, 0));
  {
    std::vector<std::thread> th;
    int64_t chunk = (nrows + RT - 1) / RT;
    for (int t = 0; t < RT; ++t) {
      th.emplace_back([&, t] {
        std::vector<Span> f;
        char numbuf[128];
        int64_t rb = t * chunk, re = std::min(nrows, rb + chunk);
        for (int64_t r = rb; r < re; ++r) {
          auto ln = lines[first + r];
          int nf = split_line(data, ln.first, ln.second, f);
          for (int j = 0; j < ncol; ++j) {
            if (j >= nf || f[j].len == 0) {
              res.missing[j][r] = 1;
              if (j < nf && f[j].quoted) {  // "" : a present, empty string (makes the column a string)
                quoted[(size_t)j * nrows + r] = 1;
                res.spans[(size_t)j * nrows + r] = {f[j].off, 0};
                any_nonempty[t][j] = 1;
                votes[t][j] |= 3;
              }
              continue;
            }
            const char* p = data + f[j].off;
            int32_t n = f[j].len;
            res.spans[(size_t)j * nrows + r] = {f[j].off, n};
            quoted[(size_t)j * nrows + r] = (uint8_t)f[j].quoted;
            any_nonempty[t][j] = 1;
            bool isint = !f[j].quoted && is_int_literal(p, n);
            bool isflt = !f[j].quoted && (isint || is_float_literal(p, n));
            if (!isint) votes[t][j] |= 1;
            if (!isflt) { votes[t][j] |= 2; res.missing[j][r] = 1; continue; }
            int m = std::min<int>(n, 127);
            std::memcpy(numbuf, p, m);
            numbuf[m] = 0;
            if (isint) {
              errno = 0;
              long long v = std::strtoll(numbuf, nullptr, 10);
              if (errno == ERANGE) votes[t][j] |= 1;  // does not fit long -> treat as double
              if (v > 2147483647LL || v < -2147483648LL) votes[t][j] |= 4;
              res.ints[j][r] = v;
              res.doubles[j][r] = (double)v;
            } else {
              res.doubles[j][r] = std::strtod(numbuf, nullptr);
            }
          }
        }
      });
    }
    for (auto& x : th) x.join();
  }

  // ---- pass 3: merge votes ----
  res.kinds.resize(ncol);
  for (int j = 0; j < ncol; ++j) {
    uint8_t v = 0, ne = 0;
    for (int t = 0; t < RT; ++t) { v |= votes[t][j]; ne |= any_nonempty[t][j]; }
    if (!ne || (v & 2)) res.kinds[j] = "string";
    else if (!(v & 1)) res.kinds[j] = (v & 4) ? "long" : "int";
    else res.kinds[j] = "double";
    if (res.kinds[j] == "string") {
      // string columns: only empty fields are missing
      for (int64_t r = 0; r < nrows; ++r) {
        auto sp = res.spans[(size_t)j * nrows + r];
        res.missing[j][r] = (sp.second == 0 && !quoted[(size_t)j * nrows + r]) ? 1 : 0;
      }
    }
  }
  res.quoted.swap(quoted);
  res.base = data;
  return res;
}

std::string CsvResult::field(int col, int64_t row) const {
  auto sp = spans[(size_t)col * nrows + row];
  return unquote(base + sp.first, sp.second, quoted[(size_t)col * nrows + row] != 0);
}

}  // namespace har
