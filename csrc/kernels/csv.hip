// Device CSV parsing: the columnar HIP ETL front end that
// replaces Spark's CSV data source (Main/main.py:18-20).
//
//   csv_count_newlines : one workgroup per 4 KiB chunk, 16 bytes per lane, counts '\n'
//   (host/torch: exclusive cumsum of the chunk counts)
//   csv_newline_pos    : recount + workgroup prefix scan -> global index of every '\n'
//   csv_parse_rows     : one lane per data row: split fields (RFC-4180 quotes), classify
//                        each field (empty / int literal / float literal / other), parse
//                        numbers to fp64, FNV-1a hash of the raw bytes (dictionary
//                        encoding of string columns), field byte spans.
// Column types (int | long | double | string) are then inferred with device reductions
// over the per-field flags, exactly like the host parser / Spark's inferSchema.
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int CHUNK = 4096;  // bytes per workgroup (256 lanes x 16 bytes)

__global__ __launch_bounds__(256) void csv_count_newlines(const uint8_t* __restrict__ buf, int64_t n,
                                                          int32_t* __restrict__ counts) {
  const int64_t base = (int64_t)blockIdx.x * CHUNK + threadIdx.x * 16;
  int c = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) c += (base + i < n && buf[base + i] == '\n');
  __shared__ int red[4];
  c = (int)wave_sum((float)c);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void csv_newline_pos(const uint8_t* __restrict__ buf, int64_t n,
                                                       const int64_t* __restrict__ block_off,
                                                       int64_t* __restrict__ pos) {
  const int64_t base = (int64_t)blockIdx.x * CHUNK + threadIdx.x * 16;
  int c = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) c += (base + i < n && buf[base + i] == '\n');
  // workgroup exclusive scan of the per-lane counts
  __shared__ int sc[256];
  sc[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    int v = threadIdx.x >= o ? sc[threadIdx.x - o] : 0;
    __syncthreads();
    sc[threadIdx.x] += v;
    __syncthreads();
  }
  int64_t k = block_off[blockIdx.x] + sc[threadIdx.x] - c;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (base + i < n && buf[base + i] == '\n') pos[k++] = base + i;
}

__device__ __forceinline__ double pow10i(int e) {
  // exact for |e| <= 22
  const double t[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                        1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  return (e >= 0 && e <= 22) ? t[e] : pow(10.0, (double)e);
}

// flags: bit0 non-empty, bit1 int literal, bit2 float literal (ints included), bit3 quoted,
// bit4 value not exactly representable by the fast path (host strtod fix-up)
__device__ void parse_field(const uint8_t* p, int len, bool quoted, double* val, uint8_t* flags) {
  uint8_t f = len > 0 ? 1 : 0;
  if (quoted) f |= 8;
  *val = NAN;
  if (len == 0 || quoted) { *flags = f; return; }
  int i = 0;
  bool neg = false;
  if (p[0] == '+' || p[0] == '-') { neg = p[0] == '-'; i = 1; }
  if (len - i == 3 && p[i] == 'N' && p[i + 1] == 'a' && p[i + 2] == 'N') { *flags = f | 4; return; }
  if (len - i == 8) {  // exactly "Infinity" (the host parser's rule; "Infected" stays a string)
    const char inf[8] = {'I', 'n', 'f', 'i', 'n', 'i', 't', 'y'};
    bool is_inf = true;
    for (int k = 0; k < 8; ++k) is_inf &= p[i + k] == (uint8_t)inf[k];
    if (is_inf) { *val = neg ? -INFINITY : INFINITY; *flags = f | 4; return; }
  }
  uint64_t mant = 0;
  int digits = 0, sig = 0, exp10 = 0;
  bool dot = false, ok = true;
  for (; i < len; ++i) {
    const uint8_t ch = p[i];
    if (ch >= '0' && ch <= '9') {
      ++digits;
      if (sig < 19) { mant = mant * 10 + (ch - '0'); if (mant) ++sig; if (dot) --exp10; }
      else if (!dot) ++exp10;  // beyond 19 significant digits: scale only
    } else if (ch == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  bool is_int = !dot && digits > 0;
  if (i < len && (p[i] == 'e' || p[i] == 'E') && digits > 0) {
    is_int = false;
    ++i;
    bool eneg = false;
    if (i < len && (p[i] == '+' || p[i] == '-')) { eneg = p[i] == '-'; ++i; }
    int e = 0, ed = 0;
    for (; i < len && p[i] >= '0' && p[i] <= '9'; ++i) { e = e * 10 + (p[i] - '0'); ++ed; }
    if (!ed) ok = false;
    exp10 += eneg ? -e : e;
  }
  if (i != len || digits == 0) ok = false;
  if (!ok) { *flags = f; return; }
  double v = (double)mant;
  v = exp10 >= 0 ? v * pow10i(exp10) : v / pow10i(-exp10);
  *val = neg ? -v : v;
  // one correctly rounded multiply / divide of two exact doubles == strtod; otherwise (mantissa
  // beyond 2^53 or |exp| > 22) bit 4 asks the host to re-parse this field with strtod
  const bool exact = mant <= (1ull << 53) && exp10 <= 22 && exp10 >= -22;
  *flags = f | 4 | (is_int ? 2 : 0) | (exact ? 0 : 16);
}

__global__ __launch_bounds__(256) void csv_parse_rows(const uint8_t* __restrict__ buf, const int64_t* __restrict__ starts,
                                                      const int64_t* __restrict__ ends, int64_t nrows, int ncols,
                                                      double* __restrict__ vals, uint64_t* __restrict__ hashes,
                                                      uint8_t* __restrict__ flags, int64_t* __restrict__ fstart,
                                                      int32_t* __restrict__ flen) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  int64_t b = starts[r], e = ends[r];
  if (e > b && buf[e - 1] == '\r') --e;
  int64_t i = b;
  for (int j = 0; j < ncols; ++j) {
    int64_t fs, fe;
    bool quoted = false;
    if (i > e) {  // the line ran out of fields: missing
      fs = fe = e;
    } else if (i < e && buf[i] == '"') {
      quoted = true;
      fs = i + 1;
      int64_t k = fs;
      while (k < e) {
        if (buf[k] == '"') {
          if (k + 1 < e && buf[k + 1] == '"') { k += 2; continue; }
          break;
        }
        ++k;
      }
      fe = k;
      i = k + 1;
      while (i < e && buf[i] != ',') ++i;
    } else {
      fs = i;
      while (i < e && buf[i] != ',') ++i;
      fe = i;
    }
    const int len = (int)(fe - fs);
    double v;
    uint8_t fl;
    parse_field(buf + fs, len, quoted, &v, &fl);
    if (quoted) fl |= 1;  // "" is a present (empty) string
    uint64_t h = 1469598103934665603ull;  // FNV-1a
    for (int k = 0; k < len; ++k) { h ^= buf[fs + k]; h *= 1099511628211ull; }
    const int64_t o = (int64_t)j * nrows + r;
    vals[o] = v;
    hashes[o] = h;
    flags[o] = fl;
    fstart[o] = fs;
    flen[o] = len;
    if (i < e) ++i;       // skip ','
    else i = e + 1;       // past the end: remaining fields are empty
  }
}

}  // namespace

extern "C" int har_csv_count_newlines(const uint8_t* buf, int64_t n, int32_t* counts, hipStream_t s) {
  if (n < 0) return -2;
  const int64_t blocks = (n + CHUNK - 1) / CHUNK;
  if (blocks == 0) return 0;
  csv_count_newlines<<<(unsigned)blocks, 256, 0, s>>>(buf, n, counts);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_csv_newline_pos(const uint8_t* buf, int64_t n, const int64_t* block_off, int64_t* pos,
                                   hipStream_t s) {
  const int64_t blocks = (n + CHUNK - 1) / CHUNK;
  if (blocks == 0) return 0;
  csv_newline_pos<<<(unsigned)blocks, 256, 0, s>>>(buf, n, block_off, pos);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_csv_parse_rows(const uint8_t* buf, const int64_t* starts, const int64_t* ends, int64_t nrows,
                                  int ncols, double* vals, uint64_t* hashes, uint8_t* flags, int64_t* fstart,
                                  int32_t* flen, hipStream_t s) {
  if (nrows == 0) return 0;
  csv_parse_rows<<<(unsigned)((nrows + 255) / 256), 256, 0, s>>>(buf, starts, ends, nrows, ncols, vals, hashes,
                                                                  flags, fstart, flen);
  HAR_CHECK_LAUNCH();
  return 0;
}
