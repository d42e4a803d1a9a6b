#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace har {

struct CsvResult {
  int64_t nrows = 0;
  int ncols = 0;
  std::vector<std::string> names;
  std::vector<std::string> kinds;                 // int | long | double | string
  std::vector<std::vector<double>> doubles;       // [col][row], NaN when missing / non-numeric
  std::vector<std::vector<int64_t>> ints;         // [col][row]
  std::vector<std::vector<uint8_t>> missing;      // [col][row]
  std::vector<std::pair<int64_t, int32_t>> spans; // [col * nrows + row] -> (offset, len)
  std::vector<uint8_t> quoted;                    // [col * nrows + row]
  const char* base = nullptr;                     // valid while the caller's buffer lives
  std::string field(int col, int64_t row) const;
};

CsvResult parse_csv(const char* data, size_t size, bool header, int num_threads);

}  // namespace har
