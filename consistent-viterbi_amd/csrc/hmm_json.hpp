// hmm_json.hpp -- hmm.json (reference serde layout) reader/writer; see hmm_json.cpp.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace cvh {

struct HmmJson {
  int nstates = 0;
  std::vector<int64_t> bdims;
  std::vector<double> pi, a, b;  // b: [N*V] state-major
};

bool parse_hmm_json(const std::string& text, HmmJson& out, std::string& err);
bool read_file(const std::string& path, std::string& out);
std::string format_hmm_json(int N, const std::vector<int64_t>& bdims, const double* pi, const double* a,
                            const double* b);

}  // namespace cvh
