// hostscan.hpp -- host scan of the constrained decode's components (hostscan.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace cvscan {

struct SeqScan {
  bool constrained;  // some component >= 0 (meaningful only when bad < 0)
  int64_t bad;       // first index k with c[k] outside [-1, ncomp), or -1
};

// One sequence's components c[0, n): the range check and whether any is constrained.
SeqScan scan_sequence(const int32_t* c, int64_t n, int32_t ncomp);

// Appends base + k for every k with c[k] >= 0, ascending (c already range-checked).
void constrained_positions(const int32_t* c, int64_t n, int64_t base, std::vector<int64_t>& out);

}  // namespace cvscan
