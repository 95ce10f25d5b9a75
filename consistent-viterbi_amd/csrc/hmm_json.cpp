// hmm_json.cpp -- reader/writer for the reference's hmm.json (serde_json of struct HMM<D>).
//
// Layout (src/hmm/hmm.rs:10-18 with ndarray 0.15 serde):
//   {"a": {"v":1,"dim":[N,N],"data":[...]},
//    "b": {"v":1,"dim":[N],"data":[{"v":1,"dim":[d0,...],"data":[...]}, ...]},
//    "pi":{"v":1,"dim":[N],"data":[...]}}
// serde_json writes non-finite floats as `null`; the reference maps null back to -inf
// (parse_transmat / parse_bmat / parse_pi, hmm.rs:248-264).  Only -inf occurs in a
// log10 model; NaN/+inf are rejected by cv_hmm_create.
#include "hmm_json.hpp"

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace cvh {
namespace {

// product of non-negative dimensions, or -1 when it overflows int64
int64_t dim_product(const std::vector<int64_t>& dim) {
  int64_t n = 1;
  for (auto d : dim)
    if (__builtin_mul_overflow(n, d, &n)) return -1;
  return n;
}

struct Parser {
  const char* p;
  const char* end;
  std::string err;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  const char* begin;
  bool fail(const char* msg) {
    if (err.empty()) {
      char buf[192];
      snprintf(buf, sizeof buf, "hmm.json: %s at byte %ld", msg, (long)(p - begin));
      err = buf;
    }
    return false;
  }
  bool expect(char c) {
    ws();
    if (p >= end || *p != c) return fail("unexpected character");
    ++p;
    return true;
  }
  bool peek(char c) {
    ws();
    return p < end && *p == c;
  }
  bool string(std::string& out) {
    if (!expect('"')) return false;
    out.clear();
    while (p < end && *p != '"') {
      if (*p == '\\') {
        ++p;
        if (p >= end) return fail("bad escape");
      }
      out.push_back(*p++);
    }
    if (p >= end) return fail("unterminated string");
    ++p;
    return true;
  }
  // number or null (-> -inf)
  bool number(double& out) {
    ws();
    if (end - p >= 4 && strncmp(p, "null", 4) == 0) {
      p += 4;
      out = -INFINITY;
      return true;
    }
    // JSON numbers only: strtod alone would also take nan/inf/hex forms serde_json never writes
    if (p >= end || !(*p == '-' || (*p >= '0' && *p <= '9'))) return fail("expected number");
    if (*p == '-' && (end - p < 2 || p[1] < '0' || p[1] > '9')) return fail("expected number");
    char* e = nullptr;
    out = strtod(p, &e);
    if (e == p) return fail("expected number");
    p = e;
    return true;
  }
  bool skip_value() {
    ws();
    if (p >= end) return fail("eof");
    if (*p == '{') {
      ++p;
      if (peek('}')) { ++p; return true; }
      for (;;) {
        std::string k;
        if (!string(k) || !expect(':') || !skip_value()) return false;
        if (peek(',')) { ++p; continue; }
        return expect('}');
      }
    }
    if (*p == '[') {
      ++p;
      if (peek(']')) { ++p; return true; }
      for (;;) {
        if (!skip_value()) return false;
        if (peek(',')) { ++p; continue; }
        return expect(']');
      }
    }
    if (*p == '"') {
      std::string s;
      return string(s);
    }
    if (end - p >= 4 && (strncmp(p, "true", 4) == 0)) { p += 4; return true; }
    if (end - p >= 5 && (strncmp(p, "false", 5) == 0)) { p += 5; return true; }
    double d;
    return number(d);
  }
  bool int_array(std::vector<int64_t>& out) {
    out.clear();
    if (!expect('[')) return false;
    if (peek(']')) { ++p; return true; }
    for (;;) {
      double d;
      if (!number(d)) return false;
      // a dimension: a non-negative integer (no cast of a huge, fractional or infinite value)
      if (!(d >= 0 && d <= 2147483647.0) || d != (double)(int64_t)d) return fail("bad dimension");
      out.push_back((int64_t)d);
      if (peek(',')) { ++p; continue; }
      return expect(']');
    }
  }
  bool num_array(std::vector<double>& out) {
    out.clear();
    if (!expect('[')) return false;
    if (peek(']')) { ++p; return true; }
    for (;;) {
      double d;
      if (!number(d)) return false;
      out.push_back(d);
      if (peek(',')) { ++p; continue; }
      return expect(']');
    }
  }
  // ndarray object {"v":1,"dim":[..],"data":[numbers]}
  bool ndarray(std::vector<int64_t>& dim, std::vector<double>& data) {
    if (!expect('{')) return false;
    bool have_dim = false, have_data = false;
    if (peek('}')) { ++p; return fail("empty ndarray object"); }
    for (;;) {
      std::string k;
      if (!string(k) || !expect(':')) return false;
      if (k == "dim") {
        if (!int_array(dim)) return false;
        have_dim = true;
      } else if (k == "data") {
        if (!num_array(data)) return false;
        have_data = true;
      } else if (!skip_value()) {
        return false;
      }
      if (peek(',')) { ++p; continue; }
      if (!expect('}')) return false;
      break;
    }
    if (!have_dim || !have_data) return fail("ndarray missing dim/data");
    const int64_t n = dim_product(dim);
    if (n < 0 || (int64_t)data.size() != n) return fail("ndarray data length != prod(dim)");
    return true;
  }
  // "b": {"v":1,"dim":[N],"data":[ndarray, ...]}
  bool ndarray_of_arrays(std::vector<int64_t>& outer_dim, std::vector<std::vector<int64_t>>& dims,
                         std::vector<std::vector<double>>& datas) {
    if (!expect('{')) return false;
    bool have_data = false;
    for (;;) {
      std::string k;
      if (!string(k) || !expect(':')) return false;
      if (k == "dim") {
        if (!int_array(outer_dim)) return false;
      } else if (k == "data") {
        if (!expect('[')) return false;
        have_data = true;
        dims.clear();
        datas.clear();
        if (peek(']')) {
          ++p;
        } else {
          for (;;) {
            dims.emplace_back();
            datas.emplace_back();
            if (!ndarray(dims.back(), datas.back())) return false;
            if (peek(',')) { ++p; continue; }
            if (!expect(']')) return false;
            break;
          }
        }
      } else if (!skip_value()) {
        return false;
      }
      if (peek(',')) { ++p; continue; }
      if (!expect('}')) return false;
      break;
    }
    if (!have_data) return fail("b missing data");
    return true;
  }
};

void put_num(std::ostream& os, double v) {
  if (!std::isfinite(v)) {
    os << "null";  // serde_json: non-finite -> null (read back as -inf, hmm.rs:248-264)
    return;
  }
  char buf[40];
  snprintf(buf, sizeof buf, "%.17g", v);
  // keep a float marker so the text reads as f64 like serde_json output
  if (!strpbrk(buf, ".eEn")) strcat(buf, ".0");
  os << buf;
}

void put_ndarray(std::ostream& os, const std::vector<int64_t>& dim, const double* data, int64_t n) {
  os << "{\"v\":1,\"dim\":[";
  for (size_t i = 0; i < dim.size(); ++i) os << (i ? "," : "") << dim[i];
  os << "],\"data\":[";
  for (int64_t i = 0; i < n; ++i) {
    if (i) os << ',';
    put_num(os, data[i]);
  }
  os << "]}";
}

}  // namespace

bool parse_hmm_json(const std::string& text, HmmJson& out, std::string& err) {
  Parser P{text.data(), text.data() + text.size(), {}, text.data()};
  bool have_a = false, have_b = false, have_pi = false;
  std::vector<int64_t> a_dim, pi_dim, b_outer;
  std::vector<std::vector<int64_t>> b_dims;
  std::vector<std::vector<double>> b_data;
  if (!P.expect('{')) { err = P.err; return false; }
  for (;;) {
    std::string k;
    if (!P.string(k) || !P.expect(':')) { err = P.err; return false; }
    bool ok;
    if (k == "a") {
      ok = P.ndarray(a_dim, out.a);
      have_a = true;
    } else if (k == "pi") {
      ok = P.ndarray(pi_dim, out.pi);
      have_pi = true;
    } else if (k == "b") {
      ok = P.ndarray_of_arrays(b_outer, b_dims, b_data);
      have_b = true;
    } else {
      ok = P.skip_value();
    }
    if (!ok) { err = P.err; return false; }
    if (P.peek(',')) { ++P.p; continue; }
    if (!P.expect('}')) { err = P.err; return false; }
    break;
  }
  if (!have_a || !have_b || !have_pi) { err = "hmm.json needs keys a, b, pi"; return false; }
  if (a_dim.size() != 2 || a_dim[0] != a_dim[1]) { err = "a must be N x N"; return false; }
  const int64_t N = a_dim[0];
  if (pi_dim.size() != 1 || pi_dim[0] != N) { err = "pi must have N entries"; return false; }
  if ((int64_t)b_data.size() != N) { err = "b must hold N emission arrays"; return false; }
  out.nstates = (int)N;
  out.bdims = N ? b_dims[0] : std::vector<int64_t>{};
  const int64_t V = dim_product(out.bdims);  // == the first emission array's length (checked)
  out.b.assign((size_t)(N * V), 0.0);
  for (int64_t s = 0; s < N; ++s) {
    if (b_dims[s] != out.bdims) { err = "emission arrays differ in shape"; return false; }
    std::copy(b_data[s].begin(), b_data[s].end(), out.b.begin() + s * V);
  }
  return true;
}

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

std::string format_hmm_json(int N, const std::vector<int64_t>& bdims, const double* pi, const double* a,
                            const double* b) {
  std::ostringstream os;
  int64_t V = 1;
  for (auto d : bdims) V *= d;
  os << "{\"a\":";
  put_ndarray(os, {N, N}, a, (int64_t)N * N);
  os << ",\"b\":{\"v\":1,\"dim\":[" << N << "],\"data\":[";
  for (int s = 0; s < N; ++s) {
    if (s) os << ',';
    put_ndarray(os, bdims, b + (int64_t)s * V, V);
  }
  os << "]},\"pi\":";
  put_ndarray(os, {N}, pi, N);
  os << "}";
  return os.str();
}

}  // namespace cvh
