// Per-handle tuning snapshot (tuning.h): the key table, the environment read and the calling
// thread's current tuning.
#include "tuning.h"

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <string>

namespace cvk {
namespace {

struct Key {
  const char* name;
  int Tuning::*field;
};

#define CVK_KEY(f) {#f, &Tuning::f}
const Key kKeys[] = {
    CVK_KEY(trace), CVK_KEY(host_threads), CVK_KEY(t64_nonpos), CVK_KEY(generic_rows),
    CVK_KEY(max_chunks), CVK_KEY(host_sums), CVK_KEY(no_trace), CVK_KEY(no_resume),
    CVK_KEY(no_side), CVK_KEY(chain_par), CVK_KEY(chain_old), CVK_KEY(chain_par_force),
    CVK_KEY(chain_spec), CVK_KEY(chain_spec_kernel), CVK_KEY(chain_copy_overlap), CVK_KEY(chain_cert_fused),
    CVK_KEY(chain_parts), CVK_KEY(chain_tail), CVK_KEY(chain_tail_div), CVK_KEY(chain_spec_prio), CVK_KEY(chain_pin_obs), CVK_KEY(chain_pin_path), CVK_KEY(t64_s),
    CVK_KEY(t64_512), CVK_KEY(t64_1024), CVK_KEY(t64_wg), CVK_KEY(t64_wg_force),
    CVK_KEY(t64_rs), CVK_KEY(t64_w2), CVK_KEY(t64_wave), CVK_KEY(t64_bal),
    CVK_KEY(t64_cp_s), CVK_KEY(t64_cp_w), CVK_KEY(t64_cp_pf), CVK_KEY(t64_bt_pf),
    CVK_KEY(generic_s), CVK_KEY(generic_split), CVK_KEY(generic_split_k), CVK_KEY(generic_wide),
    CVK_KEY(generic_wide_min), CVK_KEY(generic_prio), CVK_KEY(wide_s), CVK_KEY(ext_wide_min),
    CVK_KEY(chain_wide), CVK_KEY(chain_wide_min), CVK_KEY(f32_onebar), CVK_KEY(bw_global),
    CVK_KEY(bw_perseq), CVK_KEY(bw_gemm_path),
};
#undef CVK_KEY

const Key* find(const char* key) {
  if (!key) return nullptr;
  for (const Key& k : kKeys)
    if (std::strcmp(k.name, key) == 0) return &k;
  return nullptr;
}

const Tuning kDefaults{};
thread_local const Tuning* t_cur = nullptr;
thread_local Tuning t_copy;
thread_local int t_depth = 0;

}  // namespace

const Tuning& tuning() { return t_cur ? *t_cur : kDefaults; }

void tuning_enter(const Tuning& t) {
  // nested entries (an API call made inside another's scope) keep the outermost snapshot
  if (t_depth++ == 0) {
    t_copy = t;
    t_cur = &t_copy;
  }
}

void tuning_leave() {
  if (t_depth > 0 && --t_depth == 0) t_cur = nullptr;
}

TuningOverride::TuningOverride(int Tuning::*field, int value) : field_(field), saved_(0), on_(t_cur != nullptr) {
  if (!on_) return;
  saved_ = t_copy.*field_;
  t_copy.*field_ = value;
}

TuningOverride::~TuningOverride() {
  if (on_ && t_cur) t_copy.*field_ = saved_;
}

Tuning tuning_from_env() {
  Tuning t;
  for (const Key& k : kKeys) {
    std::string var = "CV_";
    for (const char* p = k.name; *p; ++p) var += (char)std::toupper((unsigned char)*p);
    const char* e = std::getenv(var.c_str());
    if (!e || !*e) continue;
    char* end = nullptr;
    const long v = std::strtol(e, &end, 10);
    if (end != e) t.*(k.field) = (int)v;
  }
  return t;
}

bool tuning_set(Tuning& t, const char* key, int64_t value) {
  const Key* k = find(key);
  if (!k || value < INT32_MIN || value > INT32_MAX) return false;
  t.*(k->field) = (int)value;
  return true;
}

bool tuning_get(const Tuning& t, const char* key, int64_t* value) {
  const Key* k = find(key);
  if (!k || !value) return false;
  *value = t.*(k->field);
  return true;
}

const char* tuning_key(int i) {
  return i >= 0 && i < (int)(sizeof(kKeys) / sizeof(kKeys[0])) ? kKeys[i].name : nullptr;
}

}  // namespace cvk
