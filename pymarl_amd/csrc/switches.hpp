// The library's environment switches: two variables, each a comma-separated list of `key` or `key=value` items
// (INTEGRATION.md "Switches"). The default plan needs neither.
//   MQ_PLAN  plan overrides for A/B runs and tests, read when a handle is created (mq_create / mc_create) unless
//            noted: unfused_fwd, unfused_bwd, row_tiles=0|1, hyp_in_fwd=0|1, dwh_in_bwd=0|1, fwd_pair=0|1,
//            pair_hyp_epi, mix_generic; COMA (read per train()): coma_chain=0, coma_overlap=0
//   MQ_DIAG  diagnostics and test hooks, read per train(): pair_stamp=<file> (the row-pair forward's s_memtime
//            stamps), bwd_stamp=<file> (the fused BPTT's), hyp_sched=<hex> (the pair forward's in-loop hypernet tile
//            schedule), coma_trace (the COMA chain's phase times), coma_fault=<workgroup> (a chain workgroup that
//            stops flagging)
#pragma once
#include <cstdlib>
#include <cstring>
#include <string>

namespace mq {

// Whether `key` is listed in environment variable `var`; its value ("" for a bare key) into *val.
inline bool env_item(const char* var, const char* key, std::string* val = nullptr) {
  const char* s = std::getenv(var);
  if (!s) return false;
  const size_t kl = std::strlen(key);
  for (const char* p = s; *p;) {
    const char* e = std::strchr(p, ',');
    if (!e) e = p + std::strlen(p);
    const char* eq = (const char*)std::memchr(p, '=', (size_t)(e - p));
    const char* ke = eq ? eq : e;
    if ((size_t)(ke - p) == kl && std::strncmp(p, key, kl) == 0) {
      if (val) *val = eq ? std::string(eq + 1, e) : std::string();
      return true;
    }
    p = *e ? e + 1 : e;
  }
  return false;
}

// `key`'s integer value (a bare key reads as 1), or `dflt` when it is not listed.
inline int env_int(const char* var, const char* key, int dflt, int base = 10) {
  std::string v;
  if (!env_item(var, key, &v)) return dflt;
  return v.empty() ? 1 : (int)std::strtol(v.c_str(), nullptr, base);
}

inline bool plan_flag(const char* key) { return env_item("MQ_PLAN", key); }
inline int plan_int(const char* key, int dflt) { return env_int("MQ_PLAN", key, dflt); }

}  // namespace mq
