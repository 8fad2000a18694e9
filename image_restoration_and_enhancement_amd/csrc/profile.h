// irx — optional per-launch HIP-event timing (see profile.cpp).
#pragma once
#include <string>

#include "irx_common.h"

namespace irx {
bool prof_on();
extern int g_prof_shapes;   // irx_set_option("prof_shapes", 1): profiler keys carry the call shape (per-shape tables)
int prof_start(const std::string& name, double flops, hipStream_t s);   // -1 when profiling is off
void prof_stop(int idx, hipStream_t s);
void prof_begin();
int prof_end();
bool prof_get(int i, const char** name, long* launches, double* ms, double* flops);

// RAII bracket around one kernel launch (no-op unless profiling is on)
struct ProfScope {
  int idx;
  hipStream_t s;
  ProfScope(const std::string& name, double flops, hipStream_t st) : idx(-1), s(st) {
    if (prof_on()) idx = prof_start(name, flops, st);
  }
  ~ProfScope() { if (idx >= 0) prof_stop(idx, s); }
};
}  // namespace irx
