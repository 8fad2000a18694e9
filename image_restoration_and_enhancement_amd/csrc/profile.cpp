// irx — in-process kernel timing with HIP events (bench.py's roofline numerator / denominator).
// When enabled, every MFMA GEMM/conv and attention launch is bracketed by a pair of events on
// its own stream and tagged with its instantiation name and its ALGORITHMIC flops (2*M*N*K for
// a GEMM / implicit-GEMM conv, 4*B*H*Lq*Lk*d for attention).  irx_profile_end() synchronises the
// events and aggregates per kernel instantiation.  Off by default: no events, no overhead.
#include <map>
#include <string>
#include <vector>

#include "profile.h"

namespace irx {
int g_prof_shapes = 0;
namespace {
struct Rec {
  std::string name;
  double flops;
  hipEvent_t a, b;
};
bool g_on = false;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;
size_t g_used = 0;

hipEvent_t next_event() {
  if (g_used == g_pool.size()) {
    hipEvent_t e;
    IRX_HIP(hipEventCreate(&e));
    g_pool.push_back(e);
  }
  return g_pool[g_used++];
}

struct Agg {
  long launches = 0;
  double ms = 0, flops = 0;
};
std::vector<std::pair<std::string, Agg>> g_result;
}  // namespace

bool prof_on() { return g_on; }

int prof_start(const std::string& name, double flops, hipStream_t s) {
  if (!g_on) return -1;
  Rec r{name, flops, next_event(), next_event()};
  IRX_HIP(hipEventRecord(r.a, s));
  g_recs.push_back(r);
  return (int)g_recs.size() - 1;
}

void prof_stop(int idx, hipStream_t s) {
  if (idx < 0) return;
  IRX_HIP(hipEventRecord(g_recs[idx].b, s));
}

void prof_begin() {
  g_on = true;
  g_recs.clear();
  g_used = 0;
}

int prof_end() {
  g_on = false;
  std::map<std::string, Agg> m;
  for (auto& r : g_recs) {
    IRX_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    IRX_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    Agg& a = m[r.name];
    a.launches += 1;
    a.ms += ms;
    a.flops += r.flops;
  }
  g_recs.clear();
  g_used = 0;
  g_result.assign(m.begin(), m.end());
  return (int)g_result.size();
}

bool prof_get(int i, const char** name, long* launches, double* ms, double* flops) {
  if (i < 0 || i >= (int)g_result.size()) return false;
  *name = g_result[i].first.c_str();
  *launches = g_result[i].second.launches;
  *ms = g_result[i].second.ms;
  *flops = g_result[i].second.flops;
  return true;
}

}  // namespace irx
