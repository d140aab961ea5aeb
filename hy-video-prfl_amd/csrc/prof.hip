// Optional per-kernel timing with HIP events, recorded on the stream each kernel is launched on.
// bench.py turns it on around the timed region to derive the roofline numbers of the dominant
// kernel (algorithmic FLOPs or bytes / average launch duration).  Off by default: zero cost.
#include <vector>

#include "common.h"

namespace {
struct Rec {
  int kid;
  hipEvent_t a, b;
  double work;
};
bool g_on = false;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;
int g_open[KID_COUNT + 8];
double g_pending_work = 0.0;

hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

namespace prfl_prof {
void begin(int kid, hipStream_t s) {
  if (!g_on) return;
  Rec r{kid, get_event(), get_event(), 0.0};
  if (!r.a || !r.b) return;
  (void)hipEventRecord(r.a, s);
  g_open[kid] = (int)g_recs.size();
  g_recs.push_back(r);
}
void end(int kid, hipStream_t s) {
  if (!g_on) return;
  if (g_recs.empty()) return;
  Rec& r = g_recs[g_open[kid]];
  r.work = g_pending_work;
  g_pending_work = 0.0;
  (void)hipEventRecord(r.b, s);
}
void set_work(double w) { g_pending_work = w; }
}  // namespace prfl_prof

extern "C" int prfl_prof_enable(int on) {
  g_on = on != 0;
  return 0;
}

// Synchronises the recorded events and returns, per kernel id, the launch count, the summed
// duration in ms and the summed algorithmic work (FLOPs or bytes, as each launcher reports).
extern "C" int prfl_prof_collect(int64_t* counts, double* ms, double* work, int nkid) {
  for (int k = 0; k < nkid; ++k) {
    counts[k] = 0;
    ms[k] = 0.0;
    work[k] = 0.0;
  }
  for (auto& r : g_recs) {
    if (hipEventSynchronize(r.b) != hipSuccess) return -1;
    float t = 0.f;
    (void)hipEventElapsedTime(&t, r.a, r.b);
    if (r.kid >= 0 && r.kid < nkid) {
      counts[r.kid] += 1;
      ms[r.kid] += t;
      work[r.kid] += r.work;
    }
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_recs.clear();
  return 0;
}
