// Optional per-kernel timing with HIP events, recorded on the stream each kernel is launched on.
// bench.py turns it on around the timed region to derive the roofline numbers of the dominant
// kernel (algorithmic FLOPs or bytes / average launch duration).  Off by default: zero cost.
// Clock slots: while on, a kernel that takes one (the self-attention forward) has its workgroup
// 0 write (shader cycles, 100 MHz ticks) elapsed over its lifetime (s_memtime / s_memrealtime):
// the effective shader clock during the launches the roofline is computed from.
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
constexpr int CLK_CAP = 1 << 15;   // launches per window
unsigned long long* g_clk = nullptr;
int g_clk_n = 0;

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
unsigned long long* clk_slot() {
  if (!g_on || !g_clk || g_clk_n >= CLK_CAP) return nullptr;
  return g_clk + 2 * (g_clk_n++);
}
}  // namespace prfl_prof

extern "C" int prfl_prof_enable(int on) {
  if (on && !g_clk) {
    if (hipMalloc(&g_clk, sizeof(unsigned long long) * 2 * CLK_CAP) != hipSuccess) {
      g_clk = nullptr;
      return -1;
    }
    if (hipMemset(g_clk, 0, sizeof(unsigned long long) * 2 * CLK_CAP) != hipSuccess) return -1;
    g_clk_n = 0;
  }
  g_on = on != 0;
  return 0;
}

// Effective shader clock (MHz) over the clock slots written since the last call: mean of the
// per-launch cycles / (ticks / 100 MHz) weighted by launch time, min and max; resets the slots.
extern "C" int prfl_prof_clock(double* mean_mhz, double* min_mhz, double* max_mhz, int64_t* n) {
  *mean_mhz = *min_mhz = *max_mhz = 0.0;
  *n = 0;
  if (!g_clk || !g_clk_n) return 0;
  std::vector<unsigned long long> h(2 * g_clk_n);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(h.data(), g_clk, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) !=
      hipSuccess)
    return -1;
  double cyc = 0.0, ticks = 0.0, lo = 1e30, hi = 0.0;
  int64_t k = 0;
  for (int i = 0; i < g_clk_n; ++i) {
    const double c = (double)h[2 * i], t = (double)h[2 * i + 1];
    if (t <= 0.0 || c <= 0.0) continue;
    const double mhz = c / t * 100.0;
    cyc += c;
    ticks += t;
    lo = mhz < lo ? mhz : lo;
    hi = mhz > hi ? mhz : hi;
    ++k;
  }
  if (k) {
    *mean_mhz = cyc / ticks * 100.0;
    *min_mhz = lo;
    *max_mhz = hi;
    *n = k;
  }
  g_clk_n = 0;
  return hipMemset(g_clk, 0, sizeof(unsigned long long) * 2 * CLK_CAP) == hipSuccess ? 0 : -1;
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
