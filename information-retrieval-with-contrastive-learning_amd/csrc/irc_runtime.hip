// Error plumbing and version for the libirc_hip.so C ABI (include/irc.h).
#include <stdarg.h>
#include <stdio.h>

#include "irc_common.h"

namespace irc {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? (int)e : IRC_E_LAUNCH;
  }
  return IRC_OK;
}

}  // namespace irc

extern "C" const char* irc_last_error(void) { return irc::g_err; }

extern "C" int irc_abi_version(void) { return 1; }

// ---------------------------------------------------------------- profiling
// Optional per-kernel timing with HIP events recorded on the launch stream, used
// by bench.py to measure the dominant kernel's average duration live.  Off by
// default (a single branch per launch).
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace irc {

static bool g_prof = false;
static std::mutex g_prof_mu;
struct ProfRec {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double total_ms = 0;
  int64_t count = 0;
  double work = 0;  // algorithmic flops or bytes of the recorded launches
};
static std::unordered_map<std::string, ProfRec> g_prof_tab;
static thread_local hipEvent_t g_open_ev = nullptr;

bool prof_on() { return g_prof; }

void prof_begin(hipStream_t st) {
  if (!g_prof) return;
  hipEventCreate(&g_open_ev);
  hipEventRecord(g_open_ev, st);
}

void prof_end(const char* name, hipStream_t st, double work) {
  if (!g_prof || !g_open_ev) return;
  hipEvent_t e;
  hipEventCreate(&e);
  hipEventRecord(e, st);
  std::lock_guard<std::mutex> lk(g_prof_mu);
  ProfRec& r = g_prof_tab[name];
  r.pending.emplace_back(g_open_ev, e);
  r.work += work;
  g_open_ev = nullptr;
}

// A work tally without timing (count += 1, work += work), e.g. the algorithmic
// bytes of the launches a timed record of another name covers.
void prof_work(const char* name, double work) {
  if (!g_prof) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  ProfRec& r = g_prof_tab[name];
  r.count += 1;
  r.work += work;
}

}  // namespace irc

extern "C" int irc_prof_enable(int on) {
  irc::g_prof = on != 0;
  return IRC_OK;
}

// Synchronises the recorded events of `name` and returns accumulated time/count.
extern "C" int irc_prof_query(const char* name, double* total_ms, int64_t* count,
                              double* work) {
  std::lock_guard<std::mutex> lk(irc::g_prof_mu);
  auto it = irc::g_prof_tab.find(name);
  if (it == irc::g_prof_tab.end()) {
    *total_ms = 0;
    *count = 0;
    if (work) *work = 0;
    return IRC_OK;
  }
  if (work) *work = it->second.work;
  for (auto& pr : it->second.pending) {
    hipEventSynchronize(pr.second);
    float ms = 0;
    hipEventElapsedTime(&ms, pr.first, pr.second);
    it->second.total_ms += ms;
    it->second.count += 1;
    hipEventDestroy(pr.first);
    hipEventDestroy(pr.second);
  }
  it->second.pending.clear();
  *total_ms = it->second.total_ms;
  *count = it->second.count;
  return IRC_OK;
}

extern "C" int irc_prof_reset(void) {
  std::lock_guard<std::mutex> lk(irc::g_prof_mu);
  for (auto& kv : irc::g_prof_tab)
    for (auto& pr : kv.second.pending) {
      hipEventDestroy(pr.first);
      hipEventDestroy(pr.second);
    }
  irc::g_prof_tab.clear();
  return IRC_OK;
}
