// engine.cpp — host side of the C-ABI (include/raftstep.h).
//
// Owns the device planes of one GPU, validates every call, converts the
// canonical group-major host view to/from the replica-major device layout,
// launches the kernels on the engine's own HIP stream and, when attached,
// sums tick statistics across GPUs with RCCL. Nothing here computes Raft
// state: that is all on the device (kernels.hip).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unistd.h>
#include <vector>

#include "../../include/raftstep.h"
#include "kernels.h"

using namespace raftstep;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) return fail(RAFT_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

#define RCCLCHK(expr)                                                                         \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess) return fail(RAFT_ERCCL, "%s: %s", #expr, ncclGetErrorString(_r)); \
  } while (0)

constexpr int I32 = 2147483647;

// CRC32C (Castagnoli, reflected 0x82F63B78) slice-by-8 tables, T[k][b].
std::vector<uint32_t> crc32c_tables() {
  std::vector<uint32_t> T(8 * 256);
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    T[b] = c;
  }
  for (int k = 1; k < 8; ++k)
    for (uint32_t b = 0; b < 256; ++b) T[k * 256 + b] = (T[(k - 1) * 256 + b] >> 8) ^ T[T[(k - 1) * 256 + b] & 255];
  return T;
}
const std::vector<uint32_t>& crc_tab_host() {
  static const std::vector<uint32_t> T = crc32c_tables();
  return T;
}
uint32_t host_entry_crc(int32_t term, int64_t value) {
  const std::vector<uint32_t>& T = crc_tab_host();
  uint32_t c = 0xFFFFFFFFu ^ uint32_t(term);
  c = T[768 + (c & 255)] ^ T[512 + ((c >> 8) & 255)] ^ T[256 + ((c >> 16) & 255)] ^ T[c >> 24];
  const uint32_t lo = c ^ uint32_t(uint64_t(value)), hi = uint32_t(uint64_t(value) >> 32);
  return ~(T[1792 + (lo & 255)] ^ T[1536 + ((lo >> 8) & 255)] ^ T[1280 + ((lo >> 16) & 255)] ^ T[1024 + (lo >> 24)] ^
           T[768 + (hi & 255)] ^ T[512 + ((hi >> 8) & 255)] ^ T[256 + ((hi >> 16) & 255)] ^ T[hi >> 24]);
}

// Device ring layout (raft_device.hpp ring_tile / ring_in_tile): [Gp/64][K][64][R].
inline uint64_t ring_index(uint64_t r, uint64_t g, uint64_t s, uint64_t K, uint64_t R) {
  return (((g >> 6) * K + s) * 64 + (g & 63)) * R + r;
}

// RAFTSTEP_COMM_TIMEOUT_S: seconds a communicator's init or a call's
// all-reduce may take before it fails with RAFT_ETIMEDOUT (default 300)
double comm_timeout_s() {
  const char* t = getenv("RAFTSTEP_COMM_TIMEOUT_S");
  const double v = t ? atof(t) : 300.0;
  return v > 0 ? v : 300.0;
}

bool fits32(int64_t v) { return v >= -int64_t(I32) - 1 && v <= int64_t(I32); }

}  // namespace

struct raft_engine {
  raft_config cfg{};
  int R = 0;
  uint64_t Gp = 0;
  uint64_t KP = 0;   // physical ring slots per replica (ring_depth or 2x)
  hipStream_t stream = nullptr;
  DevPlanes P{};
  std::vector<void*> allocs;
  uint64_t device_bytes = 0;
  // per-tick statistics: atomic targets [cap][STAT_TICK] u64 (kept
  // zero between calls by the reduce kernel) and the reduced per-tick records
  // [cap][NSTAT] (the 64 B per tick that RCCL sums across GPUs)
  unsigned long long* hist = nullptr;
  unsigned long long* tstat = nullptr;   // [hist_cap + 2][NSTAT]: per-tick records, then two check records
  unsigned long long* hrb = nullptr;     // pinned host copy of tstat (one async readback per call)
  // host mirror of a call's records (CallCheck::hout): a call whose records
  // are all reduced by its last launch (no communicator) has that launch write
  // them into hrb as well and publish `seq` in *hdone; raft_tick then spins on
  // hdone instead of copying the records back and waiting for the stream
  uint32_t* hdone = nullptr;             // pinned, coherent
  unsigned int* dctr = nullptr;          // device block counter of the mirror launch
  uint32_t seq = 0;
  bool mirror = false;                   // the current call's records go to hrb directly
  uint32_t hist_cap = 0;
  uint32_t last_stats_n = 0;             // nticks of the last raft_tick call with statistics (0: none yet)
  unsigned long long* cstat = nullptr;   // raft_comm_allreduce_stats staging
  uint32_t wpar = 0;            // parity of the next worklist window (its counters were zeroed by its last window tail)
  // worklists of groups the fast kernels hand to the general kernel, one per
  // window index mod NWORK (the general kernel of a window may run beside the
  // next window's first tick, whose list kernel may already defer into the
  // window after)
  uint32_t* work[NWORK] = {};   // deferred group ids (window index mod NWORK)
  int32_t* work_tick[NWORK] = {}; // tick each one was deferred at
  uint32_t* wcount = nullptr;   // counter block (raft_device.hpp WCOUNT_WORDS): worklists x2, two-pass list x2, tail words
  // Overlapped general kernel: at a window's end (not a call's last tick) the
  // general kernel runs on gen_stream beside the next tick's lean and list
  // kernels, catching its groups up through that tick too (they keep DEFER,
  // so the fast kernels leave them alone); the engine stream then waits for
  // it and runs the window tail (DEFER cleared) before the tick after.
  // RAFTSTEP_OVERLAP_GENERAL=0 runs it in line (not with the pipeline); d >= 1
  // overlaps it with the next d ticks (it catches its groups up through tick
  // t+d, the engine stream joins it before tick t+d+1). Exact for every d
  // (tests/test_gpu_pipeline.py). Default 3 since round 5 (C4 +3%, C4R +5%,
  // C4REF +6% over depth 2 in interleaved A/Bs, profiles/r05/ab/r5ab12).
  int overlap_general = 3;
  hipStream_t gen_stream = nullptr;
  hipEvent_t gen_ev[2] = {nullptr, nullptr};   // engine -> gen_stream, gen_stream -> engine
  bool gen_pending = false;     // a general kernel is running on gen_stream
  int gen_parity = 0;           // its worklist parity
  uint32_t gen_w0 = 0, gen_w1 = 0;   // its window's stats range (indices into the call's ticks)
  uint32_t gen_join = 0;        // the call's tick index after whose launches the engine stream joins it
  uint32_t gen_top = 0;         // the last tick index it counts stats into
  bool gen_stats = false;       // it counts into those per-tick slots of hist
  // per-tick atomic slots of hist a call may have counted into and not
  // reduced (the reduce re-zeroes what it reads): set when a call with
  // statistics starts launching, cleared when it has issued every reduce; a
  // call that fails in between leaves it set and the next call zeroes them
  uint32_t hist_dirty = 0;
  // VX (raft_device.hpp M_VX): groups may hold virtual suffixes (P.vx and a
  // call has run since the last flush); they are defined by the client ticks
  // before vx_tick (-1: unknown, a call failed mid-way: the engine is poisoned)
  bool vx_live = false;
  int64_t vx_tick = 0;
  // SH (raft_device.hpp ROT_SH): groups may hold shared entries (P.sh and a
  // lean / fused kernel has run since the last sh_flush)
  bool sh_live = false;
  // the running call's first tick and whether its ticks run the lean (or
  // fused) kernel over every group (the base of its statistics)
  int64_t call_t0 = 0;
  bool call_lean = false;
  int64_t sh_next = 0;          // the tick after the last call that may have left them
  bool sh_done = true;          // that call issued all its launches (else the implied heartbeat time is unknown)
  // the current run of consecutive raft_tick calls (Trace::contig_q): it
  // starts at contig_from and continues at run_next; a call at another tick,
  // a handler batch or a state replacement starts a new one
  bool run_valid = false, run_done = false;   // (run_done: the last call issued everything)
  int64_t contig_from = 0, run_next = 0;
  int force_general = 0;        // debug: route every group through the general kernel
  int lane_general = 0;         // RAFTSTEP_GENERAL=lane: one-lane-per-group general kernel (A/B) instead of the segment one
  uint32_t slow_every = 8;      // run the general kernel every this many ticks (and at the end of a call)
  int debug_work = 0;           // RAFTSTEP_DEBUG_WORK: print each general-kernel worklist size
  int debug_pipe = 0;           // RAFTSTEP_DEBUG_PIPE: print each call's pipeline choice
  // two-pass tick (RAFTSTEP_TWO_PASS, default on): the lean kernel takes the
  // compressed steady groups, the list kernel every other live group
  int two_pass = 1;
  uint32_t* blist[3] = {nullptr, nullptr, nullptr};   // groups the lean kernel passed on, one list per tick mod 3
  uint32_t lpar = 0;            // tick counter of the two-pass lists (list lpar % 3 is the next tick's)
  // Pipelined tick (RAFTSTEP_PIPELINE, default on; two-pass, list not
  // skipped): the list kernel of tick t runs on list_stream and carries its
  // groups through tick t+1 too, so the lean kernel of t+1 (which leaves those
  // groups alone, P.glst marks) runs beside it; the lean kernel of t+2 waits
  // for it. Lists and their counters rotate over three sets: lean(t+1) fills
  // one while list(t) reads another and zeroes the third.
  // RAFTSTEP_PIPELINE=0 runs the two passes in line (exact either way:
  // tests/test_gpu_pipeline.py).
  int pipeline = 1;
  // Ping-pong streams (pipelined tick, RAFTSTEP_PINGPONG, default on): tick t
  // runs lean(t) and list(t) back to back on stream t mod 2 (the engine stream
  // or list_stream); lean(t) waits for lean(t-1) on the other stream, and for
  // list(t-2) by stream order. The tick's critical chain, list(t-1) ->
  // lean(t+1) -> list(t+1), then has no cross-queue wake-up in it (~13 us per
  // such wait, measured: tools/gap_probe.hip), and list(t) no longer waits for
  // list(t-1) (their groups are disjoint: lean(t) leaves list(t-1)'s alone).
  // lean(t) zeroes the counter lean(t+1) fills (read by list(t-2), done).
  int pingpong = 1;
  hipEvent_t ev_pp = nullptr;   // list_stream -> engine stream at the end of a ping-pong call
  // Fused steady ticks (raft_config.ticks_per_launch, default 1 = off): while
  // the steady-state list skip holds (and without payload CRC, whose
  // per-follower verification the lean kernel does tick by tick), up to that
  // many ticks run in one launch of tick_fused_kernel (k_fast.hip)
  uint32_t fuse = 1;
  hipStream_t list_stream = nullptr;
  // Split steady tick: with the list skipped (lean kernel alone, one tick per
  // launch), each tick is two launches over the two halves of the groups on
  // two streams, so that one half's kernel boundary (drain, launch, the
  // previous kernel's tail) overlaps the other half's streaming. Groups never
  // address each other, so the halves are independent; they join before every
  // statistics reduce and at the end of the call. RAFTSTEP_SPLIT_STEADY=0:
  // one launch per tick (exact either way: tests/test_gpu_engine_checks.py).
  int split_steady = 1;
  hipStream_t half_stream = nullptr;
  hipEvent_t ev_half[2] = {nullptr, nullptr};   // engine -> half stream, half stream -> engine
  hipEvent_t ev_lean[2] = {nullptr, nullptr};   // engine stream -> list_stream (list(t) after lean(t))
  hipEvent_t ev_list[4] = {nullptr, nullptr, nullptr, nullptr};   // list_stream -> engine stream (list(t) done)
  // Steady-state list skip. After init_steady (every log empty, entries
  // appended from there only) and no host mutation since, once a call ends
  // with nothing deferred in its last window and an empty list at its last
  // tick, every live group is in the compressed steady state and the lean
  // kernel takes it; without isolation or corruption it then takes it again
  // every tick (its conditions only need LastApplied+E < 2^31 and E < K,
  // both checked here), so the list kernel's launch — about 5 us per tick
  // whatever its list holds — is skipped. raft_tick re-checks at the end of
  // every call with statistics: the list counters of a call that skipped are
  // never zeroed, so any group passed during it would show (RAFT_EINTERNAL).
  bool steady_origin = false;
  bool steady_ok = false;
  bool skipped_list = false;    // the current call skipped the list kernel
  // A skipping call without statistics ends with the check record written to
  // tstat[hist_cap + 1] and copied to the pinned buffer (event chk_ev); the
  // next call on the engine waits for it and verifies that nothing was passed
  // to the list kernel that did not run. If something was, ticks were lost:
  // the engine is poisoned (every call fails with RAFT_EINTERNAL) until its
  // state is replaced (init_*, load_state, checkpoint load).
  bool pend_chk = false;
  hipEvent_t chk_ev = nullptr;
  bool poisoned = false;
  std::string poison_msg;
  // diagnostics: lane class counters on the device (raft_diag_enable), host counters
  int diag_print = 0;
  unsigned long long* dbg_buf = nullptr;   // the device counters (P.dbg while counting)           // RAFTSTEP_DEBUG_FAST: print the class counters after every call (synchronising)
  uint64_t n_ticks = 0, n_skip_ticks = 0, n_general = 0;
  // handler-batch staging
  void* stage = nullptr;
  size_t stage_cap = 0;
  // RAFT_CLIENT_STAGED: the caller's client values in HBM, [cv_n][E][G]
  // int64 for ticks [cv_t0, cv_t0 + cv_n) (raft_stage_values; DevPlanes::cv)
  int64_t* cvbuf = nullptr;
  uint8_t* giso_plane = nullptr;   // DevPlanes::giso (round 6: a dense plane)
  uint64_t cv_cap = 0;          // elements allocated
  int64_t cv_t0 = 0;
  uint32_t cv_n = 0;
  // profiling: 0 off, 1 per fast-kernel dispatch (hipExtLaunchKernel events),
  // 2 one event pair around each raft_tick call's launches (no per-launch cost)
  int prof = 0;
  std::vector<hipEvent_t> ev;
  std::vector<uint32_t> ev_ticks;   // mode 1: ticks each event pair covers (fused steady ticks: several)
  size_t ev_used = 0;
  double prof_ms = 0.0;
  uint64_t prof_n = 0;
  // RCCL: the per-tick stats all-reduce runs on its own stream, ordered after
  // each window's reduce kernel by an event, so it overlaps the next ticks
  ncclComm_t comm = nullptr;
  hipStream_t comm_stream = nullptr;
  std::vector<hipEvent_t> comm_ev;
  std::vector<hipEvent_t> comm_pre;   // markers before each all-reduce since the last completed wait (wait_stream)
  size_t comm_pre_used = 0;
  int nranks = 1, rank = 0;
  uint64_t allreduces = 0;      // ncclAllReduce calls issued (diagnostics)
  bool comm_side = false;       // a sum on comm_stream the engine stream has not waited for
};

namespace {

int dev_alloc(raft_engine* e, void** p, size_t bytes) {
  hipError_t rc = hipMalloc(p, bytes ? bytes : 16);
  if (rc != hipSuccess) return fail(RAFT_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(rc));
  e->allocs.push_back(*p);
  e->device_bytes += bytes;
  return RAFT_OK;
}

Trace make_trace(const raft_engine* e, int64_t tick) {
  Trace T{};
  T.seed = e->cfg.seed;
  T.tick = tick;
  T.now = int32_t(tick * e->cfg.tick_seconds);
  T.f_min = e->cfg.follower_timeout_min;
  T.f_span = e->cfg.follower_timeout_span;
  T.c_min = e->cfg.candidate_timeout_min;
  T.c_span = e->cfg.candidate_timeout_span;
  T.iso_p = e->cfg.isolate_per_65536;
  T.iso_min = e->cfg.isolate_min_ticks;
  T.iso_span = e->cfg.isolate_max_ticks - e->cfg.isolate_min_ticks + 1;
  udiv_magic_of(T.iso_span, &T.iso_m, &T.iso_l);
  T.iso_leader = e->cfg.isolate_leader;
  T.secs = e->cfg.tick_seconds;
  T.period = e->cfg.client_period;
  T.entries = e->cfg.entries_per_tick;
  const int64_t cf = e->contig_from;
  T.contig_q = (T.period && cf > 0) ? uint64_t((cf + int64_t(T.period) - 1) / int64_t(T.period)) * T.entries : 0u;
  if (!e->run_valid) T.contig_q = ~uint64_t(0);   // (no run: nothing regenerable)
  // staged client values: no entry is ever regenerated (entry jobs read the
  // rings instead: the general kernel), whatever the run
  if (e->cfg.client_source == RAFT_CLIENT_STAGED) T.contig_q = ~uint64_t(0);
  T.n_tick = T.client_entries_slow(tick);
  T.eb_tick = T.entries_before_slow(tick);
  return T;
}

// virtual seconds must stay inside int32 (deadline = now + d)
int check_ticks(const raft_engine* e, int64_t first, uint64_t n) {
  const int64_t maxd = std::max(e->cfg.follower_timeout_min + e->cfg.follower_timeout_span,
                                e->cfg.candidate_timeout_min + e->cfg.candidate_timeout_span);
  if (first < 0) return fail(RAFT_ERANGE, "tick must be >= 0");
  const long double last_now = (long double)(first + int64_t(n)) * e->cfg.tick_seconds + maxd;
  if (last_now >= (long double)I32) return fail(RAFT_ERANGE, "virtual time leaves int32 seconds");
  return RAFT_OK;
}

int ensure_stage(raft_engine* e, size_t bytes) {
  if (bytes <= e->stage_cap) return RAFT_OK;
  if (e->stage) {
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipFree(e->stage));
    e->stage = nullptr;
  }
  size_t cap = std::max<size_t>(bytes, 1 << 20);
  HIPCHK(hipMalloc(&e->stage, cap));
  e->stage_cap = cap;
  return RAFT_OK;
}

int ensure_hist(raft_engine* e, uint32_t n) {
  if (n <= e->hist_cap) return RAFT_OK;
  HIPCHK(hipStreamSynchronize(e->stream));
  if (e->comm_stream) HIPCHK(hipStreamSynchronize(e->comm_stream));
  if (e->hist) HIPCHK(hipFree(e->hist));
  if (e->tstat) HIPCHK(hipFree(e->tstat));
  if (e->hrb) HIPCHK(hipHostFree(e->hrb));
  e->hist = e->tstat = e->hrb = nullptr;
  e->hist_cap = 0;
  e->last_stats_n = 0;
  uint32_t cap = std::max<uint32_t>(n, 64);
  const size_t hb = size_t(cap) * STAT_TICK * 8;
  const size_t tb = size_t(cap + 2) * NSTAT * 8;   // + the two check records (raft_engine::tstat)
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&e->hist), hb));
  HIPCHK(hipMalloc(reinterpret_cast<void**>(&e->tstat), tb));
  HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&e->hrb), tb, hipHostMallocCoherent));
  HIPCHK(hipMemsetAsync(e->hist, 0, hb, e->stream));   // once; the reduce kernel re-zeroes what it reads
  HIPCHK(hipMemsetAsync(e->tstat, 0, tb, e->stream));
  e->hist_cap = cap;
  return RAFT_OK;
}

// The check of the last list-skipping call without statistics (see
// raft_engine::pend_chk): waits for its record and poisons the engine if the
// lean kernel passed any group on while the list kernel was skipped.
int settle_check(raft_engine* e) {
  if (e->pend_chk) {
    e->pend_chk = false;
    HIPCHK(hipEventSynchronize(e->chk_ev));
    const unsigned long long* c = e->hrb + size_t(e->hist_cap + 1) * NSTAT;
    if (c[CHK_MAGIC] != 0x5241465443484Bull) {
      e->poisoned = true;
      e->poison_msg = "steady-state list skip: the end-of-call check record was not written";
    } else if (c[CHK_LISTED]) {
      e->poisoned = true;
      e->poison_msg = "steady-state list skip: " + std::to_string(c[CHK_LISTED]) +
                      " groups were passed to a list kernel that did not run (ticks lost)";
    }
    if (e->poisoned) e->steady_ok = false;
  }
  if (e->poisoned)
    return fail(RAFT_EINTERNAL, "%s; the engine state is invalid until init_*, load_state or a checkpoint load",
                e->poison_msg.c_str());
  return RAFT_OK;
}

// A call that replaces the state starts by dropping the list-skip proof (the
// conservative direction, whatever happens next) ...
void state_replacing(raft_engine* e) {
  e->steady_origin = e->steady_ok = false;
  e->vx_live = false;   // (the state is being replaced: no suffix survives)
  e->sh_live = false;   // (nor a shared entry: every rotation is rewritten)
  e->run_valid = false;
}
// ... and only once the new state's launches / copies have gone through
// successfully drops any poison and a still-pending end-of-call check (both
// describe the old state). A call that fails on the way leaves them as they
// were: a poisoned engine stays poisoned.
void state_replaced(raft_engine* e) {
  e->pend_chk = false;
  e->poisoned = false;
  e->poison_msg.clear();
}

// VX: every group's virtual suffix into its ring, before anything but the
// tick path reads or changes the state (host views, digests, handler batches)
// or a call starts at a tick other than the one after the last call.
int vx_flush(raft_engine* e) {
  if (!e->vx_live) return RAFT_OK;
  if (e->vx_tick < 0) {
    e->poisoned = true;
    e->steady_ok = false;
    e->poison_msg = "a failed raft_tick call left virtual log suffixes undefined (state must be replaced)";
    return fail(RAFT_EINTERNAL, "%s", e->poison_msg.c_str());
  }
  const uint64_t per = e->cfg.client_period, E = e->cfg.entries_per_tick;
  const int64_t t = e->vx_tick;
  const uint64_t Qb = (per && t > 0) ? uint64_t((t + int64_t(per) - 1) / int64_t(per)) * E : 0u;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(launch_vx_flush(e->R, e->P, Qb, uint32_t(E), uint32_t(per), e->cfg.seed, e->stream));
  e->vx_live = false;
  return RAFT_OK;
}

// SH: every group's shared entries into its replica rings, before the host
// reads or changes the rings (host views, handler batches). Exact at any time
// (nothing is regenerated); the digest reads the shared ring itself.
// The heartbeat time every group in shared form holds implicitly (now of the
// last tick run, DevPlanes::sh_hb); unknown after a call that failed mid-way.
int sh_heartbeat(raft_engine* e) {
  if (!e->sh_done) {
    e->poisoned = true;
    e->steady_ok = false;
    e->poison_msg = "a failed raft_tick call left shared entries' heartbeat times undefined (state must be replaced)";
    return fail(RAFT_EINTERNAL, "%s", e->poison_msg.c_str());
  }
  e->P.sh_hb = make_trace(e, e->sh_next - 1).now;
  return RAFT_OK;
}
int sh_flush(raft_engine* e) {
  if (!e->sh_live) return RAFT_OK;
  if (int rc = sh_heartbeat(e)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(launch_sh_flush(e->R, e->P, e->stream));
  e->sh_live = false;
  return RAFT_OK;
}
int ring_flush(raft_engine* e) {
  if (int rc = vx_flush(e)) return rc;
  return sh_flush(e);
}

hipEvent_t next_event(raft_engine* e) {
  if (e->ev_used == e->ev.size()) {
    hipEvent_t x;
    if (hipEventCreate(&x) != hipSuccess) return nullptr;
    e->ev.push_back(x);
  }
  return e->ev[e->ev_used++];
}

int check_distinct(const raft_engine* e, const uint64_t* first, size_t stride, size_t n) {
  std::vector<uint64_t> gs(n);
  for (size_t i = 0; i < n; ++i) {
    gs[i] = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(first) + i * stride);
    if (gs[i] >= e->cfg.groups) return fail(RAFT_EINVAL, "batch element %zu: group %llu out of range", i,
                                           (unsigned long long)gs[i]);
  }
  std::sort(gs.begin(), gs.end());
  for (size_t i = 1; i < n; ++i)
    if (gs[i] == gs[i - 1])
      return fail(RAFT_EINVAL, "batch targets group %llu twice; batches need distinct groups",
                  (unsigned long long)gs[i]);
  return RAFT_OK;
}

// Runs a prepared DevOp batch (+ entries) through ops_kernel and returns the results.
int run_ops(raft_engine* e, int64_t now_tick, const std::vector<DevOp>& ops, const std::vector<int32_t>& et,
            const std::vector<int64_t>& ev, const std::vector<uint32_t>& ec, std::vector<DevRes>& res) {
  const size_t n = ops.size();
  res.assign(n, DevRes{});
  if (!n) return RAFT_OK;
  if (int rc = check_ticks(e, now_tick, 1)) return rc;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t b_ops = al(n * sizeof(DevOp)), b_res = al(n * sizeof(DevRes));
  const size_t b_et = al(et.size() * 4 + 4), b_ev = al(ev.size() * 8 + 8), b_ec = al(ec.size() * 4 + 4);
  if (int rc = ensure_stage(e, b_ops + b_res + b_et + b_ev + b_ec)) return rc;
  char* base = static_cast<char*>(e->stage);
  DevOp* d_ops = reinterpret_cast<DevOp*>(base);
  DevRes* d_res = reinterpret_cast<DevRes*>(base + b_ops);
  int32_t* d_et = reinterpret_cast<int32_t*>(base + b_ops + b_res);
  int64_t* d_ev = reinterpret_cast<int64_t*>(base + b_ops + b_res + b_et);
  uint32_t* d_ec = reinterpret_cast<uint32_t*>(base + b_ops + b_res + b_et + b_ev);
  HIPCHK(hipMemcpyAsync(d_ops, ops.data(), n * sizeof(DevOp), hipMemcpyHostToDevice, e->stream));
  if (!et.empty()) {
    HIPCHK(hipMemcpyAsync(d_et, et.data(), et.size() * 4, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(d_ev, ev.data(), ev.size() * 8, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(d_ec, ec.data(), ec.size() * 4, hipMemcpyHostToDevice, e->stream));
  }
  const Trace T = make_trace(e, now_tick);
  HIPCHK(launch_ops(e->R, int(e->cfg.semantics), e->P, T, d_ops, uint32_t(n), d_et, d_ev, d_ec, d_res, e->stream));
  HIPCHK(hipMemcpyAsync(res.data(), d_res, n * sizeof(DevRes), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RAFT_OK;
}

template <typename T>
int d2h(raft_engine* e, std::vector<T>& h, const T* d, size_t n) {
  h.resize(n);
  HIPCHK(hipMemcpyAsync(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, e->stream));
  return RAFT_OK;
}
template <typename T>
int h2d(raft_engine* e, T* d, const std::vector<T>& h) {
  HIPCHK(hipMemcpyAsync(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, e->stream));
  return RAFT_OK;
}

// Group records <-> per-row host arrays [Gp][R] (row k of group g at
// blk[g*recw + k*R ..], raft_device.hpp rix)
void rec_rows(const std::vector<int32_t>& blk, int k, uint64_t R, uint64_t Gp, std::vector<int32_t>& out) {
  const uint64_t W = recw_of(uint32_t(R));
  out.resize(R * Gp);
  for (uint64_t g = 0; g < Gp; ++g)
    std::memcpy(&out[g * R], &blk[g * W + uint64_t(k) * R], R * 4);
}
void rec_put(std::vector<int32_t>& blk, int k, uint64_t R, uint64_t Gp, const std::vector<int32_t>& rows) {
  const uint64_t W = recw_of(uint32_t(R));
  for (uint64_t g = 0; g < Gp; ++g)
    std::memcpy(&blk[g * W + uint64_t(k) * R], &rows[g * R], R * 4);
}

}  // namespace

extern "C" {

void raft_config_default(raft_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof *c);
  c->abi_version = RAFT_ABI_VERSION;
  c->replicas = 3;                 // main.go:81
  c->groups = 1;
  c->ring_depth = 32;
  c->entries_per_tick = 1;
  c->client_period = 5;            // one client write per 10 s (main.go:89) at 2 s per tick
  c->semantics = RAFT_SEM_REF;
  c->seed = 0x5EED0001ULL;
  c->tick_seconds = 2;             // main.go:394
  c->follower_timeout_min = 10;    // main.go:114
  c->follower_timeout_span = 20;
  c->candidate_timeout_min = 10;   // main.go:194
  c->candidate_timeout_span = 4;
  c->isolate_min_ticks = 8;
  c->isolate_max_ticks = 32;
  c->device = 0;
  c->ticks_per_launch = 1;         // one tick per launch
}

const char* raft_last_error(void) { return g_err.c_str(); }

int raft_engine_create(const raft_config* cfg, raft_engine** out) {
  if (!cfg || !out) return fail(RAFT_EINVAL, "null argument");
  *out = nullptr;
  const raft_config& c = *cfg;
  if (c.abi_version != RAFT_ABI_VERSION) return fail(RAFT_EINVAL, "abi_version %u != %u", c.abi_version, RAFT_ABI_VERSION);
  if (c.replicas < 1 || c.replicas > RAFT_MAX_REPLICAS) return fail(RAFT_EINVAL, "replicas must be 1..8");
  if (c.groups < 1) return fail(RAFT_EINVAL, "groups must be >= 1");
  if (c.ring_depth < 2 || c.ring_depth > 4096 || (c.ring_depth & (c.ring_depth - 1)))
    return fail(RAFT_EINVAL, "ring_depth must be a power of two in [2, 4096]");
  if (c.semantics != RAFT_SEM_REF && c.semantics != RAFT_SEM_RAFT)
    return fail(RAFT_EINVAL, "semantics must be RAFT_SEM_REF or RAFT_SEM_RAFT");
  if (c.tick_seconds < 1) return fail(RAFT_EINVAL, "tick_seconds must be >= 1");
  if (c.follower_timeout_min < 1 || c.follower_timeout_span < 1 || c.candidate_timeout_min < 1 ||
      c.candidate_timeout_span < 1 || c.follower_timeout_min + c.follower_timeout_span > 1024 ||
      c.candidate_timeout_min + c.candidate_timeout_span > 1024)
    return fail(RAFT_EINVAL, "timer ranges must be >= 1 and below 1024 s (10-bit duration field)");
  if (c.isolate_per_65536 > 65536) return fail(RAFT_EINVAL, "isolate_per_65536 must be <= 65536");
  if (c.payload_crc > 1) return fail(RAFT_EINVAL, "payload_crc must be 0 or 1");
  if (c.corrupt_per_65536 > 65536) return fail(RAFT_EINVAL, "corrupt_per_65536 must be <= 65536");
  if (c.isolate_leader > 1) return fail(RAFT_EINVAL, "isolate_leader must be 0 or 1");
  if (c.isolate_per_65536 &&
      (c.isolate_min_ticks < 1 || c.isolate_max_ticks > 32 || c.isolate_min_ticks > c.isolate_max_ticks))
    return fail(RAFT_EINVAL, "isolation length must satisfy 1 <= min <= max <= 32");
  if (c.ticks_per_launch > 64) return fail(RAFT_EINVAL, "ticks_per_launch must be 0..64 (0 and 1: one tick per launch)");
  if (c.debug_flags & ~RAFT_DEBUG_ALLOW_WRONG_RESULTS) return fail(RAFT_EINVAL, "unknown debug_flags bits");
  if (c.client_source > RAFT_CLIENT_STAGED) return fail(RAFT_EINVAL, "client_source must be RAFT_CLIENT_TRACE or RAFT_CLIENT_STAGED");
  for (uint32_t w : c.reserved)
    if (w) return fail(RAFT_EINVAL, "reserved config words must be 0");
  // RAFTSTEP_DIAG_LEAN (timing diagnostics of the lean / list kernels) skips
  // work and makes results wrong: refused unless the caller says so explicitly
  uint32_t diag_lean = 0;
  if (const char* dl = getenv("RAFTSTEP_DIAG_LEAN")) diag_lean = uint32_t(atoi(dl));
  if (diag_lean && !(c.debug_flags & RAFT_DEBUG_ALLOW_WRONG_RESULTS))
    return fail(RAFT_EINVAL, "RAFTSTEP_DIAG_LEAN=%u makes results wrong; set debug_flags RAFT_DEBUG_ALLOW_WRONG_RESULTS "
                "to accept it", diag_lean);
  const uint64_t Gp = (c.groups + 255) & ~uint64_t(255);
  // device addressing (raft_device.hpp at(), rix()): 64-bit plane/tile bases,
  // 32-bit per-lane BYTE offsets, so the group records (NPL rows of R 4-B
  // words) must satisfy Gp*NPL*R*4 < 2^32 (ring tiles: KP*64*R*8 < 2^26)
  if (Gp * recw_of(c.replicas) * 4 > uint64_t(0xFFFFFFFFu))
    return fail(RAFT_EINVAL, "too many groups for one engine (need groups * %u * 4 < 2^32)", recw_of(c.replicas));
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RAFT_ENODEV, "no HIP device");
  if (c.device < 0 || c.device >= ndev) return fail(RAFT_ENODEV, "device %d out of range", c.device);
  HIPCHK(hipSetDevice(c.device));

  raft_engine* e = new raft_engine();
  e->cfg = c;
  e->R = int(c.replicas);
  e->Gp = Gp;
  int rc = RAFT_OK;
  auto A = [&](void** p, size_t bytes) {
    if (rc == RAFT_OK) rc = dev_alloc(e, p, bytes);
  };
  const uint64_t R = c.replicas;
  // physical ring slots: 2K where groups can drift out of the global ring
  // phase (EXT isolation churn), so that their rotation can be switched in
  // place (raft_device.hpp ring_slot)
  // (and where shared entries stay through rejected copies, DevPlanes::sh_keep)
  const uint64_t phys = (c.isolate_per_65536 > 0 || (c.payload_crc && c.corrupt_per_65536)) ? 2 : 1;
  const uint64_t K = c.ring_depth * phys;
  e->KP = K;
  const bool raft = c.semantics == RAFT_SEM_RAFT;
  // group records: every per-replica row of a group in NPL*R contiguous words
  A(reinterpret_cast<void**>(&e->P.rec), Gp * recw_of(R) * 4);
  if (rc == RAFT_OK) {
    int32_t* rec = e->P.rec;
    e->P.term = rec + PL_TERM * R;
    e->P.last = rec + PL_LAST * R;
    e->P.commit = rec + PL_COMMIT * R;
    e->P.tstart = rec + PL_TSTART * R;
    e->P.lterm = rec + PL_LTERM * R;
    e->P.rs = rec + PL_RS * R;
    e->P.lmatch = rec + PL_LMATCH * R;
    if (raft) {   // NextIndex rows and high-water marks exist only in RAFT mode (null: REF)
      e->P.lnext = rec + PL_LNEXT * R;
      e->P.hwm = rec + PL_HWM * R;
    }
  }
  A(reinterpret_cast<void**>(&e->P.hb), Gp * 4);
  A(reinterpret_cast<void**>(&e->P.xmatch), R * R * Gp * 4);
  A(reinterpret_cast<void**>(&e->P.gmeta), Gp * 2);
  A(reinterpret_cast<void**>(&e->P.gseg), Gp * sizeof(GSeg));   // (grota / grotb / gsb2 / gshf: views, below)
  A(reinterpret_cast<void**>(&e->giso_plane), Gp);               // (DevPlanes::giso)
  A(reinterpret_cast<void**>(&e->P.gss), Gp * sizeof(SsRec));
  A(reinterpret_cast<void**>(&e->P.glx), Gp * sizeof(LxRec));
  A(reinterpret_cast<void**>(&e->P.grot), Gp * 2);
  A(reinterpret_cast<void**>(&e->P.gsb), Gp * 4);
  if (rc == RAFT_OK) {
    e->P.giso = Strided<uint8_t, 1>{e->giso_plane};
    e->P.grota = Strided<uint16_t, 16>{&e->P.gseg->rota};
    e->P.grotb = Strided<uint16_t, 16>{&e->P.gseg->rotb};
    e->P.gsb2 = Strided<int32_t, 16>{&e->P.gseg->sb2};
    e->P.gshf = Strided<int32_t, 16>{&e->P.gseg->shf};
  }
  // sharded group lists (raft_device.hpp): NSHARD shards of scap entries
  // shard chunks (raft_device.hpp shard_home): 2^sb consecutive blocks per
  // chunk, at most 64 blocks and at least NSHARD chunks over the engine's
  // blocks; a shard holds its chunks' groups (RAFTSTEP_SHARD_SB: A/B knob)
  const uint64_t nblk = (Gp + 255) / 256;
  uint32_t ssb = 0;
  while (ssb < 6 && (nblk >> (ssb + 1)) >= uint64_t(NSHARD)) ++ssb;
  if (const char* sv = getenv("RAFTSTEP_SHARD_SB")) ssb = uint32_t(std::min(6, std::max(0, atoi(sv))));
  const uint64_t nchunk = (nblk + (1ull << ssb) - 1) >> ssb;
  const uint64_t scap = ((nchunk + NSHARD - 1) / NSHARD) << (ssb + 8);
  for (int q = 0; q < NWORK; ++q) {
    A(reinterpret_cast<void**>(&e->work[q]), NSHARD * scap * 4);
    A(reinterpret_cast<void**>(&e->work_tick[q]), NSHARD * scap * 4);
  }
  A(reinterpret_cast<void**>(&e->wcount), WCOUNT_WORDS * 4);
  A(reinterpret_cast<void**>(&e->dctr), 64);
  // (each list: the group ids, then the words the lean kernel read for them,
  // raft_device.hpp LIST_WORDS: the list kernel stages those coalesced)
  for (int q = 0; q < 3; ++q) A(reinterpret_cast<void**>(&e->blist[q]), NSHARD * scap * 4 * LIST_WORDS);
  A(reinterpret_cast<void**>(&e->P.glst), Gp);
  A(reinterpret_cast<void**>(&e->P.log_term), R * K * Gp * 4);
  A(reinterpret_cast<void**>(&e->P.log_value), R * K * Gp * 8);
  if (c.payload_crc) A(reinterpret_cast<void**>(&e->P.log_crc), R * K * Gp * 4);
  // shared entries (raft_device.hpp ROT_SH): without EXT isolation churn (under
  // it groups leave the steady form too often for the copy-back to pay), with
  // slots below the rotation's flag bit; RAFTSTEP_SH=0 turns them off
  // (round 6: measured again under churn with every group closing its shared
  // form ahead of its next isolation window, so that no copy-back was needed:
  // C4 2.51 -> 2.18-2.23e10 — a wave's lanes then mix shared and R-copy
  // ring rows, and both kinds of row store go out with holes)
  e->P.sh = (c.isolate_per_65536 == 0 && K < ROT_SH) ? 1u : 0u;
  if (const char* sh = getenv("RAFTSTEP_SH"); sh && atoi(sh) == 0) e->P.sh = 0;
  if (const char* sh = getenv("RAFTSTEP_SH"); sh && atoi(sh) == 2 && K < ROT_SH) e->P.sh = 1;   // (also under churn)
  // REF with corrupted copies: the shared form survives a rejection (DevPlanes::sh_keep; KP = 2K above)
  e->P.sh_keep = (e->P.sh && !raft && c.payload_crc && c.corrupt_per_65536 && K >= 2ull * c.ring_depth) ? 1u : 0u;
  if (const char* sk = getenv("RAFTSTEP_SH_KEEP"); sk && atoi(sk) == 0) e->P.sh_keep = 0;
  // the shared ring's slot chunk (sh_in_tile): 16 consecutive slots of a group
  // contiguous where the list kernel writes whole batches of kept groups
  // (REF with corrupted copies, E >= 16: C5V); one row per slot otherwise
  e->P.sh_cs = (e->P.sh_keep && c.entries_per_tick >= 16 && (K & 15u) == 0) ? 4u : 0u;
  if (const char* cs = getenv("RAFTSTEP_SH_CHUNK"); cs && atoi(cs) == 0) e->P.sh_cs = 0;
  e->P.list_sort = 1;
  if (const char* ls = getenv("RAFTSTEP_LIST_SORT"); ls && atoi(ls) == 0) e->P.list_sort = 0;
  if (e->P.sh) {
    A(reinterpret_cast<void**>(&e->P.sh_term), K * Gp * 4);
    A(reinterpret_cast<void**>(&e->P.sh_value), K * Gp * 8);
    if (c.payload_crc) A(reinterpret_cast<void**>(&e->P.sh_crc), K * Gp * 4);
  }
  if (raft) A(reinterpret_cast<void**>(&e->P.xnext), R * R * Gp * 4);
  uint32_t* d_tab = nullptr;
  A(reinterpret_cast<void**>(&d_tab), 8 * 256 * 4);
  e->P.crc_tab = d_tab;
  if (rc == RAFT_OK) {
    hipError_t h = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (h == hipSuccess) h = hipStreamCreateWithFlags(&e->gen_stream, hipStreamNonBlocking);
    if (h == hipSuccess) h = hipStreamCreateWithFlags(&e->list_stream, hipStreamNonBlocking);
    if (h == hipSuccess) h = hipStreamCreateWithFlags(&e->half_stream, hipStreamNonBlocking);
    for (int q = 0; q < 2 && h == hipSuccess; ++q) h = hipEventCreateWithFlags(&e->ev_half[q], hipEventDisableTiming);
    for (int q = 0; q < 2 && h == hipSuccess; ++q) h = hipEventCreateWithFlags(&e->gen_ev[q], hipEventDisableTiming);
    for (int q = 0; q < 2 && h == hipSuccess; ++q) h = hipEventCreateWithFlags(&e->ev_lean[q], hipEventDisableTiming);
    for (int q = 0; q < 4 && h == hipSuccess; ++q) h = hipEventCreateWithFlags(&e->ev_list[q], hipEventDisableTiming);
    if (h == hipSuccess) h = hipEventCreateWithFlags(&e->ev_pp, hipEventDisableTiming);
    if (h != hipSuccess) rc = fail(RAFT_EHIP, "hipStreamCreate / hipEventCreate: %s", hipGetErrorString(h));
  }
  if (rc != RAFT_OK) {
    std::string keep = g_err;
    raft_engine_destroy(e);
    g_err = keep;
    return rc;
  }
  e->P.Gp = Gp;
  e->P.scap = uint32_t(scap);
  e->P.shard_sb = ssb;
  e->P.G = c.groups;
  e->P.gbase = c.group_base;
  e->P.K = c.ring_depth;
  e->P.KP = uint32_t(K);
  e->P.kmask = uint32_t(K) - 1;
  e->P.crc_on = c.payload_crc;
  e->P.rec_nt = Gp * 40 > (uint64_t(256) << 20) ? 1u : 0u;   // (raft_device.hpp DevPlanes::rec_nt)
  // virtual suffixes (M_VX): RAFT leader isolation without payload CRC; RAFTSTEP_VX=0 turns them off
  e->P.vx = (raft && c.isolate_per_65536 && c.isolate_leader && !c.payload_crc) ? 1u : 0u;
  if (const char* vx = getenv("RAFTSTEP_VX"); vx && atoi(vx) == 0) e->P.vx = 0;
  // a virtual suffix is regenerated from the trace RNG: never with staged client values
  if (c.client_source == RAFT_CLIENT_STAGED) e->P.vx = 0;
  e->P.cv = nullptr;   // (raft_stage_values)
  e->P.corrupt_p = c.corrupt_per_65536;
  if (const char* fg = getenv("RAFTSTEP_FORCE_GENERAL")) e->force_general = atoi(fg) != 0;
  if (const char* gk = getenv("RAFTSTEP_GENERAL")) e->lane_general = std::strcmp(gk, "lane") == 0;
  if (const char* se = getenv("RAFTSTEP_SLOW_EVERY")) e->slow_every = std::max(1, atoi(se));
  if (const char* dw = getenv("RAFTSTEP_DEBUG_WORK")) e->debug_work = atoi(dw) != 0;
  if (const char* dp = getenv("RAFTSTEP_DEBUG_PIPE")) e->debug_pipe = atoi(dp) != 0;
  if (const char* tp = getenv("RAFTSTEP_TWO_PASS")) e->two_pass = atoi(tp) != 0;
  e->P.diag = diag_lean;
  if (const char* sp = getenv("RAFTSTEP_SPLIT_STEADY")) e->split_steady = atoi(sp) != 0;

  // (the depths the oracle tests cover: 0..3, tests/test_gpu_pipeline.py)
  if (const char* og = getenv("RAFTSTEP_OVERLAP_GENERAL")) e->overlap_general = std::min(3, std::max(0, atoi(og)));
  if (const char* pp = getenv("RAFTSTEP_PIPELINE")) e->pipeline = atoi(pp) != 0;
  if (const char* pg = getenv("RAFTSTEP_PINGPONG")) e->pingpong = atoi(pg) != 0;
  e->fuse = std::max<uint32_t>(1u, c.ticks_per_launch);
  e->P.dbg_pass = 0xFFFFFFFFu;
  if (const char* df = getenv("RAFTSTEP_DEBUG_FAST"); df && atoi(df) != 0) {
    e->diag_print = 1;
    if (rc == RAFT_OK) rc = dev_alloc(e, reinterpret_cast<void**>(&e->P.dbg), RAFT_DIAG_DEVICE_COUNTERS * 8);
    if (rc == RAFT_OK && hipMemset(e->P.dbg, 0, RAFT_DIAG_DEVICE_COUNTERS * 8) != hipSuccess)
      rc = fail(RAFT_EHIP, "hipMemset failed");
    if (rc != RAFT_OK) {
      std::string keep = g_err;
      raft_engine_destroy(e);
      g_err = keep;
      return rc;
    }
  }
  // zero everything once so that padding / unused rows are deterministic
  for (void* p : e->allocs) (void)p;
  hipError_t z = hipSuccess;
  z = z == hipSuccess ? hipMemsetAsync(e->P.rec, 0, Gp * recw_of(R) * 4, e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->P.hb, 0x80, Gp * 4, e->stream) : z;  // 0x80808080 < any time
  z = z == hipSuccess ? hipMemsetAsync(e->P.xmatch, 0, R * R * Gp * 4, e->stream) : z;
  z = z == hipSuccess ? hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(e->P.gmeta), uint16_t(NO_PRIMARY), Gp,
                                           e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->P.gseg, 0, Gp * sizeof(GSeg), e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->giso_plane, 0, Gp, e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->P.glst, 0, Gp, e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->P.gss, 0, Gp * sizeof(SsRec), e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->P.glx, 0, Gp * sizeof(LxRec), e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->P.grot, 0, Gp * 2, e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->P.gsb, 0, Gp * 4, e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->wcount, 0, WCOUNT_WORDS * 4, e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->dctr, 0, 64, e->stream) : z;
  z = z == hipSuccess ? hipHostMalloc(reinterpret_cast<void**>(&e->hdone), 64, hipHostMallocCoherent) : z;
  if (z == hipSuccess) *e->hdone = 0u;
  z = z == hipSuccess ? hipMemsetAsync(e->P.log_term, 0, R * K * Gp * 4, e->stream) : z;
  z = z == hipSuccess ? hipMemsetAsync(e->P.log_value, 0, R * K * Gp * 8, e->stream) : z;
  if (c.payload_crc) z = z == hipSuccess ? hipMemsetAsync(e->P.log_crc, 0, R * K * Gp * 4, e->stream) : z;
  if (raft) z = z == hipSuccess ? hipMemsetAsync(e->P.xnext, 0, R * R * Gp * 4, e->stream) : z;
  z = z == hipSuccess ? hipMemcpyAsync(d_tab, crc_tab_host().data(), 8 * 256 * 4, hipMemcpyHostToDevice, e->stream) : z;
  z = z == hipSuccess ? hipStreamSynchronize(e->stream) : z;
  if (z != hipSuccess) {
    raft_engine_destroy(e);
    return fail(RAFT_EHIP, "initial memset: %s", hipGetErrorString(z));
  }
  *out = e;
  return RAFT_OK;
}

int raft_engine_destroy(raft_engine* e) {
  if (!e) return RAFT_OK;
  (void)hipSetDevice(e->cfg.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->comm_stream) (void)hipStreamSynchronize(e->comm_stream);
  if (e->comm) (void)ncclCommDestroy(e->comm);
  for (hipEvent_t x : e->ev) (void)hipEventDestroy(x);
  for (hipEvent_t x : e->comm_ev) (void)hipEventDestroy(x);
  for (hipEvent_t x : e->comm_pre) (void)hipEventDestroy(x);
  if (e->comm_stream) (void)hipStreamDestroy(e->comm_stream);
  if (e->gen_stream) (void)hipStreamSynchronize(e->gen_stream);
  if (e->list_stream) (void)hipStreamSynchronize(e->list_stream);
  if (e->half_stream) (void)hipStreamSynchronize(e->half_stream);
  for (hipEvent_t x : e->ev_half)
    if (x) (void)hipEventDestroy(x);
  for (hipEvent_t x : e->gen_ev)
    if (x) (void)hipEventDestroy(x);
  for (hipEvent_t x : e->ev_lean)
    if (x) (void)hipEventDestroy(x);
  for (hipEvent_t x : e->ev_list)
    if (x) (void)hipEventDestroy(x);
  if (e->ev_pp) (void)hipEventDestroy(e->ev_pp);
  if (e->gen_stream) (void)hipStreamDestroy(e->gen_stream);
  if (e->list_stream) (void)hipStreamDestroy(e->list_stream);
  if (e->half_stream) (void)hipStreamDestroy(e->half_stream);
  for (void* p : e->allocs) (void)hipFree(p);
  if (e->hist) (void)hipFree(e->hist);
  if (e->tstat) (void)hipFree(e->tstat);
  if (e->hrb) (void)hipHostFree(e->hrb);
  if (e->hdone) (void)hipHostFree(e->hdone);
  if (e->chk_ev) (void)hipEventDestroy(e->chk_ev);
  if (e->cstat) (void)hipFree(e->cstat);
  if (e->stage) (void)hipFree(e->stage);
  if (e->cvbuf) (void)hipFree(e->cvbuf);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return RAFT_OK;
}

int raft_engine_info(const raft_engine* e, raft_config* cfg_out, uint64_t* device_bytes) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  if (cfg_out) *cfg_out = e->cfg;
  if (device_bytes) *device_bytes = e->device_bytes;
  return RAFT_OK;
}

int raft_engine_features(const raft_engine* e, uint32_t* flags) {
  if (!e || !flags) return fail(RAFT_EINVAL, "null argument");
  *flags = (e->P.sh ? RAFT_FEATURE_SHARED_ENTRIES : 0u) | (e->P.vx ? RAFT_FEATURE_VIRTUAL_SUFFIXES : 0u);
  return RAFT_OK;
}

int raft_init_new_nodes(raft_engine* e, int64_t tick0) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  state_replacing(e);
  if (int rc = check_ticks(e, tick0, 1)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(launch_init_new(e->R, e->P, make_trace(e, tick0), e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  state_replaced(e);
  return RAFT_OK;
}

int raft_init_steady(raft_engine* e, int32_t leader, int64_t tick0) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  state_replacing(e);
  if (int rc = check_ticks(e, tick0, 1)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(launch_init_steady(e->R, e->P, make_trace(e, tick0), leader, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  state_replaced(e);
  e->steady_origin = true;   // empty logs; the list skip still needs a call that proves the list empty
  return RAFT_OK;
}

}  // extern "C"

namespace {

// Canonical view of groups [g0, g0+n): only that slice of every plane (and
// the ring tiles holding it) is copied out; the view is indexed by the
// local group g - g0.
int store_range(raft_engine* e, uint64_t g0, uint64_t n, raft_state_view* v) {
  HIPCHK(hipSetDevice(e->cfg.device));
  const uint64_t R = e->cfg.replicas, Gp = e->Gp, K = e->cfg.ring_depth;
  const bool raft = e->cfg.semantics == RAFT_SEM_RAFT;
  std::vector<int32_t> term, last, commit, ts, hb, lm, xm, lt, ln, xn, hw, rs, blk;
  std::vector<uint16_t> meta, rot, rota, rotb;
  std::vector<uint8_t> giso;
  std::vector<int32_t> sb, sb2;
  std::vector<int64_t> lv;
  std::vector<uint32_t> lcrc;
  const uint64_t W = recw_of(uint32_t(R));
  int rc = RAFT_OK;
  if (!rc) rc = d2h(e, blk, e->P.rec + g0 * W, n * W);   // group records (rows extracted below)
  if (!rc) rc = d2h(e, hb, e->P.hb + g0, n);
  // [R][R][Gp] rows of further leaders: R*R strided slices
  auto rows2d = [&](std::vector<int32_t>& h, const int32_t* d) -> int {
    h.resize(R * R * n);
    HIPCHK(hipMemcpy2DAsync(h.data(), n * 4, d + g0, Gp * 4, n * 4, R * R, hipMemcpyDeviceToHost, e->stream));
    return RAFT_OK;
  };
  if (!rc) rc = rows2d(xm, e->P.xmatch);
  if (!rc) rc = d2h(e, meta, e->P.gmeta + g0, n);
  std::vector<GSeg> cold;   // the packed cold words (GSeg), split below
  if (!rc && (v->iso_victim || v->log_term || v->log_value || v->log_crc)) rc = d2h(e, cold, e->P.gseg + g0, n);
  if (!rc && v->iso_victim) rc = d2h(e, giso, e->giso_plane + g0, n);

  if (!rc && raft) rc = rows2d(xn, e->P.xnext);
  const bool logs = v->log_term || v->log_value || v->log_crc;
  std::vector<int32_t> ltm;
  const uint64_t KP = e->KP;
  const uint64_t t0 = g0 >> 6, nt = ((g0 + n - 1) >> 6) - t0 + 1;   // ring tiles [t0, t0+nt)
  const uint64_t tile = KP * 64 * R;
  if (!rc && logs) rc = d2h(e, rot, e->P.grot + g0, n);
  if (!rc && logs) rc = d2h(e, sb, e->P.gsb + g0, n);

  std::vector<SsRec> gss;
  if (!rc) rc = d2h(e, gss, e->P.gss + g0, n);
  std::vector<LxRec> glx;
  if (!rc) rc = d2h(e, glx, e->P.glx + g0, n);
  if (!rc && logs) rc = d2h(e, lt, e->P.log_term + t0 * tile, nt * tile);
  if (!rc && logs) rc = d2h(e, lv, e->P.log_value + t0 * tile, nt * tile);
  const bool crcs = v->log_crc && e->cfg.payload_crc;
  if (!rc && crcs) rc = d2h(e, lcrc, e->P.log_crc + t0 * tile, nt * tile);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(e->stream));
  if (!cold.empty()) {   // (the packed cold words, copied above, split after the copy completed)
    rota.resize(n);
    rotb.resize(n);
    sb2.resize(n);
    for (uint64_t g = 0; g < n; ++g) {
      rota[g] = cold[g].rota;
      rotb[g] = cold[g].rotb;
      sb2[g] = cold[g].sb2;
    }
  }
  rec_rows(blk, PL_TERM, R, n, term);
  rec_rows(blk, PL_LAST, R, n, last);
  rec_rows(blk, PL_COMMIT, R, n, commit);
  rec_rows(blk, PL_TSTART, R, n, ts);
  rec_rows(blk, PL_RS, R, n, rs);
  rec_rows(blk, PL_LMATCH, R, n, lm);
  if (raft) rec_rows(blk, PL_LNEXT, R, n, ln);
  if (raft) rec_rows(blk, PL_HWM, R, n, hw);
  if (logs) rec_rows(blk, PL_LTERM, R, n, ltm);
  std::vector<int32_t>().swap(blk);
  // SSYNC groups: the planes are stale, the gss record (+ glx) is the state
  for (uint64_t g = 0; g < n; ++g) {
    const int pr = meta[g] & 0xF;
    if (!(meta[g] & M_SSYNC) || pr >= int(R)) continue;
    for (uint64_t r = 0; r < R; ++r) {
      term[g * R + r] = ss_term(gss[g], int(r), meta[g], glx[g]);
      last[g * R + r] = ss_last(gss[g], int(r), pr, meta[g], glx[g]);
      commit[g * R + r] = ss_commit(gss[g], int(r), pr, meta[g], glx[g], commit[g * R + r]);
      if (!ltm.empty()) ltm[g * R + r] = ss_term(gss[g], int(r), meta[g], glx[g]);
    }
  }
  for (uint64_t g = 0; g < n; ++g) {
    const int primary = meta[g] & 0xF;
    const bool msync = meta[g] & M_MSYNC;
    const LxRec lxg = (meta[g] & M_SSYNC) ? glx[g] : LxRec{0, 0};
    const uint64_t gt = g0 + g - t0 * 64;   // group index inside the copied ring tiles
    if (v->fault) v->fault[g] = uint8_t((meta[g] >> 4) & 7);
    if (v->iso_victim) v->iso_victim[g] = giso[g];
    for (uint64_t r = 0; r < R; ++r) {
      const uint64_t d = g * R + r, c = g * R + r;   // per-replica planes are group-major (rix)
      const int role = rs[d] & 3;
      if (v->role) v->role[c] = uint8_t(role);
      if (v->voted) v->voted[c] = uint8_t((rs[d] >> 2) & 15);
      if (v->term) v->term[c] = term[d];
      if (v->last) v->last[c] = last[d];
      if (v->commit) v->commit[c] = commit[d];
      // deadline = effective timer start + d; followers/candidates also count hb
      if (v->deadline) v->deadline[c] = (role == ROLE_L ? ts[d] : std::max(ts[d], hb[g])) + int32_t(rs[d] >> 6);
      if (v->timeout) v->timeout[c] = int32_t(rs[d] >> 6);
      // RAFT + MSYNC: high-water marks and the primary's NextIndex row are implicit too
      // (MSYNC: max(plane, LastApplied), raft_device.hpp M_HWX)
      const int32_t hwm = raft ? (msync ? std::max(hw[d], last[d]) : hw[d]) : last[d];
      if (v->hwm) v->hwm[c] = hwm;
      if (v->match)
        for (uint64_t p = 0; p < R; ++p) {
          int32_t m = 0;
          if (role == ROLE_L && p != r)
            m = (int(r) == primary) ? (msync_peer(meta[g], lxg, int(p)) ? last[g * R + p] : lm[g * R + p])
                                    : xm[(r * R + p) * n + g];
          v->match[c * R + p] = m;
        }
      if (v->next)
        for (uint64_t p = 0; p < R; ++p) {
          int32_t nx = 0;
          if (role == ROLE_L && p != r) {
            const bool mp = msync_peer(meta[g], lxg, int(p));
            if (raft) nx = (int(r) == primary) ? (mp ? last[g * R + p] + 1 : ln[g * R + p]) : xn[(r * R + p) * n + g];
            else nx = ((int(r) == primary) ? (mp ? last[g * R + p] : lm[g * R + p]) : xm[(r * R + p) * n + g]) + 1;
          }
          v->next[c * R + p] = nx;
        }
      // physical slot of entry idx (raft_device.hpp ring_slot)
      auto pslot = [&](int64_t idx) {
        return uint64_t((idx - 1 + (idx >= sb[g] ? rot[g] : (idx >= sb2[g] ? rota[g] : rotb[g]))) & int64_t(KP - 1));
      };
      if (logs && last[d] > 0) {
        const int32_t want = lt[ring_index(r, gt, pslot(last[d]), KP, R)];
        if (ltm[d] != want)
          return fail(RAFT_EINTERNAL, "last-entry term cache of group %llu replica %llu is %d, ring says %d",
                      (unsigned long long)(g0 + g), (unsigned long long)r, ltm[d], want);
      }
      if (logs) {
        const int64_t l = last[d];
        for (uint64_t s = 0; s < K; ++s) {
          // slot s holds the largest index i <= l with (i-1) mod K == s
          int64_t idx = l >= 1 ? l - ((l - 1 - int64_t(s)) & int64_t(K - 1)) : 0;
          const bool live = idx >= 1 && idx <= l && idx > int64_t(hwm) - int64_t(K);
          const uint64_t o = live ? ring_index(r, gt, pslot(idx), KP, R) : 0;
          if (v->log_term) v->log_term[c * K + s] = live ? lt[o] : 0;
          if (v->log_value) v->log_value[c * K + s] = live ? lv[o] : 0;
          if (v->log_crc) v->log_crc[c * K + s] = (live && crcs) ? lcrc[o] : 0u;
        }
      }
    }
  }
  return RAFT_OK;
}

}  // namespace

extern "C" {

int raft_store_state(raft_engine* e, raft_state_view* v) {
  if (!e || !v) return fail(RAFT_EINVAL, "null argument");
  if (int rc = settle_check(e)) return rc;
  if (int rc = ring_flush(e)) return rc;
  return store_range(e, 0, e->cfg.groups, v);
}

int raft_store_state_range(raft_engine* e, uint64_t first_group, uint64_t n_groups, raft_state_view* v) {
  if (!e || !v) return fail(RAFT_EINVAL, "null argument");
  if (n_groups == 0 || first_group >= e->cfg.groups || n_groups > e->cfg.groups - first_group)
    return fail(RAFT_ERANGE, "groups [%llu, +%llu) outside the engine's %llu", (unsigned long long)first_group,
                (unsigned long long)n_groups, (unsigned long long)e->cfg.groups);
  if (int rc = settle_check(e)) return rc;
  if (int rc = ring_flush(e)) return rc;
  return store_range(e, first_group, n_groups, v);
}

int raft_load_state(raft_engine* e, const raft_state_view* v) {
  if (e) state_replacing(e);
  if (!e || !v) return fail(RAFT_EINVAL, "null argument");
  if (!v->role || !v->voted || !v->term || !v->last || !v->commit || !v->deadline || !v->timeout ||
      !v->match || !v->fault || !v->log_term || !v->log_value)
    return fail(RAFT_EINVAL, "raft_load_state needs every field of the view");
  HIPCHK(hipSetDevice(e->cfg.device));
  const uint64_t R = e->cfg.replicas, G = e->cfg.groups, Gp = e->Gp, K = e->cfg.ring_depth;
  const uint64_t KP = e->KP;
  std::vector<int32_t> term(R * Gp, 0), last(R * Gp, 0), commit(R * Gp, 0), ts(R * Gp, 0), lm(R * Gp, 0),
      xm(R * R * Gp, 0), lt(R * KP * Gp, 0), hb(Gp, HB_NONE);
  std::vector<int32_t> rs(R * Gp, 0);
  std::vector<uint16_t> meta(Gp, uint16_t(NO_PRIMARY));
  std::vector<uint8_t> giso(Gp, 0);
  std::vector<int64_t> lv(R * KP * Gp, 0);
  std::vector<int32_t> ltm(R * Gp, 0);
  std::vector<uint32_t> lcrc(e->cfg.payload_crc ? R * KP * Gp : 0, 0);
  const bool raft = e->cfg.semantics == RAFT_SEM_RAFT;
  std::vector<int32_t> ln(raft ? R * Gp : 0, 0), xn(raft ? R * R * Gp : 0, 0), hw(raft ? R * Gp : 0, 0);
  const int max_vote = raft ? int(R) : 1;   // REF Voted bool; RAFT votedFor + 1
  for (uint64_t g = 0; g < G; ++g) {
    if (v->fault[g] > RAFT_F_OVERFLOW) return fail(RAFT_EINVAL, "group %llu: bad fault code", (unsigned long long)g);
    if (v->iso_victim) {   // nibbles 0 or 8 | replica
      const uint8_t x = v->iso_victim[g];
      for (int sh = 0; sh < 8; sh += 4) {
        const int nib = (x >> sh) & 0xF;
        if (nib && (!(nib & 8) || uint32_t(nib & 7) >= R))
          return fail(RAFT_EINVAL, "group %llu: bad iso_victim %#x", (unsigned long long)g, x);
      }
      giso[g] = x;
    }
    int primary = NO_PRIMARY;
    for (uint64_t r = 0; r < R; ++r) {
      const uint64_t c = g * R + r;
      if (v->role[c] > RAFT_LEADER || v->voted[c] > max_vote || v->last[c] < 0 || v->timeout[c] < 0 ||
          v->timeout[c] > 1023)
        return fail(RAFT_EINVAL, "group %llu replica %llu: field out of range", (unsigned long long)g,
                    (unsigned long long)r);
      if (v->role[c] == RAFT_LEADER && primary == NO_PRIMARY) primary = int(r);
    }
    bool steady = primary != NO_PRIMARY;
    for (uint64_t r = 0; r < R; ++r)
      if (int(r) != primary && v->role[g * R + r] != RAFT_FOLLOWER) steady = false;
    meta[g] = uint16_t(primary | (v->fault[g] << 4) | (steady ? M_STEADY : 0));
    for (uint64_t r = 0; r < R; ++r) {
      const uint64_t d = g * R + r, c = g * R + r;   // per-replica planes are group-major (rix)
      term[d] = v->term[c];
      last[d] = v->last[c];
      commit[d] = v->commit[c];
      ts[d] = v->deadline[c] - v->timeout[c];
      rs[d] = int32_t(v->role[c] | (v->voted[c] << 2) | (uint32_t(v->timeout[c]) << 6));
      if (v->role[c] == RAFT_LEADER)
        for (uint64_t p = 0; p < R; ++p) {
          if (p == r) continue;
          const int32_t m = v->match[c * R + p];
          // RAFT: NextIndex as given, 0/absent derives match+1 (the oracle's rule)
          const int32_t nx = (v->next && v->next[c * R + p] > 0) ? v->next[c * R + p] : m + 1;
          if (int(r) == primary) {
            lm[g * R + p] = m;
            if (raft) ln[g * R + p] = nx;
          } else {
            xm[(r * R + p) * Gp + g] = m;
            if (raft) xn[(r * R + p) * Gp + g] = nx;
          }
        }
      if (raft) {
        const int32_t h = (v->hwm && v->hwm[c] > v->last[c]) ? v->hwm[c] : v->last[c];
        if (v->last[c] > 0 && int64_t(v->last[c]) <= int64_t(h) - int64_t(K))
          return fail(RAFT_EINVAL, "group %llu replica %llu: last entry outside the ring window (hwm - K, hwm]",
                      (unsigned long long)g, (unsigned long long)r);
        hw[d] = h;
      }
      // view slot s = (idx-1) mod K; loaded rings use rotation 0 (physical slot (idx-1) mod KP).
      // With KP == K every slot is copied as is; with KP = 2K only the entries the view
      // holds for indices <= LastApplied (the others can never be read).
      const int64_t l = v->last[c];
      for (uint64_t s = 0; s < K; ++s) {
        uint64_t ps = s;
        if (KP != K) {
          const int64_t idx = l >= 1 ? l - ((l - 1 - int64_t(s)) & int64_t(K - 1)) : 0;
          if (idx < 1) continue;
          ps = uint64_t(idx - 1) & (KP - 1);
        }
        const uint64_t o = ring_index(r, g, ps, KP, R);
        lt[o] = v->log_term[c * K + s];
        lv[o] = v->log_value[c * K + s];
        if (e->cfg.payload_crc)
          lcrc[o] = v->log_crc ? v->log_crc[c * K + s] : host_entry_crc(v->log_term[c * K + s], v->log_value[c * K + s]);
      }
      if (v->last[c] > 0) ltm[d] = v->log_term[c * K + uint64_t((v->last[c] - 1) & int64_t(K - 1))];
    }
  }
  std::vector<int32_t> blk(Gp * recw_of(R), 0);   // group records
  rec_put(blk, PL_TERM, R, Gp, term);
  rec_put(blk, PL_LAST, R, Gp, last);
  rec_put(blk, PL_COMMIT, R, Gp, commit);
  rec_put(blk, PL_TSTART, R, Gp, ts);
  rec_put(blk, PL_LTERM, R, Gp, ltm);
  rec_put(blk, PL_RS, R, Gp, rs);
  rec_put(blk, PL_LMATCH, R, Gp, lm);
  if (raft) rec_put(blk, PL_LNEXT, R, Gp, ln);
  if (raft) rec_put(blk, PL_HWM, R, Gp, hw);
  int rc = RAFT_OK;
  if (!rc) rc = h2d(e, e->P.rec, blk);
  if (!rc) rc = h2d(e, e->P.hb, hb);
  if (!rc) rc = h2d(e, e->P.xmatch, xm);
  if (!rc) rc = h2d(e, e->P.gmeta, meta);
  const std::vector<GSeg> cold(Gp, GSeg{});   // loaded rings: rotation 0, one segment
  if (!rc) rc = h2d(e, e->P.gseg, cold);
  if (!rc) rc = h2d(e, e->giso_plane, giso);   // the isolation victims
  const std::vector<uint16_t> rot(Gp, 0);
  const std::vector<int32_t> sb0(Gp, 0);
  if (!rc) rc = h2d(e, e->P.grot, rot);
  if (!rc) rc = h2d(e, e->P.gsb, sb0);
  if (!rc && raft) rc = h2d(e, e->P.xnext, xn);
  if (!rc && e->cfg.payload_crc) rc = h2d(e, e->P.log_crc, lcrc);
  if (!rc) rc = h2d(e, e->P.log_term, lt);
  if (!rc) rc = h2d(e, e->P.log_value, lv);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(e->stream));
  state_replaced(e);
  return RAFT_OK;
}

static int wait_stream(raft_engine* e, hipStream_t s = nullptr);
static int comm_marker(raft_engine* e, hipStream_t s);

// Stats of the window [w0, w1] (indices into this call's ticks) are final
// once its general kernel has run: reduce them to per-tick records and, with
// a communicator, sum those across GPUs on the comm stream (ordered by an
// event, overlapping the following ticks on the engine stream). The call's
// last flush also writes the end-of-call check record (chk); its sum (call_end)
// runs on the engine stream itself: nothing follows it to overlap, and the two
// cross-stream hops cost ~13 us each (round 4) — after the call's earlier sums
// on the comm stream, so the communicator sees its collectives in issue order.
static int flush_window_stats(raft_engine* e, uint32_t w0, uint32_t w1, const CallCheck* chk,
                              hipStream_t s = nullptr, bool call_end = false) {
  if (!s) s = e->stream;
  const uint32_t n = w1 - w0 + 1;
  // (the lean / fused kernels' statistics are exceptions to a base of every
  // group taking a normal tick: tick_common.hpp lean_stats)
  const LeanBase lb{e->call_lean ? e->cfg.groups : 0ull, e->call_t0 + int64_t(w0), e->cfg.entries_per_tick,
                    e->cfg.client_period, uint32_t(e->R), e->cfg.semantics == RAFT_SEM_RAFT ? 1u : 0u};
  HIPCHK(launch_stats_reduce(e->hist + size_t(w0) * STAT_TICK, e->tstat + size_t(w0) * NSTAT, n, lb, s, chk));
  if (!e->comm) return RAFT_OK;
  while (e->comm_ev.size() < 2) {
    hipEvent_t x;
    HIPCHK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    e->comm_ev.push_back(x);
  }
  hipStream_t cs = e->comm_stream;
  if (call_end) {
    if (e->comm_side) {
      HIPCHK(hipEventRecord(e->comm_ev[1], e->comm_stream));
      HIPCHK(hipStreamWaitEvent(s, e->comm_ev[1], 0));
      e->comm_side = false;
    }
    cs = s;
  } else {
    HIPCHK(hipEventRecord(e->comm_ev[0], s));
    HIPCHK(hipStreamWaitEvent(e->comm_stream, e->comm_ev[0], 0));
    e->comm_side = true;
  }
  if (int rc = comm_marker(e, cs)) return rc;
  RCCLCHK(ncclAllReduce(e->tstat + size_t(w0) * NSTAT, e->tstat + size_t(w0) * NSTAT, size_t(n) * NSTAT, ncclUint64,
                        ncclSum, e->comm, cs));
  ++e->allreduces;
  return RAFT_OK;
}

// Counters of two-pass list q (of 3).
static uint32_t* lcount(raft_engine* e, uint32_t q) { return e->wcount + (NWORK + q) * SHARD_WORDS; }

// Join of an overlapped general kernel (see raft_engine::overlap_general):
// the engine stream waits for gen_stream, the window tail clears the
// window's DEFER flags and zeroes its worklist, its ticks' records are reduced.
// (s: the stream of the next tick's lean kernel, the engine stream by default)
static int join_general(raft_engine* e, bool stats, hipStream_t s = nullptr) {
  if (!s) s = e->stream;
  HIPCHK(hipStreamWaitEvent(s, e->gen_ev[1], 0));
  HIPCHK(launch_window_tail(e->P, e->work[e->gen_parity], e->wcount, e->gen_parity, s));
  e->gen_pending = false;
  if (stats)
    if (int rc = flush_window_stats(e, e->gen_w0, e->gen_w1, nullptr, s)) return rc;
  return RAFT_OK;
}

// Stream of tick i of a ping-pong call (raft_engine::pingpong).
static hipStream_t pp_stream(const raft_engine* e, uint32_t i) { return (i & 1u) ? e->list_stream : e->stream; }

static int tick_impl(raft_engine* e, int64_t first_tick, uint32_t nticks, bool stats) {
  if (int rc = settle_check(e)) return rc;
  if (int rc = check_ticks(e, first_tick, nticks)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  if (e->gen_pending) {   // (only after a failed call: every call joins its general kernels)
    if (int rc = join_general(e, false)) return rc;
  }
  if (e->hist_dirty) {
    // a failed call's per-tick slots were never reduced (the reduce is what
    // re-zeroes them): zero every slot it may have counted into, after all of
    // its kernels are done, or the next call's stats would include them. Only
    // this engine's streams are joined (not the whole device, which
    // would wait on other engines too), the comm stream with wait_stream's bound.
    for (hipStream_t s : {e->gen_stream, e->list_stream, e->half_stream})
      if (s) HIPCHK(hipStreamSynchronize(s));
    if (e->comm_stream)
      if (int rc = wait_stream(e, e->comm_stream)) return rc;
    if (int rc = wait_stream(e)) return rc;
    HIPCHK(hipMemsetAsync(e->hist, 0, size_t(e->hist_dirty) * STAT_TICK * 8, e->stream));
    e->hist_dirty = 0;
  }
  // a failed call may have left groups in shared form with an unknown implied
  // heartbeat time: poison now, whatever tick this call starts at (ADVICE r5;
  // sh_flush below runs only for a call after a tick gap)
  if (e->sh_live && !e->sh_done)
    if (int rc = sh_heartbeat(e)) return rc;
  if (e->cfg.client_source == RAFT_CLIENT_STAGED && nticks &&
      (!e->cv_n || first_tick < e->cv_t0 || first_tick + int64_t(nticks) > e->cv_t0 + int64_t(e->cv_n)))
    return fail(RAFT_EINVAL, "client_source RAFT_CLIENT_STAGED: ticks [%lld, %lld) are not staged (raft_stage_values "
                "holds [%lld, %lld))", (long long)first_tick, (long long)(first_tick + nticks), (long long)e->cv_t0,
                (long long)(e->cv_t0 + e->cv_n));
  // (the per-tick records need nticks slots; the check records exist at any capacity)
  if (int rc = ensure_hist(e, stats ? std::max<uint32_t>(nticks, 1) : 1)) return rc;
  if (!nticks) return RAFT_OK;
  // virtual suffixes are defined by consecutive calls: another first tick flushes them first
  if (e->vx_live && first_tick != e->vx_tick)
    if (int rc = vx_flush(e)) return rc;
  if (stats) e->hist_dirty = nticks;   // (cleared once every reduce of this call is issued)
  if (e->P.vx) {   // (unknown until the call has issued all its launches)
    e->vx_live = true;
    e->vx_tick = -1;
  }
  // shared entries across a tick gap: copied back first (a group in shared
  // form out of the global ring phase would go to the list kernel, which a
  // list-skipping call does not run; a drifted group without them is the lean
  // kernel's own-segment case)
  if (e->sh_live && first_tick != e->sh_next)
    if (int rc = sh_flush(e)) return rc;
  if (e->P.sh) {   // (any lean / fused launch may leave shared entries)
    e->sh_live = true;
    e->sh_next = first_tick + int64_t(nticks);
    e->sh_done = false;   // (until the call has issued all its launches)
  }
  if (!e->run_valid || !e->run_done || first_tick != e->run_next) {   // a new run of consecutive calls
    e->contig_from = first_tick;
    e->run_valid = true;
  }
  e->run_next = first_tick + int64_t(nticks);
  e->run_done = false;
  const Trace T0 = make_trace(e, first_tick);
  int64_t win_first = first_tick;   // first tick of the current general-kernel window
  // steady-state list skip (see raft_engine): entries per tick at most E, so
  // LastApplied + E stays below 2^31 while E * (last tick + 2) does
  const bool skip_list = e->steady_ok && e->steady_origin && T0.iso_p == 0 && e->P.corrupt_p == 0 &&
                         !e->force_general && uint64_t(e->cfg.entries_per_tick) < e->cfg.ring_depth &&
                         double(e->cfg.entries_per_tick) * double(first_tick + int64_t(nticks) + 2) < 2.0e9;
  e->skipped_list = skip_list;
  e->n_ticks += nticks;
  if (skip_list) e->n_skip_ticks += nticks;
  const bool two = e->two_pass && !e->force_general;
  e->call_t0 = first_tick;
  e->call_lean = two && T0.iso_p == 0;   // (under isolation churn the lean kernel counts absolutely)
  const bool pipe = two && !skip_list && !e->debug_work && e->pipeline;
  const bool pp = pipe && e->pingpong;
  if (e->debug_pipe)
    fprintf(stderr, "raftstep: ticks %lld..%lld pipeline %d\n", (long long)first_tick,
            (long long)(first_tick + nticks - 1), int(pipe));
  const uint32_t fuse = (two && skip_list && !e->cfg.payload_crc && e->prof != 3) ? e->fuse : 1u;
  // split steady tick (see raft_engine::split_steady): halves of whole
  // 256-group blocks (A/B, round 4: giving the half stream 45% or 40% of the
  // groups, so that it would run ahead and the call-end join find it done,
  // was 2% / 9% slower than equal halves)
  const uint64_t Gs = e->cfg.groups;
  const uint64_t half = (Gs / 2) & ~uint64_t(255);
  const bool split = two && skip_list && fuse == 1 && e->split_steady && half >= 65536 && Gs - half >= 65536;

  bool half_busy = false;   // the half stream has work the engine stream has not joined
  auto join_half = [&]() -> int {
    if (!half_busy) return RAFT_OK;
    HIPCHK(hipEventRecord(e->ev_half[1], e->half_stream));
    HIPCHK(hipStreamWaitEvent(e->stream, e->ev_half[1], 0));
    half_busy = false;
    return RAFT_OK;
  };
  // the half stream starts after everything issued before this call (a
  // cross-stream wait costs ~10 us on the critical path: skipped when the
  // engine stream is idle already, e.g. after a call that read its stats back)
  if (split && hipStreamQuery(e->stream) != hipSuccess) {
    HIPCHK(hipEventRecord(e->ev_half[0], e->stream));
    HIPCHK(hipStreamWaitEvent(e->half_stream, e->ev_half[0], 0));
  }
  // every call that runs list kernels starts with the lists' counters zeroed
  // (a pipelined call's last list kernel leaves the carried list's count)
  if (two && !skip_list) HIPCHK(hipMemsetAsync(lcount(e, 0), 0, size_t(NLISTS) * SHARD_WORDS * 4, e->stream));
  uint32_t stats_first = 0;   // first tick (index in this call) whose records are not reduced yet
  hipEvent_t ra = nullptr, rb = nullptr;
  if (e->prof == 2) {
    ra = next_event(e);
    rb = next_event(e);
    if (!ra || !rb) return fail(RAFT_EHIP, "hipEventCreate failed");
    HIPCHK(hipEventRecord(ra, e->stream));
  }
  hipEvent_t prof_a = nullptr, prof_b = nullptr;   // profile mode 1, steady calls: the span of the call's launches
  for (uint32_t i = 0; i < nticks; ++i) {
    const int64_t t = first_tick + int64_t(i);
    const Trace T = make_trace(e, t);
    unsigned long long* st = stats ? e->hist + size_t(i) * STAT_TICK : nullptr;
    // worklist counter of this window; zeroed by the previous general kernel
    // (or at engine creation), so no per-call memset
    uint32_t* cnt = e->wcount + (e->wpar % NWORK) * SHARD_WORDS;
    hipEvent_t a = nullptr, b = nullptr;
    const bool fused = fuse > 1;
    if (e->prof == 1 && skip_list) {
      // steady calls (the lean or fused kernel alone, back to back): one
      // event pair spanning the call's launches — the start event on the
      // first dispatch, the stop event on the last — so that the kernels
      // run exactly as in the timed region (an event pair on every dispatch
      // puts ~9 us between them, and a kernel that starts on a drained
      // device runs ~1 us shorter than back to back)
      const uint32_t last_launch = fused ? (nticks - 1) / fuse * fuse : nticks - 1;
      if (i == 0) {
        prof_a = next_event(e);
        prof_b = next_event(e);
        if (!prof_a || !prof_b) return fail(RAFT_EHIP, "hipEventCreate failed");
        e->ev_ticks.push_back(nticks);
        a = prof_a;
      }
      if (i == last_launch && !split) b = prof_b;
    } else if (e->prof == 1 && (!fused || i % fuse == 0)) {
      a = next_event(e);
      b = next_event(e);
      if (!a || !b) return fail(RAFT_EHIP, "hipEventCreate failed");
      e->ev_ticks.push_back(fused ? std::min<uint32_t>(fuse, nticks - i) : 1u);
    }
    const int force = e->force_general;
    if (fused) {
      // fused steady ticks: one launch per `fuse` ticks (its first), stats of
      // each tick in its own record; the list counters rotate per tick as usual
      if (i % fuse == 0)
        HIPCHK(launch_tick_fused(e->R, int(e->cfg.semantics), e->P, T, int(std::min<uint32_t>(fuse, nticks - i)), st,
                                 e->blist[e->lpar % 3], lcount(e, e->lpar % 3), e->stream, a, b));
      ++e->lpar;
    } else if (pipe) {
      // lean(t) appends to list L; list(t) reads it, zeroes list L+2 (last
      // read by list(t-1), next filled by lean(t+2), which waits for list(t))
      const uint32_t L = e->lpar % 3;
      const bool carry = i + 1 < nticks;   // list(t) runs its groups through t+1 too
      const int lflags = (i > 0 ? 1 : 0) | (carry ? 2 : 0);
      hipEvent_t c = nullptr, d = nullptr;
      if (e->prof == 3) {
        c = next_event(e);
        d = next_event(e);
        if (!c || !d) return fail(RAFT_EHIP, "hipEventCreate failed");
      }
      // (ping-pong: lean(t) after lean(t-1) on the other stream; list(t-2),
      // which carried its groups through t-1, is before it on its own)
      hipStream_t cs = pp ? pp_stream(e, i) : e->stream;
      if (pp) {
        if (i >= 1) HIPCHK(hipStreamWaitEvent(cs, e->ev_lean[(i - 1) & 1], 0));
      } else if (i >= 2) {
        HIPCHK(hipStreamWaitEvent(e->stream, e->ev_list[(i - 2) & 3], 0));   // carried its groups through t-1
      }
      // (ping-pong: the events are the kernels' own stop events — no marker
      // packet between lean(t) and list(t): C4 +2.5% in an A/B, round 4)
      const bool evk = pp && !b;
      HIPCHK(launch_tick_lean(e->R, int(e->cfg.semantics), e->P, T, st, e->blist[L], lcount(e, L), lflags, cs, a,
                              evk ? e->ev_lean[i & 1] : b, 0, ~0ull, pp ? lcount(e, (L + 1) % 3) : nullptr));
      if (!evk) HIPCHK(hipEventRecord(e->ev_lean[i & 1], cs));
      if (!pp) HIPCHK(hipStreamWaitEvent(e->list_stream, e->ev_lean[i & 1], 0));
      ListNext nx{};
      if (carry) {   // tick t+1: its stats record, the worklist of its window
        const int np = int((e->wpar + ((i + 1) % e->slow_every == 0 ? 1u : 0u)) % NWORK);
        nx = ListNext{stats ? st + size_t(STAT_TICK) : nullptr, e->work[np], e->work_tick[np],
                      e->wcount + np * SHARD_WORDS};
      }
      // (the call's last list kernel zeroes nothing: list L+2 then still
      // counts the groups list(t-1) carried into this tick, which the
      // end-of-call check counts as listed at the last tick; every pipelined
      // call starts with the three lists' counters zeroed)
      HIPCHK(launch_tick_list(e->R, int(e->cfg.semantics), e->P, T, st, e->work[e->wpar % NWORK], e->work_tick[e->wpar % NWORK],
                              cnt, e->blist[L], lcount(e, L), (carry && !pp) ? lcount(e, (L + 2) % 3) : nullptr,
                              carry ? &nx : nullptr, pp ? cs : e->list_stream, c,
                              (pp && !d) ? e->ev_list[i & 3] : d));
      if (!(pp && !d)) HIPCHK(hipEventRecord(e->ev_list[i & 3], pp ? cs : e->list_stream));
      ++e->lpar;
    } else if (two) {
      // lean pass appends to list counter lpar, the list pass zeroes the other one
      hipEvent_t c = nullptr, d = nullptr;
      if (e->prof == 3 && !skip_list) {
        c = next_event(e);
        d = next_event(e);
        if (!c || !d) return fail(RAFT_EHIP, "hipEventCreate failed");
      }
      const uint32_t L = e->lpar % 3;
      const int sem = int(e->cfg.semantics);
      if (split) {   // the two halves on two streams (the span's stop event is recorded after the join)
        HIPCHK(launch_tick_lean(e->R, sem, e->P, T, st, e->blist[L], lcount(e, L), 0, e->stream, a,
                                nullptr, 0, half));
        HIPCHK(launch_tick_lean(e->R, sem, e->P, T, st, e->blist[L], lcount(e, L), 0, e->half_stream,
                                nullptr, nullptr, half, Gs - half));
        half_busy = true;
      } else {
        HIPCHK(launch_tick_two_pass(e->R, int(e->cfg.semantics), e->P, T, st, e->work[e->wpar % NWORK],
                                    e->work_tick[e->wpar % NWORK], cnt, e->blist[L], lcount(e, L),
                                    lcount(e, (L + 2) % 3), e->stream, a, b, c, d, skip_list));
      }
      ++e->lpar;
    } else {
      HIPCHK(launch_tick_fast(e->R, int(e->cfg.semantics), e->P, T, st, e->work[e->wpar % NWORK],
                              e->work_tick[e->wpar % NWORK], cnt, force, e->stream, a, b));
    }
    // the previous window's general kernel, overlapped with this tick's fast
    // kernels: the engine stream waits for it, then its window tail clears
    // its groups' DEFER (before the next tick's lean kernel) and its ticks'
    // records are final
    if (e->gen_pending && i >= e->gen_join) {
      // (ping-pong: on the stream of lean(t+1), after lean(t))
      hipStream_t js = pp ? pp_stream(e, i + 1) : e->stream;
      if (pp) HIPCHK(hipStreamWaitEvent(js, e->ev_lean[i & 1], 0));
      if (int rc = join_general(e, stats, js)) return rc;
    }
    // deferred groups catch up every slow_every ticks and at the end of the call
    if ((i + 1) % e->slow_every == 0 || i + 1 == nticks) {
      if (e->debug_work) {   // diagnostics: worklist size of each general-kernel launch (synchronising)
        uint32_t sh[SHARD_WORDS], nw = 0;
        HIPCHK(hipMemcpyAsync(sh, cnt, sizeof sh, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        for (int k = 0; k < NSHARD; ++k) nw += sh[k * SHARD_STRIDE];
        fprintf(stderr, "raftstep: general kernel ticks %lld..%lld worklist %u\n", (long long)win_first, (long long)t, nw);
      }
      const bool last = i + 1 == nticks;
      const int par = int(e->wpar % NWORK);
      // pipelined: the window's deferrals are complete once list(t) is done
      // (its second step, tick t+1, defers to the next window's worklist)
      hipStream_t after = pipe ? e->list_stream : e->stream;
      // (with the list skipped nothing can be deferred — only the list kernel
      // defers — so both worklists stay empty and there is nothing to catch up)
      // (pipelined, a window's general kernel must run through tick t+1 and
      // its tail come after the lean kernel of t+1, which leaves the groups
      // list(t) passed on alone even when list(t) deferred them at tick t:
      // so the pipeline always takes this form)
      const bool overlap = !skip_list && two && (e->overlap_general || pipe) && !last && !e->debug_work;
      if (overlap) {
        // beside the lean and list kernels of ticks t+1 .. t+d, through tick
        // t+d (its groups keep DEFER, so those kernels leave them alone; their
        // deferrals go to the other worklist): d = the overlap depth, within
        // the call and at most one window (the next window's general kernel
        // starts after this one has joined)
        const uint32_t d = std::min<uint32_t>({uint32_t(std::max(e->overlap_general, 1)), e->slow_every, nticks - 1 - i});
        if (pp) {   // ping-pong: list(t) and list(t-1) (tick t's deferrals) are on the two streams
          HIPCHK(hipStreamWaitEvent(e->gen_stream, e->ev_list[i & 3], 0));
          if (i >= 1) HIPCHK(hipStreamWaitEvent(e->gen_stream, e->ev_list[(i - 1) & 3], 0));
        } else {
          HIPCHK(hipEventRecord(e->gen_ev[0], after));
          HIPCHK(hipStreamWaitEvent(e->gen_stream, e->gen_ev[0], 0));
        }
        HIPCHK(launch_tick_slow(e->R, int(e->cfg.semantics), e->P, T0, first_tick, win_first, t + int64_t(d),
                                stats ? e->hist : nullptr, e->work[par], e->work_tick[par], cnt, nullptr,
                                e->lane_general, e->gen_stream));
        HIPCHK(hipEventRecord(e->gen_ev[1], e->gen_stream));
        e->gen_pending = true;
        e->gen_parity = par;
        e->gen_w0 = stats_first;
        e->gen_w1 = i;
        e->gen_join = i + d;
        e->gen_top = i + d;
        e->gen_stats = stats;
        ++e->n_general;
      } else if (!skip_list) {
        if (pp) {   // everything on list_stream (list(t) or list(t-1), a window join) before the engine stream
          HIPCHK(hipEventRecord(e->ev_pp, e->list_stream));
          HIPCHK(hipStreamWaitEvent(e->stream, e->ev_pp, 0));
        } else if (pipe) {
          HIPCHK(hipStreamWaitEvent(e->stream, e->ev_list[i & 3], 0));
        }
        HIPCHK(launch_tick_slow(e->R, int(e->cfg.semantics), e->P, T0, first_tick, win_first, t,
                                stats ? e->hist : nullptr, e->work[par], e->work_tick[par], cnt, nullptr,
                                e->lane_general, e->stream));
        HIPCHK(launch_window_tail(e->P, e->work[par], e->wcount, par, e->stream));
        ++e->n_general;
      }
      ++e->wpar;
      // per-tick records: reduced (and all-reduced) per window — an overlapped
      // window's once its general kernel has joined; with the list skipped
      // nothing overlaps them, so one reduce (and one all-reduce) at the end of
      // the call covers every tick (with a communicator too: a per-window
      // flush costs the split tick a cross-stream join each, 418-424 vs
      // 366-374 us per 20-tick call, round 4). The last one carries the check
      // record.
      CallCheck chk{e->wcount, par, skip_list ? 1 : 0, e->tstat + size_t(nticks) * NSTAT, int((e->lpar + 2) % 3),
                    nullptr, nullptr, nullptr, 0u};
      // the call's only reduce (every record in this launch), no communicator:
      // the records also go straight to the host (CallCheck::hout)
      e->mirror = stats && last && two && stats_first == 0 && !e->comm;
      if (e->mirror) {
        chk.hout = e->hrb;
        chk.hdone = e->hdone;
        chk.ctr = e->dctr;
        chk.seq = ++e->seq;
      }
      const bool wflush = !skip_list || last;
      if (stats && !overlap && wflush) {
        if (int rc = join_half()) return rc;
        // profile mode 1: the span of the call's launches ends with both
        // halves, before the reduce (raftstep.h)
        if (last && split && prof_b) {
          HIPCHK(hipEventRecord(prof_b, e->stream));
          prof_b = nullptr;
        }
        if (int rc = flush_window_stats(e, stats_first, i, (last && two) ? &chk : nullptr, nullptr, last)) return rc;
      }
      if (wflush) stats_first = i + 1;
      win_first = t + 1;
    }
  }
  if (int rc = join_half()) return rc;   // (the check record and the readback come after both halves)
  if (split && prof_b) HIPCHK(hipEventRecord(prof_b, e->stream));   // the span ends with both halves
  e->hist_dirty = 0;   // every reduce of the call is issued
  if (e->P.vx) e->vx_tick = first_tick + int64_t(nticks);
  e->sh_done = true;
  e->run_done = true;
  if (e->comm && e->comm_side) {   // the engine stream (readback, next call) waits for the side-stream sums
    HIPCHK(hipEventRecord(e->comm_ev[1], e->comm_stream));
    HIPCHK(hipStreamWaitEvent(e->stream, e->comm_ev[1], 0));
    e->comm_side = false;
  }
  if (!stats && skip_list) {
    // no readback in this call: the check record goes to tstat[cap + 1] and
    // its pinned copy is verified by the next call (settle_check)
    const CallCheck chk{e->wcount, int((e->wpar + NWORK - 1) % NWORK), 1, e->tstat + size_t(e->hist_cap + 1) * NSTAT,
                        int((e->lpar + 2) % 3), nullptr, nullptr, nullptr, 0u};
    HIPCHK(launch_stats_reduce(nullptr, nullptr, 0, LeanBase{}, e->stream, &chk));
    const size_t off = size_t(e->hist_cap + 1) * NSTAT;
    HIPCHK(hipMemcpyAsync(e->hrb + off, e->tstat + off, NSTAT * 8, hipMemcpyDeviceToHost, e->stream));
    if (!e->chk_ev) HIPCHK(hipEventCreateWithFlags(&e->chk_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(e->chk_ev, e->stream));
    e->pend_chk = true;
  }
  if (e->prof == 2) {
    HIPCHK(hipEventRecord(rb, e->stream));
    e->prof_n += nticks;
  }
  if (e->P.dbg && e->diag_print) {   // diagnostics: lane classes summed over this call's ticks (synchronising)
    unsigned long long d[64];
    HIPCHK(hipMemcpyAsync(d, e->P.dbg, sizeof d, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemsetAsync(e->P.dbg, 0, sizeof d, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    fprintf(stderr, "raftstep: ticks %lld..%lld lean:", (long long)first_tick, (long long)(first_tick + nticks - 1));
    for (int k = 0; k < 64; ++k) {
      if (k == 32) fprintf(stderr, " | list:");
      if (d[k]) fprintf(stderr, " %d=%llu", k & 31, d[k]);
    }
    fprintf(stderr, "\n");
  }
  return RAFT_OK;
}

// Waits for the engine stream. With a communicator the wait is bounded by
// RAFTSTEP_COMM_TIMEOUT_S: an all-reduce whose peers never arrive (a rank
// gone, or ranks issuing different collectives) aborts the communicator and
// poisons the engine with RAFT_ETIMEDOUT instead of hanging the caller.
// The clock times the collectives, not the call's compute: every
// all-reduce is preceded by a marker event on its stream (comm_pre, recorded
// by flush_window_stats / raft_comm_allreduce_stats), and the budget runs
// from the latest marker that has completed — i.e. only while an all-reduce
// (and the short compute after it) is outstanding, restarting whenever the
// call makes progress past another marker. Compute before the first marker
// always finishes and is waited for without a bound. The host sleeps between
// polls after the first 2 ms.
static int wait_stream(raft_engine* e, hipStream_t s) {
  if (!s) s = e->stream;
  if (!e->comm) {
    HIPCHK(hipStreamSynchronize(s));
    return RAFT_OK;
  }
  const double tmo = comm_timeout_s();
  const auto start = std::chrono::steady_clock::now();
  auto t0 = start;
  bool armed = false;            // a marker has completed: an all-reduce may be what is outstanding
  size_t seen = 0;               // markers known complete (they complete in issue order per stream)
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) {
      e->comm_pre_used = 0;
      return RAFT_OK;
    }
    if (q != hipErrorNotReady) return fail(RAFT_EHIP, "hipStreamQuery: %s", hipGetErrorString(q));
    const auto now = std::chrono::steady_clock::now();
    bool progress = false;
    while (seen < e->comm_pre_used && hipEventQuery(e->comm_pre[seen]) == hipSuccess) {
      ++seen;
      progress = true;
    }
    if (progress) {
      armed = true;
      t0 = now;
    }
    const double el = std::chrono::duration<double>(now - t0).count();
    if (armed && el > tmo) {
      (void)ncclCommAbort(e->comm);
      e->comm = nullptr;
      e->comm_pre_used = 0;
      e->poisoned = true;
      e->poison_msg = "RCCL statistics all-reduce did not complete within " + std::to_string(int(tmo)) +
                      " s (RAFTSTEP_COMM_TIMEOUT_S): communicator aborted";
      return fail(RAFT_ETIMEDOUT, "%s", e->poison_msg.c_str());
    }
    if (std::chrono::duration<double>(now - start).count() > 2e-3)
      std::this_thread::sleep_for(std::chrono::microseconds(50));
#if defined(__x86_64__) || defined(__i386__)
    else __builtin_ia32_pause();
#endif
  }
}

// A marker on stream s just before an all-reduce is enqueued there (wait_stream).
static int comm_marker(raft_engine* e, hipStream_t s) {
  if (e->comm_pre_used == e->comm_pre.size()) {
    hipEvent_t x;
    HIPCHK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    e->comm_pre.push_back(x);
  }
  HIPCHK(hipEventRecord(e->comm_pre[e->comm_pre_used++], s));
  return RAFT_OK;
}

// longest host spin on a mirrored call's completion word (raft_tick)
constexpr std::chrono::microseconds kMirrorSpin{2000};

int raft_tick(raft_engine* e, int64_t first_tick, uint32_t nticks, raft_tick_stats* out) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  if (int rc = tick_impl(e, first_tick, nticks, out != nullptr)) return rc;
  if (out) {
    std::memset(out, 0, sizeof *out);
    if (!nticks) return RAFT_OK;
    // one readback per call: the per-tick records (already summed over slots,
    // and over GPUs) and, behind them, the end-of-call check record
    const bool two = e->two_pass && !e->force_general;
    const size_t words = size_t(nticks + (two ? 1 : 0)) * NSTAT;
    if (e->mirror) {
      // the records are already in hrb: wait for the launch's completion flag
      // (spinning; the stream is polled too, so a failed launch ends the wait),
      // then for the stream (its completion signal follows within microseconds)
      // The spin is bounded: past kMirrorSpin the host blocks in
      // hipStreamSynchronize below instead of holding a core for a long call.
      const volatile uint32_t* done = e->hdone;
      const auto t_spin = std::chrono::steady_clock::now();
      for (uint32_t k = 1; *done != e->seq; ++k) {
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#endif
        if ((k & 1023u) == 0 && (hipStreamQuery(e->stream) != hipErrorNotReady ||
                                 std::chrono::steady_clock::now() - t_spin > kMirrorSpin))
          break;
      }
      e->mirror = false;
    } else {
      HIPCHK(hipMemcpyAsync(e->hrb, e->tstat, words * 8, hipMemcpyDeviceToHost, e->stream));
    }
    if (int rc = wait_stream(e)) return rc;
    e->last_stats_n = nticks;
    for (size_t i = 0; i < size_t(nticks) * NSTAT; ++i) out->v[i % NSTAT] += int64_t(e->hrb[i]);
    if (two) {
      const unsigned long long* c = e->hrb + size_t(nticks) * NSTAT;
      if (c[CHK_MAGIC] != 0x5241465443484Bull) {
        e->steady_ok = false;
        return fail(RAFT_EINTERNAL, "end-of-call check record missing");
      }
      if (e->skipped_list && c[CHK_LISTED]) {   // (the check block zeroed the list counters)
        e->poisoned = true;
        e->steady_ok = false;
        e->poison_msg = "steady-state list skip: " + std::to_string(c[CHK_LISTED]) +
                        " groups were passed to a list kernel that did not run (ticks lost)";
        return fail(RAFT_EINTERNAL, "%s", e->poison_msg.c_str());
      }
      // steady-state list skip: proven for the next call when nothing was
      // listed at the last tick and the last general window took nothing
      if (e->steady_origin) e->steady_ok = c[CHK_LISTED] == 0 && c[CHK_DEFERRED] == 0;
    }
  }
  return RAFT_OK;
}

int raft_stage_values(raft_engine* e, int64_t first_tick, uint32_t nticks, const int64_t* values) {
  if (!e || (nticks && !values)) return fail(RAFT_EINVAL, "null argument");
  if (e->cfg.client_source != RAFT_CLIENT_STAGED)
    return fail(RAFT_EINVAL, "raft_stage_values needs client_source RAFT_CLIENT_STAGED");
  if (int rc = check_ticks(e, first_tick, nticks)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  // every kernel that may read the previous values has finished once the
  // engine stream has: each call joins its other streams into it at its end
  HIPCHK(hipStreamSynchronize(e->stream));
  const uint64_t n = uint64_t(nticks) * e->cfg.entries_per_tick * e->cfg.groups;
  if (n > e->cv_cap) {
    if (e->cvbuf) HIPCHK(hipFree(e->cvbuf));
    e->cvbuf = nullptr;
    e->cv_cap = 0;
    e->cv_n = 0;
    e->P.cv = nullptr;
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&e->cvbuf), n * 8));
    e->cv_cap = n;
  }
  e->cv_n = 0;   // (until the copy has gone through)
  e->P.cv = nullptr;
  if (n) HIPCHK(hipMemcpy(e->cvbuf, values, n * 8, hipMemcpyHostToDevice));
  e->cv_t0 = first_tick;
  e->cv_n = nticks;
  e->P.cv = nticks ? e->cvbuf : nullptr;
  e->P.cv_t0 = first_tick;
  e->P.cv_stride = e->cfg.groups;
  e->P.cv_tstride = uint64_t(e->cfg.entries_per_tick) * e->cfg.groups;
  return RAFT_OK;
}

int raft_tick_records(raft_engine* e, uint32_t nticks, raft_tick_stats* per_tick) {
  if (!e || (nticks && !per_tick)) return fail(RAFT_EINVAL, "null argument");
  if (nticks > e->last_stats_n || !e->tstat)
    return fail(RAFT_ERANGE, "the last raft_tick call with statistics produced %u per-tick records", e->last_stats_n);
  HIPCHK(hipSetDevice(e->cfg.device));
  std::vector<unsigned long long> h(size_t(nticks) * NSTAT);
  HIPCHK(hipMemcpyAsync(h.data(), e->tstat, h.size() * 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  for (uint32_t t = 0; t < nticks; ++t)
    for (int s = 0; s < NSTAT; ++s) per_tick[t].v[s] = int64_t(h[size_t(t) * NSTAT + s]);
  return RAFT_OK;
}

int raft_sync(raft_engine* e) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(hipStreamSynchronize(e->stream));
  return settle_check(e);
}

int raft_append_entries_batch(raft_engine* e, int64_t now_tick, const raft_ae_req* reqs, size_t n,
                              const raft_log_entry* entries, size_t n_entries_total, raft_ae_resp* out) {
  if (!e || (n && (!reqs || !out))) return fail(RAFT_EINVAL, "null argument");
  if (int rc = settle_check(e)) return rc;
  if (int rc = ring_flush(e)) return rc;
  e->run_valid = false;   // host mutation: entries from here on are not the trace's
  e->steady_origin = e->steady_ok = false;   // host mutation (the list skip needs a fresh proof)
  if (n == 0) return RAFT_OK;
  if (int rc = check_distinct(e, &reqs[0].group, sizeof(raft_ae_req), n)) return rc;
  std::vector<DevOp> ops(n);
  std::vector<int32_t> et;
  std::vector<int64_t> ev;
  std::vector<uint32_t> ec;
  for (size_t i = 0; i < n; ++i) {
    const raft_ae_req& q = reqs[i];
    if (q.to >= e->cfg.replicas) return fail(RAFT_EINVAL, "req %zu: receiver out of range", i);
    if (!fits32(q.term) || !fits32(q.prev_log_index) || !fits32(q.prev_log_term) || !fits32(q.leader_commit))
      return fail(RAFT_EINVAL, "req %zu: term/index outside the int32 range of the engine", i);
    if (q.n_entries > uint64_t(I32) || q.entries_offset > n_entries_total ||
        q.n_entries > n_entries_total - q.entries_offset || (q.n_entries && !entries))
      return fail(RAFT_EINVAL, "req %zu: entries out of range", i);
    DevOp& o = ops[i];
    std::memset(&o, 0, sizeof o);
    o.group = q.group; o.replica = q.to; o.kind = OP_AE;
    o.term = int32_t(q.term); o.prev_idx = int32_t(q.prev_log_index);
    o.prev_term = int32_t(q.prev_log_term); o.lc = int32_t(q.leader_commit);
    o.n = uint32_t(q.n_entries);
    o.off = et.size();
    o.voff = ev.size();
    // only the last K entries of a request can land in the ring: their values
    // and stamps are staged; every term is (RAFT compares terms before it
    // truncates, HostSrc)
    const uint64_t K = e->cfg.ring_depth;
    const uint64_t j0 = q.n_entries > K ? q.n_entries - K : 0;
    o.skip = uint32_t(j0);
    for (uint64_t j = 0; j < q.n_entries; ++j) {
      const raft_log_entry& le = entries[q.entries_offset + j];
      if (!fits32(le.term)) return fail(RAFT_EINVAL, "req %zu: entry term outside int32", i);
      et.push_back(int32_t(le.term));
      if (j < j0) continue;
      ev.push_back(le.value);
      ec.push_back(e->cfg.payload_crc ? host_entry_crc(int32_t(le.term), le.value) : 0u);  // stamped on ingest
    }
  }
  std::vector<DevRes> res;
  if (int rc = run_ops(e, now_tick, ops, et, ev, ec, res)) return rc;
  for (size_t i = 0; i < n; ++i) {
    out[i].term = res[i].term;
    out[i].match_index = res[i].value;
    out[i].success = res[i].ok;
    out[i].fault = res[i].fault;
  }
  return RAFT_OK;
}

int raft_request_vote_batch(raft_engine* e, int64_t now_tick, const raft_vote_req* reqs, size_t n,
                            raft_vote_resp* out) {
  if (!e || (n && (!reqs || !out))) return fail(RAFT_EINVAL, "null argument");
  if (int rc = settle_check(e)) return rc;
  if (int rc = ring_flush(e)) return rc;
  e->run_valid = false;   // host mutation: entries from here on are not the trace's
  e->steady_origin = e->steady_ok = false;   // host mutation (the list skip needs a fresh proof)
  if (n == 0) return RAFT_OK;
  if (int rc = check_distinct(e, &reqs[0].group, sizeof(raft_vote_req), n)) return rc;
  std::vector<DevOp> ops(n);
  for (size_t i = 0; i < n; ++i) {
    const raft_vote_req& q = reqs[i];
    if (q.to >= e->cfg.replicas) return fail(RAFT_EINVAL, "req %zu: receiver out of range", i);
    if (q.candidate_id >= e->cfg.replicas) return fail(RAFT_EINVAL, "req %zu: candidate out of range", i);
    if (!fits32(q.term) || !fits32(q.last_log_index) || !fits32(q.last_log_term))
      return fail(RAFT_EINVAL, "req %zu: term/index outside int32", i);
    std::memset(&ops[i], 0, sizeof(DevOp));
    ops[i].group = q.group; ops[i].replica = q.to; ops[i].kind = OP_VR; ops[i].term = int32_t(q.term);
    // RAFT mode only (REF ignores them): CandidateId, LastLogIndex, LastLogTerm
    ops[i].arg = q.candidate_id;
    ops[i].prev_idx = int32_t(q.last_log_index);
    ops[i].prev_term = int32_t(q.last_log_term);
  }
  std::vector<DevRes> res;
  if (int rc = run_ops(e, now_tick, ops, {}, {}, {}, res)) return rc;
  for (size_t i = 0; i < n; ++i) {
    out[i].term = res[i].term;
    out[i].vote_granted = res[i].ok;
    out[i].fault = res[i].fault;
  }
  return RAFT_OK;
}

int raft_group_ops_batch(raft_engine* e, int64_t now_tick, const raft_group_op* ops_in, size_t n,
                         raft_op_result* out) {
  if (!e || (n && (!ops_in || !out))) return fail(RAFT_EINVAL, "null argument");
  if (int rc = settle_check(e)) return rc;
  if (int rc = ring_flush(e)) return rc;
  e->run_valid = false;   // host mutation: entries from here on are not the trace's
  e->steady_origin = e->steady_ok = false;   // host mutation (the list skip needs a fresh proof)
  if (n == 0) return RAFT_OK;
  if (int rc = check_distinct(e, &ops_in[0].group, sizeof(raft_group_op), n)) return rc;
  std::vector<DevOp> ops(n);
  for (size_t i = 0; i < n; ++i) {
    const raft_group_op& q = ops_in[i];
    if (q.replica >= e->cfg.replicas) return fail(RAFT_EINVAL, "op %zu: replica out of range", i);
    if (q.kind < RAFT_OP_CLIENT_APPEND || q.kind > RAFT_OP_LEADER_COMMIT)
      return fail(RAFT_EINVAL, "op %zu: unknown kind %u", i, q.kind);
    std::memset(&ops[i], 0, sizeof(DevOp));
    ops[i].group = q.group; ops[i].replica = q.replica; ops[i].kind = q.kind; ops[i].arg = q.arg;
  }
  std::vector<DevRes> res;
  if (int rc = run_ops(e, now_tick, ops, {}, {}, {}, res)) return rc;
  for (size_t i = 0; i < n; ++i) {
    out[i].status = res[i].status;
    out[i].fault = res[i].fault;
    out[i].value = res[i].value;
  }
  return RAFT_OK;
}

int raft_comm_unique_id(uint8_t id_out[128]) {
  if (!id_out) return fail(RAFT_EINVAL, "null argument");
  ncclUniqueId id;
  RCCLCHK(ncclGetUniqueId(&id));
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  std::memcpy(id_out, &id, 128);
  return RAFT_OK;
}

int raft_comm_init(raft_engine* e, int nranks, int rank, const uint8_t id[128]) {
  if (!e || !id) return fail(RAFT_EINVAL, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(RAFT_EINVAL, "bad rank/nranks");
  if (e->comm) return fail(RAFT_EINVAL, "communicator already attached");
  HIPCHK(hipSetDevice(e->cfg.device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  if (!e->comm_stream) HIPCHK(hipStreamCreateWithFlags(&e->comm_stream, hipStreamNonBlocking));
  // ncclCommInitRank blocks until every rank has joined: it runs on a helper
  // thread so that a missing rank, or ranks disagreeing on nranks or the id,
  // ends in RAFT_ETIMEDOUT with a message instead of a hang (the caller then
  // exits; a helper still blocked in RCCL is abandoned with the process)
  // (a helper that completes after the caller gave up finds the
  // job abandoned and aborts the communicator it made, so peers that did
  // finish their init see its rank leave instead of a rank that never
  // issues a collective; a retry starts a fresh job)
  struct InitJob {
    std::mutex m;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclResult_t r = ncclSuccess;
    ncclComm_t comm = nullptr;
  };
  auto job = std::make_shared<InitJob>();
  const int dev = e->cfg.device;
  std::thread([job, dev, nranks, rank, uid]() {
    ncclComm_t c = nullptr;
    ncclResult_t r = hipSetDevice(dev) == hipSuccess ? ncclCommInitRank(&c, nranks, uid, rank) : ncclInvalidUsage;
    std::lock_guard<std::mutex> lk(job->m);
    if (job->abandoned) {
      if (c) (void)ncclCommAbort(c);
      return;
    }
    job->r = r;
    job->comm = c;
    job->done = true;
    job->cv.notify_all();
  }).detach();
  const double tmo = comm_timeout_s();
  std::unique_lock<std::mutex> lk(job->m);
  if (!job->cv.wait_for(lk, std::chrono::duration<double>(tmo), [&] { return job->done; })) {
    job->abandoned = true;
    return fail(RAFT_ETIMEDOUT, "raft_comm_init: ncclCommInitRank(nranks=%d, rank=%d) did not complete within %.0f s "
                "(RAFTSTEP_COMM_TIMEOUT_S): a rank is missing, or the ranks disagree on nranks or the unique id",
                nranks, rank, tmo);
  }
  if (job->r != ncclSuccess)
    return fail(RAFT_ERCCL, "raft_comm_init: ncclCommInitRank(nranks=%d, rank=%d): %s", nranks, rank,
                ncclGetErrorString(job->r));
  e->comm = job->comm;
  int n = 0, r = -1;
  if (ncclCommCount(e->comm, &n) != ncclSuccess || ncclCommUserRank(e->comm, &r) != ncclSuccess || n != nranks ||
      r != rank) {
    (void)ncclCommAbort(e->comm);
    e->comm = nullptr;
    return fail(RAFT_ERCCL, "raft_comm_init: communicator has %d ranks / rank %d, asked for %d / %d", n, r, nranks, rank);
  }
  e->nranks = nranks;
  e->rank = rank;
  return RAFT_OK;
}

int raft_comm_info(raft_engine* e, int32_t* nranks, int32_t* rank, uint64_t* allreduces) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  int n = 1, r = 0;
  if (e->comm) {
    RCCLCHK(ncclCommCount(e->comm, &n));
    RCCLCHK(ncclCommUserRank(e->comm, &r));
  }
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  if (allreduces) *allreduces = e->allreduces;
  return RAFT_OK;
}

int raft_comm_allreduce_stats(raft_engine* e, raft_tick_stats* stats) {
  if (!e || !stats) return fail(RAFT_EINVAL, "null argument");
  if (!e->comm) return RAFT_OK;
  HIPCHK(hipSetDevice(e->cfg.device));
  if (!e->cstat) HIPCHK(hipMalloc(reinterpret_cast<void**>(&e->cstat), NSTAT * 8));
  std::vector<unsigned long long> h(NSTAT);
  for (int s = 0; s < NSTAT; ++s) h[s] = (unsigned long long)stats->v[s];
  HIPCHK(hipMemcpyAsync(e->cstat, h.data(), NSTAT * 8, hipMemcpyHostToDevice, e->stream));
  if (int rc = comm_marker(e, e->stream)) return rc;
  RCCLCHK(ncclAllReduce(e->cstat, e->cstat, NSTAT, ncclUint64, ncclSum, e->comm, e->stream));
  HIPCHK(hipMemcpyAsync(h.data(), e->cstat, NSTAT * 8, hipMemcpyDeviceToHost, e->stream));
  if (int rc = wait_stream(e)) return rc;
  for (int s = 0; s < NSTAT; ++s) stats->v[s] = int64_t(h[s]);
  return RAFT_OK;
}

int raft_profile_enable(raft_engine* e, int mode) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  if (mode < 0 || mode > 3) return fail(RAFT_EINVAL, "profile mode must be 0, 1, 2 or 3");
  HIPCHK(hipSetDevice(e->cfg.device));
  // events are created here, not inside the timed calls (hipEventCreate costs
  // tens of microseconds); more are added on demand
  while (mode && e->ev.size() < 128) {
    hipEvent_t x;
    HIPCHK(hipEventCreate(&x));
    e->ev.push_back(x);
  }
  e->prof = mode;
  e->ev_used = 0;
  e->ev_ticks.clear();
  e->prof_ms = 0.0;
  e->prof_n = 0;
  return RAFT_OK;
}

int raft_profile_read(raft_engine* e, double* total_ms, uint64_t* launches) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(hipStreamSynchronize(e->stream));
  for (size_t i = 0; i + 1 < e->ev_used; i += 2) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e->ev[i], e->ev[i + 1]));
    e->prof_ms += ms;
    if (e->prof != 2) e->prof_n += (e->prof == 1 && i / 2 < e->ev_ticks.size()) ? e->ev_ticks[i / 2] : 1u;   // mode 1: ticks
    // (mode 2 counts ticks as it records)
  }
  e->ev_used = 0;
  e->ev_ticks.clear();
  if (total_ms) *total_ms = e->prof_ms;
  if (launches) *launches = e->prof_n;
  return RAFT_OK;
}

// ---- diagnostics -----------------------------------------------------------

int raft_diag_enable(raft_engine* e, int on) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  HIPCHK(hipSetDevice(e->cfg.device));
  if (!e->dbg_buf && e->P.dbg) e->dbg_buf = e->P.dbg;   // (allocated at creation by RAFTSTEP_DEBUG_FAST)
  if (on && !e->dbg_buf) {
    if (int rc = dev_alloc(e, reinterpret_cast<void**>(&e->dbg_buf), RAFT_DIAG_DEVICE_COUNTERS * 8)) return rc;
  }
  if (e->dbg_buf) HIPCHK(hipMemsetAsync(e->dbg_buf, 0, RAFT_DIAG_DEVICE_COUNTERS * 8, e->stream));
  e->P.dbg = on ? e->dbg_buf : nullptr;   // (the buffer stays allocated; counting stops)
  e->n_ticks = e->n_skip_ticks = e->n_general = 0;
  HIPCHK(hipStreamSynchronize(e->stream));
  return RAFT_OK;
}

int raft_diag_read(raft_engine* e, uint64_t* counters, uint32_t n) {
  if (!e || (n && !counters)) return fail(RAFT_EINVAL, "null argument");
  if (n > RAFT_DIAG_COUNTERS) return fail(RAFT_ERANGE, "at most %u counters", RAFT_DIAG_COUNTERS);
  HIPCHK(hipSetDevice(e->cfg.device));
  uint64_t all[RAFT_DIAG_COUNTERS] = {};
  if (e->P.dbg) {
    HIPCHK(hipMemcpyAsync(all, e->P.dbg, RAFT_DIAG_DEVICE_COUNTERS * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemsetAsync(e->P.dbg, 0, RAFT_DIAG_DEVICE_COUNTERS * 8, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  all[RAFT_DIAG_TICKS] = e->n_ticks;
  all[RAFT_DIAG_TICKS_LIST_SKIPPED] = e->n_skip_ticks;
  all[RAFT_DIAG_GENERAL_LAUNCHES] = e->n_general;
  e->n_ticks = e->n_skip_ticks = e->n_general = 0;
  for (uint32_t i = 0; i < n; ++i) counters[i] = all[i];
  return RAFT_OK;
}

int raft_debug_group_words(raft_engine* e, uint64_t group, int32_t* out, uint32_t n) {
  if (!e || (n && !out)) return fail(RAFT_EINVAL, "null argument");
  if (group >= e->cfg.groups) return fail(RAFT_EINVAL, "group out of range");
  if (int rc = ring_flush(e)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  uint16_t meta = 0, rot = 0, rota = 0, rotb = 0;
  uint8_t iso = 0;
  int32_t hb = 0, sb = 0, sb2 = 0;
  SsRec ss{};
  LxRec lx{};
  HIPCHK(hipMemcpyAsync(&meta, e->P.gmeta + group, 2, hipMemcpyDeviceToHost, e->stream));
  GSeg cw{};
  HIPCHK(hipMemcpyAsync(&cw, e->P.gseg + group, sizeof cw, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&hb, e->P.hb + group, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&ss, e->P.gss + group, sizeof ss, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&lx, e->P.glx + group, sizeof lx, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&rot, e->P.grot + group, 2, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&sb, e->P.gsb + group, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(&iso, e->giso_plane + group, 1, hipMemcpyDeviceToHost));
  rota = cw.rota;
  rotb = cw.rotb;
  sb2 = cw.sb2;
  const int32_t w[RAFT_DEBUG_GROUP_WORDS] = {meta, iso, hb, ss.last, ss.term, ss.cl, ss.cf, lx.k, lx.dl, rot, rota, sb,
                                             rotb, sb2};
  for (uint32_t i = 0; i < n && i < RAFT_DEBUG_GROUP_WORDS; ++i) out[i] = w[i];
  return RAFT_OK;
}

int raft_stream_probe(int device, uint32_t replicas, uint64_t elems, uint32_t reps, uint32_t flags,
                      double* us_per_pass, double* bytes_per_pass) {
  if (!us_per_pass || !bytes_per_pass) return fail(RAFT_EINVAL, "null argument");
  if (replicas < 1 || replicas > RAFT_MAX_REPLICAS || elems < 64 || elems > (1ull << 26) || reps < 1)
    return fail(RAFT_EINVAL, "replicas 1..8, elems 64..2^26, reps >= 1");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return fail(RAFT_ENODEV, "no such device");
  HIPCHK(hipSetDevice(device));
  const uint64_t n = (elems + 255) & ~uint64_t(255), R = replicas, KS = 2;
  std::vector<void*> mem;
  auto alloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    mem.push_back(p);
    return hipMemset(p, 0, bytes) == hipSuccess ? p : nullptr;
  };
  auto* a = static_cast<uint16_t*>(alloc(n * 2));
  auto* b = static_cast<SsRec*>(alloc(n * sizeof(SsRec)));
  auto* c = static_cast<uint16_t*>(alloc(n * 2));
  auto* d = static_cast<int32_t*>(alloc(n * 4));
  auto* rt = static_cast<int32_t*>(alloc(n * KS * R * 4));
  auto* rv = static_cast<int64_t*>(alloc(n * KS * R * 8));
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = RAFT_OK;
  if (!a || !b || !c || !d || !rt || !rv) rc = fail(RAFT_ENOMEM, "stream probe: hipMalloc failed");
  if (rc == RAFT_OK && (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
                        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess))
    rc = fail(RAFT_EHIP, "stream probe: stream / event creation failed");
  float ms = 0.f;
  // (flags, raftstep.h RAFT_PROBE_*: bit 0 plain ring stores, bit 1 non-temporal record stores,
  // bit 2 no heartbeat store — the mix of a group in shared form, which bench.py selects for those
  // lines; the environment variable RAFTSTEP_PROBE_MODE replaces them, for A/Bs only)
  if (flags & ~7u) return fail(RAFT_EINVAL, "unknown stream probe flags");
  const char* pm = getenv("RAFTSTEP_PROBE_MODE");
  const uint32_t mode = pm ? uint32_t(atoi(pm)) & 7u : flags;
  if (rc == RAFT_OK) {
    hipError_t h = launch_stream_probe(int(R), a, b, c, d, rt, rv, uint32_t(n), 1u, uint32_t(KS), s, mode);
    if (h == hipSuccess) h = hipEventRecord(e0, s);
    for (uint32_t i = 0; i < reps && h == hipSuccess; ++i)
      h = launch_stream_probe(int(R), a, b, c, d, rt, rv, uint32_t(n), i & 1u, uint32_t(KS), s, mode);
    if (h == hipSuccess) h = hipEventRecord(e1, s);
    if (h == hipSuccess) h = hipEventSynchronize(e1);
    if (h == hipSuccess) h = hipEventElapsedTime(&ms, e0, e1);
    if (h != hipSuccess) rc = fail(RAFT_EHIP, "stream probe: %s", hipGetErrorString(h));
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (s) (void)hipStreamDestroy(s);
  for (void* p : mem) (void)hipFree(p);
  if (rc != RAFT_OK) return rc;
  *us_per_pass = double(ms) * 1e3 / reps;
  *bytes_per_pass = double(n) * double(((mode & 4u) ? 36 : 40) + 12 * R);   // (bit 2: no heartbeat store)
  return RAFT_OK;
}

int raft_debug_diag_mode(raft_engine* e, uint32_t mode) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  if (mode && !(e->cfg.debug_flags & RAFT_DEBUG_ALLOW_WRONG_RESULTS))
    return fail(RAFT_EINVAL, "diagnostic mode %u makes results wrong; create the engine with debug_flags "
                "RAFT_DEBUG_ALLOW_WRONG_RESULTS", mode);
  e->P.diag = mode;
  return RAFT_OK;
}

int raft_debug_force_pass(raft_engine* e, int64_t group) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  if (group >= int64_t(e->cfg.groups)) return fail(RAFT_EINVAL, "group out of range");
  e->P.dbg_pass = group < 0 ? 0xFFFFFFFFu : uint32_t(group);
  return RAFT_OK;
}

// ---- audit: digest, nodelog, checkpoints ----------------------------------

int raft_state_digest(raft_engine* e, uint64_t* per_group, uint64_t* total) {
  if (!e) return fail(RAFT_EINVAL, "null engine");
  if (int rc = settle_check(e)) return rc;
  if (int rc = vx_flush(e)) return rc;
  if (e->sh_live)   // (the digest reads shared entries and implied heartbeat times directly)
    if (int rc = sh_heartbeat(e)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  const uint64_t G = e->cfg.groups;
  uint64_t* d_pg = nullptr;
  unsigned long long* d_tot = nullptr;
  HIPCHK(hipMalloc(&d_pg, G * 8 + 64));
  d_tot = reinterpret_cast<unsigned long long*>(d_pg + G);
  int rc = RAFT_OK;
  hipError_t h = hipMemsetAsync(d_tot, 0, 8, e->stream);
  if (h == hipSuccess) h = launch_digest(e->R, e->P, e->cfg.semantics == RAFT_SEM_RAFT, d_pg, d_tot, e->stream);
  if (h == hipSuccess && per_group) h = hipMemcpyAsync(per_group, d_pg, G * 8, hipMemcpyDeviceToHost, e->stream);
  uint64_t tot = 0;
  if (h == hipSuccess) h = hipMemcpyAsync(&tot, d_tot, 8, hipMemcpyDeviceToHost, e->stream);
  if (h == hipSuccess) h = hipStreamSynchronize(e->stream);
  if (h != hipSuccess) rc = fail(RAFT_EHIP, "raft_state_digest: %s", hipGetErrorString(h));
  (void)hipFree(d_pg);
  if (rc == RAFT_OK && total) *total = tot;
  return rc;
}

int raft_nodelog(raft_engine* e, uint64_t group, char* buf, size_t cap) {
  if (!e || (!buf && cap)) return fail(RAFT_EINVAL, "null argument");
  if (group >= e->cfg.groups) return fail(RAFT_EINVAL, "group %llu out of range", (unsigned long long)group);
  if (int rc = settle_check(e)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  static const char* names[] = {"follower", "candidate", "leader", "?"};   // State (main.go:51-57)
  std::string out;
  uint16_t meta = 0;
  SsRec ss{};
  LxRec lx{};
  HIPCHK(hipMemcpyAsync(&meta, e->P.gmeta + group, 2, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&ss, e->P.gss + group, sizeof ss, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&lx, e->P.glx + group, sizeof lx, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  const int pr = meta & 0xF;
  const bool ssync = (meta & M_SSYNC) && pr < int(e->cfg.replicas);   // compressed state
  for (uint32_t r = 0; r < e->cfg.replicas; ++r) {
    const uint64_t d = group * recw_of(e->cfg.replicas) + r;   // group record (rix)
    int32_t term = 0, commit = 0, last = 0, rs = 0;
    HIPCHK(hipMemcpyAsync(&term, e->P.term + d, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&commit, e->P.commit + d, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&last, e->P.last + d, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(&rs, e->P.rs + d, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (ssync) {
      term = ss_term(ss, int(r), meta, lx);
      last = ss_last(ss, int(r), pr, meta, lx);
      commit = ss_commit(ss, int(r), pr, meta, lx, commit);
    }
    char line[128];
    snprintf(line, sizeof line, "[Server%u:%d:%d:%d][%s]\n", r, term, commit, last, names[rs & 3]);
    out += line;
  }
  if (out.size() + 1 > cap) return fail(RAFT_ERANGE, "nodelog needs %zu bytes", out.size() + 1);
  std::memcpy(buf, out.c_str(), out.size() + 1);
  return int(out.size());
}

}  // extern "C"

namespace {

// CRC32C over a byte stream (slice-by-8, same tables as the entry stamps).
uint32_t crc32c_update(uint32_t crc, const uint8_t* p, size_t n) {
  const std::vector<uint32_t>& T = crc_tab_host();
  uint32_t c = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = T[1792 + (lo & 255)] ^ T[1536 + ((lo >> 8) & 255)] ^ T[1280 + ((lo >> 16) & 255)] ^ T[1024 + (lo >> 24)] ^
        T[768 + (hi & 255)] ^ T[512 + ((hi >> 8) & 255)] ^ T[256 + ((hi >> 16) & 255)] ^ T[hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ T[(c ^ *p++) & 255];
  return ~c;
}

constexpr char CKPT_MAGIC[8] = {'R', 'A', 'F', 'T', 'C', 'K', 'P', 'T'};
constexpr uint32_t CKPT_VERSION = 2;   // 2: + iso_victim
struct CkptHeader {
  char magic[8];
  uint32_t version, nfields;
  raft_config cfg;
};
struct CkptField {   // followed by count * elem bytes
  char name[12];
  uint32_t elem;
  uint64_t count;
};

// The canonical view's fields in file order.
struct ViewField {
  const char* name;
  void** ptr;
  uint32_t elem;
  uint64_t count;
};
std::vector<ViewField> view_fields(raft_state_view& v, uint64_t G, uint64_t R, uint64_t K) {
  return {{"role", reinterpret_cast<void**>(&v.role), 1, G * R},
          {"voted", reinterpret_cast<void**>(&v.voted), 1, G * R},
          {"term", reinterpret_cast<void**>(&v.term), 4, G * R},
          {"last", reinterpret_cast<void**>(&v.last), 4, G * R},
          {"commit", reinterpret_cast<void**>(&v.commit), 4, G * R},
          {"deadline", reinterpret_cast<void**>(&v.deadline), 4, G * R},
          {"timeout", reinterpret_cast<void**>(&v.timeout), 4, G * R},
          {"match", reinterpret_cast<void**>(&v.match), 4, G * R * R},
          {"fault", reinterpret_cast<void**>(&v.fault), 1, G},
          {"log_term", reinterpret_cast<void**>(&v.log_term), 4, G * R * K},
          {"log_value", reinterpret_cast<void**>(&v.log_value), 8, G * R * K},
          {"log_crc", reinterpret_cast<void**>(&v.log_crc), 4, G * R * K},
          {"next", reinterpret_cast<void**>(&v.next), 4, G * R * R},
          {"hwm", reinterpret_cast<void**>(&v.hwm), 4, G * R},
          {"iso_victim", reinterpret_cast<void**>(&v.iso_victim), 1, G}};
}

struct File {
  FILE* f = nullptr;
  ~File() {
    if (f) fclose(f);
  }
};

}  // namespace

extern "C" {

int raft_checkpoint_save(raft_engine* e, const char* path) {
  if (!e || !path) return fail(RAFT_EINVAL, "null argument");
  const uint64_t G = e->cfg.groups, R = e->cfg.replicas, K = e->cfg.ring_depth;
  raft_state_view v{};
  auto fields = view_fields(v, G, R, K);
  std::vector<std::vector<uint8_t>> bufs(fields.size());
  for (size_t i = 0; i < fields.size(); ++i) {
    bufs[i].assign(fields[i].count * fields[i].elem, 0);
    *fields[i].ptr = bufs[i].data();
  }
  if (int rc = raft_store_state(e, &v)) return rc;
  // written to <path>.tmp, flushed to disk, then renamed over <path>: a crash
  // mid-write leaves the previous checkpoint intact
  const std::string tmp = std::string(path) + ".tmp";
  File f;
  f.f = fopen(tmp.c_str(), "wb");
  if (!f.f) return fail(RAFT_EINVAL, "cannot open %s for writing", tmp.c_str());
  uint32_t crc = 0;
  auto put = [&](const void* p, size_t n) {
    crc = crc32c_update(crc, static_cast<const uint8_t*>(p), n);
    return fwrite(p, 1, n, f.f) == n;
  };
  CkptHeader h{};
  std::memcpy(h.magic, CKPT_MAGIC, 8);
  h.version = CKPT_VERSION;
  h.nfields = uint32_t(fields.size());
  h.cfg = e->cfg;
  bool ok = put(&h, sizeof h);
  for (size_t i = 0; ok && i < fields.size(); ++i) {
    CkptField fh{};
    std::strncpy(fh.name, fields[i].name, sizeof fh.name - 1);
    fh.elem = fields[i].elem;
    fh.count = fields[i].count;
    ok = put(&fh, sizeof fh) && put(bufs[i].data(), bufs[i].size());
  }
  ok = ok && fwrite(&crc, 1, 4, f.f) == 4;
  ok = ok && fflush(f.f) == 0 && fsync(fileno(f.f)) == 0;
  ok = fclose(f.f) == 0 && ok;
  f.f = nullptr;
  if (!ok) {
    std::remove(tmp.c_str());
    return fail(RAFT_EINVAL, "short write to %s", tmp.c_str());
  }
  if (std::rename(tmp.c_str(), path) != 0) {
    std::remove(tmp.c_str());
    return fail(RAFT_EINVAL, "cannot rename %s to %s", tmp.c_str(), path);
  }
  return RAFT_OK;
}

int raft_checkpoint_load(raft_engine* e, const char* path) {
  if (e) state_replacing(e);
  if (!e || !path) return fail(RAFT_EINVAL, "null argument");
  const uint64_t G = e->cfg.groups, R = e->cfg.replicas, K = e->cfg.ring_depth;
  File f;
  f.f = fopen(path, "rb");
  if (!f.f) return fail(RAFT_EINVAL, "cannot open %s", path);
  uint32_t crc = 0;
  auto get = [&](void* p, size_t n) {
    if (fread(p, 1, n, f.f) != n) return false;
    crc = crc32c_update(crc, static_cast<const uint8_t*>(p), n);
    return true;
  };
  CkptHeader h{};
  if (!get(&h, sizeof h) || std::memcmp(h.magic, CKPT_MAGIC, 8) != 0)
    return fail(RAFT_EINVAL, "%s: not a raftstep checkpoint", path);
  // version 1 (before leader isolation) has every field but iso_victim, the last one
  if (h.version != CKPT_VERSION && h.version != 1)
    return fail(RAFT_EINVAL, "%s: checkpoint version %u unsupported", path, h.version);
  if (h.cfg.replicas != e->cfg.replicas || h.cfg.groups != e->cfg.groups || h.cfg.ring_depth != e->cfg.ring_depth ||
      h.cfg.semantics != e->cfg.semantics || h.cfg.payload_crc != e->cfg.payload_crc)
    return fail(RAFT_EINVAL, "%s: checkpoint of R=%u G=%llu K=%u sem=%u crc=%u does not fit this engine", path,
                h.cfg.replicas, (unsigned long long)h.cfg.groups, h.cfg.ring_depth, h.cfg.semantics, h.cfg.payload_crc);
  // the trace (client values, timer draws, isolation, corruption) is keyed by
  // the seed and the GLOBAL group id: resuming on another shard or another
  // trace would silently continue on a different RNG stream
  {
    const raft_config& a = h.cfg;
    const raft_config& b = e->cfg;
    const char* bad = nullptr;
    if (a.group_base != b.group_base) bad = "group_base";
    else if (a.seed != b.seed) bad = "seed";
    else if (a.tick_seconds != b.tick_seconds) bad = "tick_seconds";
    else if (a.follower_timeout_min != b.follower_timeout_min || a.follower_timeout_span != b.follower_timeout_span)
      bad = "follower timeout range";
    else if (a.candidate_timeout_min != b.candidate_timeout_min || a.candidate_timeout_span != b.candidate_timeout_span)
      bad = "candidate timeout range";
    else if (a.client_period != b.client_period) bad = "client_period";
    else if (a.entries_per_tick != b.entries_per_tick) bad = "entries_per_tick";
    else if (a.isolate_per_65536 != b.isolate_per_65536 || a.isolate_min_ticks != b.isolate_min_ticks ||
             a.isolate_max_ticks != b.isolate_max_ticks || a.isolate_leader != b.isolate_leader)
      bad = "isolation parameters";
    else if (a.corrupt_per_65536 != b.corrupt_per_65536) bad = "corrupt_per_65536";
    if (bad) return fail(RAFT_EINVAL, "%s: checkpoint %s differs from this engine's (trace would diverge)", path, bad);
  }
  raft_state_view v{};
  auto fields = view_fields(v, G, R, K);
  if (h.version == 1) fields.pop_back();   // iso_victim: absent (loads as 0)
  if (h.nfields != fields.size()) return fail(RAFT_EINVAL, "%s: %u fields, expected %zu", path, h.nfields, fields.size());
  std::vector<std::vector<uint8_t>> bufs(fields.size());
  for (size_t i = 0; i < fields.size(); ++i) {
    CkptField fh{};
    if (!get(&fh, sizeof fh)) return fail(RAFT_EINVAL, "%s: truncated", path);
    if (std::strncmp(fh.name, fields[i].name, sizeof fh.name) != 0 || fh.elem != fields[i].elem ||
        fh.count != fields[i].count)
      return fail(RAFT_EINVAL, "%s: field %zu is %.12s[%llu x %u], expected %s", path, i, fh.name,
                  (unsigned long long)fh.count, fh.elem, fields[i].name);
    bufs[i].resize(fh.count * fh.elem);
    if (!get(bufs[i].data(), bufs[i].size())) return fail(RAFT_EINVAL, "%s: truncated", path);
    *fields[i].ptr = bufs[i].data();
  }
  const uint32_t want = crc;
  uint32_t stored = 0;
  if (fread(&stored, 1, 4, f.f) != 4) return fail(RAFT_EINVAL, "%s: missing CRC32C trailer", path);
  if (stored != want) return fail(RAFT_EINVAL, "%s: CRC32C mismatch (file %08x, computed %08x)", path, stored, want);
  return raft_load_state(e, &v);
}

}  // extern "C"
