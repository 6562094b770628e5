// kernels.h — host-side launchers and device argument records of the engine.
//
//  tick_fast_kernel<R,CRC,SEM> (k_fast.hip): steady-state tick, one lane
//        per group, HBM-bound (~233 B per group-step at R=5, E=1); groups it
//        cannot take go to a worklist.
//  tick_slow_kernel<R,SEM> (k_ref.hip / k_raft.hip): the general tick
//        (elections, step-downs, faults, EXT drops) over the worklist.
//  ops_kernel<R,SEM>: the message-level handler API (AppendEntries /
//        RequestVote receivers, node steps) over distinct groups.
//  init_*_kernel<R> (k_init.hip): NewNode state / post-election state.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "raft_device.hpp"

namespace raftstep {

enum : uint32_t {
  OP_CLIENT_APPEND = 1, OP_LEADER_ROUND = 2, OP_CANDIDATE_ROUND = 3, OP_TIMEOUT = 4,
  OP_LEADER_COMMIT = 5, OP_AE = 100, OP_VR = 101
};

// One handler-batch element after host-side range checks (int64 -> int32).
struct DevOp {
  uint64_t group;
  uint32_t replica;   // receiving / acting replica
  uint32_t kind;
  int64_t arg;        // CLIENT_APPEND value
  int32_t term, prev_idx, prev_term, lc;  // AE / VR request fields
  uint32_t n;         // AE: len(Logs)
  uint32_t skip;      // AE: values/stamps of Logs[0..skip) are not staged (only the last K can land in the ring)
  uint64_t off;       // AE: offset of Logs[0] in the term array
  uint64_t voff;      // AE: offset of Logs[skip] in the value / stamp arrays
};
struct DevRes {
  int32_t status, fault, ok, term;
  int64_t value;      // AE: MatchIndex; VR: granted; ops: see raft_op_result
};

// Steady-state fast kernel; groups it does not take are DEFERred to `work`.
// ev_start/ev_stop (may be null) time the dispatch itself (hipExtLaunchKernel).
hipError_t launch_tick_fast(int R, int sem, const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                            int32_t* work_tick, uint32_t* work_count, int force_slow, hipStream_t s,
                            hipEvent_t ev_start, hipEvent_t ev_stop);
// Two-pass tick: tick_lean_kernel takes the compressed steady groups and
// appends every other live group to `list` (counter `count`), then
// tick_list_kernel runs the full fast_group over that list and zeroes
// `next_count`. Events (may be null) time each dispatch.
hipError_t launch_tick_two_pass(int R, int sem, const DevPlanes& P, const Trace& T, unsigned long long* stats,
                                uint32_t* work, int32_t* work_tick, uint32_t* work_count, uint32_t* list,
                                uint32_t* count, uint32_t* next_count, hipStream_t s, hipEvent_t lean_start,
                                hipEvent_t lean_stop, hipEvent_t list_start, hipEvent_t list_stop, bool skip_list);
// The two passes launched separately (the pipelined tick, engine.cpp):
// lflags bit 0 = leave the groups marked in P.glst alone (and clear the
// marks), bit 1 = mark the groups passed on. With `next` the list kernel
// runs its groups through the following tick too (a second fast_group step
// on the staged state; its stats and deferrals go to next's record and
// worklist), so that the next lean kernel can run beside it.
struct ListNext {
  unsigned long long* stats;    // the following tick's stats slots
  uint32_t* work;               // the worklist of the following tick's window
  int32_t* work_tick;
  uint32_t* work_count;
};
// Fused steady ticks (steady-state list skip): nticks ticks of every
// compressed steady group in one launch; stats of tick j at stats + j slots.
hipError_t launch_tick_fused(int R, int sem, const DevPlanes& P, const Trace& T, int nticks, unsigned long long* stats,
                             uint32_t* list, uint32_t* count, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop);
// (g0, ng: the launch covers groups [g0, g0 + ng) only; g0 a multiple of 256;
// zero_count: list counters the launch zeroes, block 0, before anything else)
hipError_t launch_tick_lean(int R, int sem, const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* list,
                            uint32_t* count, int lflags, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop,
                            uint64_t g0 = 0, uint64_t ng = ~0ull, uint32_t* zero_count = nullptr);

hipError_t launch_tick_list(int R, int sem, const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                            int32_t* work_tick, uint32_t* work_count, uint32_t* list, uint32_t* count,
                            uint32_t* next_count, const ListNext* next, hipStream_t s, hipEvent_t ev_start,
                            hipEvent_t ev_stop);
// General kernel: catches every worklisted group up to last_tick; zeroes
// `next_count`. lane_per_group: the one-lane-per-group form (tick_slow_kernel)
// instead of the replica-parallel one (tick_seg_kernel).
hipError_t launch_tick_slow(int R, int sem, const DevPlanes& P, const Trace& T0, int64_t first_tick, int64_t win_first, int64_t last_tick,
                            unsigned long long* stats, const uint32_t* work, const int32_t* work_tick,
                            const uint32_t* work_count, uint32_t* next_count, int lane_per_group, hipStream_t s);
hipError_t launch_ops(int R, int sem, const DevPlanes& P, const Trace& T, const DevOp* ops, uint32_t n,
                      const int32_t* et, const int64_t* ev, const uint32_t* ec, DevRes* out, hipStream_t s);
hipError_t launch_init_new(int R, const DevPlanes& P, const Trace& T, hipStream_t s);
// Per-group state digest (same definition as oracle_state_digest) + wrapping sum.
hipError_t launch_digest(int R, const DevPlanes& P, int raft, uint64_t* per_group, unsigned long long* total,
                         hipStream_t s);
// End-of-call check record (one more block of the stats reduce launch):
// out[CHK_LISTED] = groups on the two-pass list counters (both parities),
// out[CHK_DEFERRED] = groups the last general window's worklist held,
// out[CHK_LAST_LIST] = groups on list llast alone (what the lean kernel passed
// on at the call's last tick; the engine's pipeline choice, RAFTSTEP_PIPELINE=2),
// out[CHK_MAGIC] = a constant proving the record was written this call.
// zero_lists: zero both list counters afterwards (a list-skipping call).
enum : int { CHK_LISTED = 0, CHK_DEFERRED = 1, CHK_LAST_LIST = 2, CHK_MAGIC = 7 };
struct CallCheck {
  uint32_t* wcount;             // the engine's counter block (raft_device.hpp WCOUNT_WORDS)
  int wlast;                    // parity of the worklist the last window tail took
  int zero_lists;
  unsigned long long* out;      // NSTAT words
  int llast;                    // list set of the call's last tick
  // host mirror (a call whose records are all reduced by this one launch, no
  // communicator): every block also writes its record to hout (pinned,
  // coherent host memory, same layout as `out` of the launch), and the last
  // block to finish stores `seq` to *hdone (system scope), so that the host
  // reads the call's records without a device-to-host copy and sees the end
  // of the call without waiting for the stream's completion signal
  unsigned long long* hout;
  uint32_t* hdone;
  unsigned int* ctr;            // device counter of finished blocks (zero between launches)
  uint32_t seq;
};
// Sums the STAT_SLOTS slots of nticks consecutive per-tick records of `hist`
// into out[nticks][NSTAT] and zeroes those slots; with `chk` also writes the
// check record (nticks may then be 0).
// Clears DEFER of the groups on worklist `parity` (work), records their
// number and zeroes that worklist's counters (k_init.hip window_tail_kernel).
hipError_t launch_window_tail(const DevPlanes& P, const uint32_t* work, uint32_t* wcount, int parity, hipStream_t s);
// The base the lean / fused kernels' exception statistics are relative to
// (tick_common.hpp lean_stats): every tick of a two-pass call, G live groups
// each taking a normal tick.
struct LeanBase {
  uint64_t G;          // groups (0: no lean kernel ran, no base)
  int64_t t0;          // tick of the reduce's first record
  uint32_t E, period;  // client entries per client tick, ticks per client tick
  uint32_t R, raft;
};
hipError_t launch_stats_reduce(unsigned long long* hist, unsigned long long* out, uint32_t nticks, const LeanBase& lb,
                               hipStream_t s, const CallCheck* chk = nullptr);
hipError_t launch_init_steady(int R, const DevPlanes& P, const Trace& T, int32_t leader, hipStream_t s);
hipError_t launch_vx_flush(int R, const DevPlanes& P, uint64_t Qb, uint32_t E, uint32_t period, uint64_t seed,
                           hipStream_t s);
// SH (raft_device.hpp ROT_SH): every group's shared entries into its replica rings
hipError_t launch_sh_flush(int R, const DevPlanes& P, hipStream_t s);
hipError_t launch_stream_probe(int R, const uint16_t* a, SsRec* b, const uint16_t* c, int32_t* d, int32_t* rt,
                               int64_t* rv, uint32_t n, uint32_t slot, uint32_t kslots, hipStream_t s,
                               uint32_t mode = 0);

}  // namespace raftstep
