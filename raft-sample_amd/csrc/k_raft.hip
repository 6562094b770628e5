// k_raft.hip — general tick + handler kernels, EXT RAFT-paper semantics.
#include "k_slow.inc"

namespace raftstep {

hipError_t launch_tick_slow_raft(int R, const DevPlanes& P, const Trace& T0, int64_t first_tick, int64_t win_first, int64_t last_tick,
                                unsigned long long* stats, const uint32_t* work, const int32_t* work_tick,
                                const uint32_t* work_count, uint32_t* next_count, int lane_per_group, hipStream_t s) {
  return launch_tick_slow_sem<SEM_RAFT>(R, P, T0, first_tick, win_first, last_tick, stats, work, work_tick, work_count, next_count,
                                         lane_per_group, s);
}
hipError_t launch_ops_raft(int R, const DevPlanes& P, const Trace& T, const DevOp* ops, uint32_t n, const int32_t* et,
                          const int64_t* ev, const uint32_t* ec, DevRes* out, hipStream_t s) {
  return launch_ops_sem<SEM_RAFT>(R, P, T, ops, n, et, ev, ec, out, s);
}

}  // namespace raftstep
