// raft_device.hpp — CDNA4 device code of the batched Raft step engine.
//
// One lane owns one Raft group for the duration of a launch. The group's R
// replicas are loaded from struct-of-arrays planes ([Gp][R]: a wave's 64
// groups read one contiguous 64*R*4-B span per plane) into registers, every message between
// replicas is a register hand-off inside the lane, and only changed fields
// are stored back. Handler semantics follow main.go (eastwd/raft-sample)
// exactly; each function cites the lines it implements. The CPU oracle in
// oracle/ restates the same lines independently and the parity tests diff
// the two.
//
// Register discipline: arrays indexed by a compile-time replica id stay in
// VGPRs; arrays indexed by a runtime replica id go through sel()/put()
// (v_cndmask chains) so nothing spills to scratch. Per-replica roles and
// flags are bit-packed into one 32-bit register.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace raftstep {

enum : int { ROLE_F = 0, ROLE_C = 1, ROLE_L = 2 };
enum : int { SEM_REF = 0, SEM_RAFT = 1 };
enum : int {
  F_NONE = 0, F_PANIC_GETLOG = 1, F_DEADLOCK_VRES = 2, F_DEADLOCK_LEADER_VREQ = 3,
  F_RING_EVICTED = 4, F_OVERFLOW = 5
};
enum : uint32_t { ST_VALUE = 1, ST_TIMER_F = 2, ST_TIMER_C = 3, ST_ISOLATE = 4, ST_CORRUPT = 5 };
enum : int {
  S_COMMITTED = 0, S_WON = 1, S_BUMPS = 2, S_AE_OK = 3, S_AE_FAIL = 4, S_VOTES = 5,
  S_FAULTS = 6, S_LEADER_GROUPS = 7, NSTAT = 8
};
constexpr int NO_PRIMARY = 0xF;
// gmeta flag bits (above primary:4 | fault:3; fault codes are 0..5)
// VX (RAFT, with LXS, ONESTALE or SXS; round 5): the group's one cut-off
// leader xr — the LXS primary, or the ONESTALE / SXS stale leader — holds a
// VIRTUAL suffix: its entries xlo+1 .. last[xr] are not in its ring column
// but are its own client appends, one batch per client tick up to the last
// client tick before the tick being run (a leader appends at every client
// tick, main.go:327-329, a cut-off one too), so entry xlo+j is regenerated
// from the trace RNG (vx_entry). xlo is the followers' LastApplied (LXS: the
// gss record) or the primary's NextIndex for xr minus one (ONESTALE / SXS).
// Its column there holds the primary's entries instead (every write of the
// primary's entries includes it), so the stale leader's return — truncation
// at xlo and the primary's entries appended — needs no ring copy. Only the
// fast paths that keep both properties take a VX group (k_fast.hip); every
// other reader first writes the suffix into the column and drops the flag
// (vx_materialize: the general kernel at load, the engine before host reads
// and handler batches).
constexpr int M_VX = 1 << 7;
constexpr int M_DEFER = 1 << 8;   // on the worklist with ticks pending; the fast kernel leaves it alone
constexpr int M_MSYNC = 1 << 9;   // primary's MatchIndex[p] == LastApplied[p] for every peer; lmatch is stale
constexpr int M_STEADY = 1 << 10; // exactly one leader (the primary), every other replica a follower
constexpr int M_ONECAND = 1 << 11; // as STEADY, except that exactly one other replica is a candidate
constexpr int M_ONESTALE = 1 << 12; // as STEADY, except that exactly one other replica is a leader of a lower term
// SSYNC (with STEADY and MSYNC): every replica holds the same log length and
// term, every last entry is of that term, the followers share one
// CommitIndex. The group's term / last / commit / lterm planes are then stale
// and the 16-B record gss[g] = {LastApplied, Term, leader's CommitIndex,
// followers' CommitIndex} is the state (the steady-state kernel reads and
// writes only it); every other reader materialises the planes from it.
constexpr int M_SSYNC = 1 << 13;
// HWX (RAFT, with MSYNC): some replica's log was truncated below its
// high-water mark, which the hwm plane holds. Under MSYNC every replica's
// high-water mark is max(hwm plane, LastApplied) (the plane is exact when
// MSYNC is entered and no log is truncated while it holds); without HWX the
// plane is at most LastApplied everywhere, so readers that only need the
// steady case (the lean kernel) skip the plane.
constexpr int M_HWX = 1 << 14;
// LXS (RAFT, with SSYNC, MSYNC and STEADY): the primary leader is cut off
// (leader isolation) and appends alone; the gss record holds the followers
// (and the shared term / commit fields), the leader's log is k entries longer,
// glx[g] = {k, D} with D the earliest follower election deadline (no
// follower timer moves while the leader is cut off).
constexpr int M_LXS = 1 << 15;
// SXS (RAFT; SSYNC + ONESTALE + MSYNC, never LXS): the primary (a new leader)
// replicates to its followers while the group's one stale leader xs (the
// previous leader, term T-1, cut off) appends alone. The gss record holds the
// primary and its followers; glx[g] = {k, xs}: xs's log is k entries longer
// than theirs, its term and last-entry term are T-1, and its CommitIndex, its
// high-water mark and the primary's MatchIndex / NextIndex for it stay
// explicit in the record planes (none of them moves while it is cut off).
struct __attribute__((aligned(8))) LxRec { int32_t k, dl; };
struct __attribute__((aligned(16))) SsRec { int32_t last, term, cl, cf; };
__device__ __host__ __forceinline__ bool is_sxs(int meta) {
  return (meta & (M_SSYNC | M_ONESTALE)) == (M_SSYNC | M_ONESTALE);
}
// the compressed form keeps something in glx (LXS or SXS)
__device__ __host__ __forceinline__ bool uses_glx(int meta) { return (meta & M_LXS) || is_sxs(meta); }
// LastApplied of replica r of an SSYNC group (LXS: the primary is k ahead; SXS: the stale leader)
__device__ __host__ __forceinline__ int32_t ss_last(const SsRec& s, int r, int primary, int meta, const LxRec& x) {
  return s.last + ((((meta & M_LXS) && r == primary) || (is_sxs(meta) && r == x.dl)) ? x.k : 0);
}
// Term (= term of the last entry) of replica r of an SSYNC group
__device__ __host__ __forceinline__ int32_t ss_term(const SsRec& s, int r, int meta, const LxRec& x) {
  return s.term - ((is_sxs(meta) && r == x.dl) ? 1 : 0);
}
// CommitIndex of replica r of an SSYNC group; `plane`: the commit plane's value (SXS's stale leader)
__device__ __host__ __forceinline__ int32_t ss_commit(const SsRec& s, int r, int primary, int meta, const LxRec& x,
                                                      int32_t plane) {
  return r == primary ? s.cl : ((is_sxs(meta) && r == x.dl) ? plane : s.cf);
}
// MSYNC: the primary's MatchIndex (NextIndex) for peer p is implicit = LastApplied (+1),
// except for SXS's stale leader, whose row stays explicit
__device__ __host__ __forceinline__ bool msync_peer(int meta, const LxRec& x, int p) {
  return (meta & M_MSYNC) && !(is_sxs(meta) && p == x.dl);
}
constexpr int HB_NONE = -2147483647 - 1;
constexpr int I32MAX = 2147483647;
constexpr int STAT_SLOTS = 64;   // per-tick stats are spread over 64 slots to cut atomic contention
// Per tick the statistics area holds the STAT_SLOTS x NSTAT counters, then
// STAT_PKS 64-B slots of the lean / fused kernels' exception sums (lean_stats
// in tick_common.hpp; the reduce kernel adds them to the base it computes).
constexpr int STAT_PKS = 256;
constexpr int STAT_PK = STAT_SLOTS * NSTAT;                  // offset of the exception slots in a tick's area
constexpr int STAT_TICK = STAT_SLOTS * NSTAT + STAT_PKS * 8;   // words per tick

// Device layout. Per-replica scalar planes are [Gp][R] (rix below); the
// log rings are wave tiles [Gp/64][KP][64][R] (see ring_tile below).
// The cold per-group words — the rotations and boundary of the older ring
// segments and the leader-isolation victims — packed into one 16-B record per
// group (round 5): every reader that needs one of them (the list kernel's
// staging, the general kernel, the digest) needs them all, and a scattered
// group then costs one line for the four instead of four. The lean kernel's
// per-group words (gmeta, gss, grot, gsb, hb, glx) stay separate planes.
struct __attribute__((aligned(16))) GSeg {
  uint16_t rota, rotb;   // rotation of the previous / older segment
  int32_t sb2;           // first index of the previous segment (0: none older)
  uint8_t iso_unused;    // (round 5's leader-isolation victims; now the dense DevPlanes::giso plane)
  uint8_t pad[3];
  int32_t shf;           // SH (ROT_SH): the first index whose entries live in the shared ring
};
// A plane of T with a byte stride S (a field of an array of records): the
// accessors index it like a plain plane (at(), operator[]).
template <typename T, uint32_t S>
struct Strided {
  T* p;
  __host__ __device__ __forceinline__ T& operator[](uint32_t i) const {
    return *reinterpret_cast<T*>(reinterpret_cast<char*>(p) + size_t(i) * S);
  }
};

struct DevPlanes {
  int32_t* term;       // Node.Term                 (main.go:19)
  int32_t* last;       // Node.LastApplied=len(Log) (main.go:25)
  int32_t* commit;     // Node.CommitIndex          (main.go:24)
  int32_t* tstart;     // election timer start (virtual s); deadline = start + d
  int32_t* hb;         // [Gp] time of the last steady-state heartbeat that reset every follower
  int32_t* rs;         // role:2 | vote:4 | timer duration d:10 (main.go:16, 20, 114, 194);
                       // vote = Voted (REF) or votedFor+1 (RAFT, 0 = none)
  int32_t* lmatch;     // [Gp][R] MatchIndex row of the group's primary leader (main.go:29)
  int32_t* xmatch;     // [R][R][Gp] rows of any further concurrent leaders (EXT only)
  int32_t* lnext;      // RAFT mode: [Gp][R] NextIndex row of the primary leader (REF derives match+1)
  int32_t* xnext;      // RAFT mode: [R][R][Gp] NextIndex rows of further leaders
  int32_t* hwm;        // RAFT mode: [Gp][R] highest LastApplied ever (== last in REF)
  uint16_t* gmeta;     // primary leader id:4 | fault:4 | DEFER | MSYNC | STEADY
  GSeg* gseg;          // [Gp] the packed cold words (GSeg); giso / grota / grotb / gsb2 are views of its fields
  // EXT leader-isolation victims, nibble per epoch parity: 8 | replica (0 =
  // none). Round 6: a dense [Gp] byte plane (it was GSeg::iso): the lean
  // kernel reads it for every lane with a window active, and a strided
  // 1-of-16-B read cost each such lane a whole sector (C4's lean kernel
  // fetched 1.27x its algorithmic bytes)
  Strided<uint8_t, 1> giso;
  SsRec* gss;          // [Gp] the compressed state of an SSYNC group
  LxRec* glx;          // [Gp] LXS: the cut-off leader's extra entries and the earliest follower deadline
  uint16_t* grot;      // ring rotation of the current segment: entry idx >= gsb sits at slot (idx-1+grot) mod KP
  Strided<uint16_t, 16> grota;  // rotation of the previous segment (entries idx < gsb)
  int32_t* gsb;        // first index of the current segment (0: one segment)
  Strided<uint16_t, 16> grotb;  // rotation of the segment before the previous one (entries idx < gsb2)
  Strided<int32_t, 16> gsb2;    // first index of the previous segment (0: none older)
  int32_t* lterm;      // [Gp][R] Log[len-1].Term: cached term of each replica's last entry
  int32_t* log_term;   // Log.Term  ring, tiles [Gp/64][KP][64][R] (ring_tile / ring_in_tile)
  int64_t* log_value;  // Log.Value ring
  uint32_t* log_crc;   // EXT: CRC32C stamp ring (payload_crc only)
  // SH (ROT_SH): one shared copy of the entries every replica of an SSYNC
  // group holds alike, tiles [Gp/64][KP][64] (sh_tile / sh_in_tile), the
  // same slots as the replica rings; null when P.sh is off
  int32_t* sh_term;
  int64_t* sh_value;
  uint32_t* sh_crc;
  Strided<int32_t, 16> gshf;    // GSeg::shf
  const uint32_t* crc_tab;  // 8 x 256 slice-by-8 CRC32C tables
  uint32_t crc_on;     // payload_crc
  uint32_t corrupt_p;  // EXT corruption probability / 65536
  uint64_t Gp;         // plane pitch (groups, padded)
  uint64_t G;          // groups on this engine
  uint64_t gbase;      // global id of local group 0
  uint32_t K;          // ring depth (power of two): the last K entries of every log stay readable
  uint32_t KP;         // physical ring slots per replica: K, or 2K when segment switches are on
  uint32_t kmask;      // KP - 1 (physical slot mask)
  unsigned long long* dbg;  // diagnostics (raft_diag_enable): lane class counters [0,32) lean kernel,
                            // [32,64) fast_group (list / one-pass kernels), else null
  uint32_t dbg_pass;   // test knob (raft_debug_force_pass): the lean kernel passes this group to the list (~0u: none)
  int32_t* rec;        // [Gp][NPL][R] group records holding every per-replica row above (see rix)
  uint32_t scap;       // capacity of one shard of a sharded group list (see below)
  uint32_t shard_sb;   // log2 of the consecutive 256-group blocks per shard chunk (shard_home)
  uint8_t* glst;       // [Gp] two-step list marks: 1 = passed by the last lean kernel to a list kernel that
                       // also runs this tick for it (the lean kernel leaves the group alone and clears the mark)
  // the lean kernel's record / heartbeat stores are non-temporal when the
  // per-group words cannot stay in the 256 MiB Infinity Cache between ticks
  // anyway (engine.cpp: 40 B x Gp above it; round 5, C2 at 2^24: +2%);
  // below that, plain stores keep them resident (C2 at 2^20: nt 3% slower)
  uint32_t rec_nt;
  // VX (see M_VX) enabled: RAFT, leader isolation, no payload CRC
  // (RAFTSTEP_VX=0 turns it off); the fast paths then give a group entering
  // LXS a virtual suffix
  uint32_t vx;
  // SH (ROT_SH) enabled: steady groups' entries go to the shared ring (no
  // EXT isolation configured, KP < 2^15; RAFTSTEP_SH=0 turns it off)
  uint32_t sh;
  // SH kept through rejections (round 6; REF with payload CRC and EXT
  // corruption, KP = 2K): a follower that rejects a corrupted copy keeps a
  // log that is a prefix of the leader's, and the shared ring's 2K slots still
  // hold its whole window while it lags by less than K, so the list kernel
  // runs the rejection and the catch-up on the shared form without copying
  // it back (k_fast.hip fast_group, `shf`)
  uint32_t sh_keep;
  uint32_t sh_cs;      // log2 of the shared ring's slot chunk (sh_in_tile)
  // list kernel: each block orders its staged groups by their form bits
  // before the tick (round 6), so that a wave's lanes run fewer distinct paths
  // of fast_group (RAFTSTEP_LIST_SORT=0 turns it off)
  uint32_t list_sort;
  // SH: a group in shared form is taken by the lean (or fused) kernel every
  // tick, so its heartbeat time (hb, every follower's timer reset) is implied:
  // now of the last tick run. Its hb store is skipped; whoever copies the
  // group back writes it (the list kernel: now of the tick before its own;
  // the engine's flush and the digest: sh_hb, now of the last call's last tick)
  int32_t sh_hb;
  // RAFT_CLIENT_STAGED: the caller's client values (raft_stage_values),
  // [ticks][E][G] int64 from tick cv_t0 on; null: the trace RNG (cv_base)
  const int64_t* cv;
  int64_t cv_t0;
  uint64_t cv_stride;   // G: between a group's entries e and e+1 of one tick
  uint64_t cv_tstride;  // E * G: between two ticks
  uint32_t diag;       // timing-only diagnostics (RAFTSTEP_DIAG_LEAN; results are wrong when set): 1 = drifted
                       // lanes of the lean kernel skip their ring writes, 2 = they write the wave's common row
                       // (list kernel: 32 = staging alone, 64 = no tick, 128 = no ring writes / copies)
};

// Sharded group lists (the general kernel's worklist, the two-pass tick's
// list). A returning device-scope atomicAdd on one word saturates at ~88 per
// us (MI355X_MICROARCH.md, work queues), so one counter bumped once by each
// of the ~16K blocks of a 4M-group launch costs ~190 us. A list is instead
// NSHARD sub-lists, one counter each (64 B apart): group g belongs to shard
// (g >> 8) & (NSHARD-1), the shard of its block in the dense launches, so a
// dense block appends with one atomic on its own shard and every shard holds
// at most scap = ceil(blocks / NSHARD) * 256 entries (each group is listed at
// most once per list). Consumers take the block-level prefix over the NSHARD
// counts and map a dense index to (shard, slot).
constexpr int NSHARD = 64;
constexpr int SHARD_STRIDE = 16;   // u32 words between two shard counters
constexpr int SHARD_WORDS = NSHARD * SHARD_STRIDE;
// engine counter block (u32 words): worklist counters [NWORK windows][SHARD_WORDS],
// two-pass list counters [NLISTS ticks][SHARD_WORDS], then the window tail's
// words: the total each worklist's last tail took (WC_TAKEN + index) and its
// blocks-done counter (WC_DONE)
constexpr int NWORK = 3;
constexpr int NLISTS = 3;
constexpr int WC_TAKEN = (NWORK + NLISTS) * SHARD_WORDS;
constexpr int WC_DONE = WC_TAKEN + 8;
constexpr int WCOUNT_WORDS = WC_TAKEN + SHARD_STRIDE;
// (round 6: 2^sb consecutive blocks share a shard — DevPlanes::shard_sb — so
// that a shard's entries, appended roughly in dispatch order, are groups of
// a few neighbouring blocks: the list kernel's wave then works on groups
// whose records, ring tiles and per-group words are near each other)
__device__ __forceinline__ uint32_t shard_of_block(uint32_t b, uint32_t sb) { return (b >> sb) & uint32_t(NSHARD - 1); }
__device__ __forceinline__ uint32_t shard_home(uint32_t g, uint32_t sb) { return shard_of_block(g >> 8, sb); }
// pre[0..NSHARD] (LDS) = exclusive prefix of the shard counts; returns the total.
// Block-wide: every thread calls it.
__device__ __forceinline__ uint32_t shard_prefix(const uint32_t* cnt, uint32_t* pre) {
  if (threadIdx.x < 64) {
    const uint32_t v = threadIdx.x < uint32_t(NSHARD) ? cnt[threadIdx.x * SHARD_STRIDE] : 0u;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (int(threadIdx.x) >= o) x += y;
    }
    if (threadIdx.x < uint32_t(NSHARD)) pre[threadIdx.x + 1] = x;
    if (threadIdx.x == 0) pre[0] = 0;
  }
  __syncthreads();
  return pre[NSHARD];
}
// element index of dense position i < total
__device__ __forceinline__ uint32_t shard_locate(const uint32_t* pre, uint32_t scap, uint32_t i) {
  uint32_t k = 0;
#pragma unroll
  for (uint32_t step = NSHARD / 2; step > 0; step >>= 1)
    if (pre[k + step] <= i) k += step;
  return k * scap + (i - pre[k]);
}

// Two-pass list entry: the list of cap = NSHARD * scap slots holds the group
// ids, then, per slot, the words the lean kernel already read for that group
// (gmeta | grot << 16, the segment boundary gsb, the 16-B record gss): the
// list kernel stages them with loads coalesced by list slot instead of three
// or four scattered lines per group (round 5).
constexpr uint32_t LIST_WORDS = 8;   // [cap] ids, [cap] meta|rot, [cap] gsb, [cap] pad, [cap] SsRec (4 words)
__device__ __forceinline__ uint32_t* list_mr(uint32_t* list, uint64_t cap) { return list + cap; }
__device__ __forceinline__ int32_t* list_sb(uint32_t* list, uint64_t cap) { return reinterpret_cast<int32_t*>(list + 2 * cap); }
__device__ __forceinline__ SsRec* list_ss(uint32_t* list, uint64_t cap) { return reinterpret_cast<SsRec*>(list + 4 * cap); }
__device__ __forceinline__ void shard_zero(uint32_t* cnt) {   // block 0, threads 0..NSHARD-1 (cnt null: nothing)
  if (cnt && blockIdx.x == 0 && threadIdx.x < uint32_t(NSHARD)) cnt[threadIdx.x * SHARD_STRIDE] = 0;
}

// Ring phase segments. A group whose logs stop growing for L ticks (no
// leader under churn) comes back out of phase with the global slot
// entries_before(t) mod KP that every steady wave writes, and would write
// partial ring lines from then on. With KP = 2K its rotation can instead be
// switched without moving a single entry: entries idx >= gsb use the new
// rotation, entries in [gsb2, gsb) the previous one (grota), older ones the
// one before (grotb). A switch shifts the three (grotb = grota, gsb2 = gsb,
// grota = grot, gsb = first new index) and is safe when no log holds an
// entry at or above the new gsb yet, the oldest segment (idx < gsb2) holds
// no readable entry (the last K of any log), and the live entries still fit
// KP = 2K slots: in unwrapped slot positions they span K-1 plus the jumps
// between live segments, so the new jump d plus the previous one (when the
// previous segment is still live) must be at most K (ring_switch_ok).
__device__ __forceinline__ uint32_t ring_slot(int idx, uint32_t rot, uint32_t rota, uint32_t rotb, int sb, int sb2,
                                              uint32_t kmask) {
  return uint32_t(idx - 1 + int(idx >= sb ? rot : (idx >= sb2 ? rota : rotb))) & kmask;
}
// lo: the shortest log (before this tick); d: the jump to the global phase
__device__ __forceinline__ bool ring_switch_ok(uint32_t d, uint32_t rot, uint32_t rota, int sb, int sb2, int lo,
                                               uint32_t K, uint32_t kmask) {
  const int first = lo - int(K) + 1;   // oldest readable index of any log
  if (d == 0u || d > K || !(sb2 <= 1 || sb2 <= first)) return false;
  if (sb <= 1 || sb <= first) return true;                    // the previous segment is dead too
  return ((rot - rota) & kmask) + d <= K;                      // it stays live: both jumps inside the window
}

// Ring layout: the log rings of all R replicas are tiled by waves of 64
// groups, [Gp/64][KP][64][R] (replica innermost): entry slot s of replica r
// of group g sits at element ((g/64)*K + s)*64*R + (g%64)*R + r.
// * steady groups (logs in step, the same slot across a wave) write one
//   contiguous 64*R*4-B term row / 64*R*8-B value row per wave and entry;
// * groups whose log lengths drifted apart (churn) still write the R copies
//   of an entry next to each other (R*4 + R*8 contiguous bytes per lane
//   instead of 2R separate lines), and a wave stays inside one KP*64*R tile.
// The tile base is 64-bit (wave-uniform in the fast kernel), the offset
// inside a tile 32-bit (KP*64*R <= 2^22).
__device__ __forceinline__ uint64_t ring_tile(uint32_t g, uint32_t K, uint32_t R) {
  return uint64_t(g >> 6) * (K * 64u * R);
}
__device__ __forceinline__ uint32_t ring_in_tile(uint32_t g, uint32_t R, uint32_t slot, uint32_t r) {
  return (slot * 64u + (g & 63u)) * R + r;
}

// SH — shared entries of a group in step (round 5). While an SSYNC group is
// taken by the lean kernel's normal class every tick, all R logs receive the
// same entries (the leader's client append and the AppendEntries every
// follower accepts, main.go:121-156, 327-372), so the lean kernel stores one
// copy of each in the shared ring (12 B per entry instead of 12·R, +4 / +4·R
// with CRC32C) and marks the group: bit 15 of grot (ROT_SH; slot arithmetic
// masks rotations with kmask < 2^15, so the bit never moves a slot) and, on
// entry, GSeg::shf = the first shared index. Entries idx >= shf of every log
// then live in the shared ring at the replica rings' slot, and the replica
// rings' slots there are stale. Every other reader or writer of the group's
// rings first copies the live shared entries back into the R columns and
// clears the bit (sh_materialize: the list, one-pass and general kernels when
// they load a group; the engine's flush before host reads, digests and
// handler batches). Nothing is regenerated: a flush at any time is exact.
constexpr uint32_t ROT_SH = 0x8000u;
__device__ __forceinline__ uint64_t sh_tile(uint32_t g, uint32_t KP) { return uint64_t(g >> 6) * (KP * 64u); }
// Inside a tile (64 groups x KP slots) the slots go in chunks of 2^cs
// (DevPlanes::sh_cs): chunk-major, then group, then the slot in the chunk.
// cs = 0 (the default): one row of 64 groups per slot, which a wave of 64
// consecutive groups writes whole. cs = 4 (round 6: REF with corrupted copies
// and batches of >= 16 entries, C5V): one group's 16 consecutive slots are
// contiguous, so the list kernel's write of a rejected / catching-up group's
// batch touches a few lines per plane instead of one line per entry.
__device__ __forceinline__ uint32_t sh_in_tile(uint32_t g, uint32_t slot, uint32_t cs) {
  return ((slot >> cs) << (6u + cs)) + ((g & 63u) << cs) + (slot & ((1u << cs) - 1u));
}

// Addressing: every access is a wave-uniform base (SGPRs: the plane, or a
// ring tile) plus a 32-bit per-lane byte offset, so the compiler emits
// global_load/store with an SGPR base and ONE shared VGPR offset instead of
// a 64-bit VGPR address per (plane, replica). The byte offset idx*sizeof(T)
// must fit 32 bits: raft_engine_create rejects Gp*R*4 >= 2^32 (per-replica
// planes hold at most 4-B elements; ring offsets are taken inside a KP*64*R
// tile, < 2^26 bytes).
template <typename T>
__device__ __forceinline__ T* prow(T* plane, int r, uint64_t Gp) {   // [..][Gp] row r (xmatch / xnext)
  return plane + uint64_t(r) * Gp;
}
// Per-replica rows live in one record per group, [Gp][NPL][R] int32 padded to
// recw(R) = NPL*R rounded up to 16 B: row k of group g is R contiguous words
// at g*recw + k*R, and the plane pointers term, last, ... are rec + k*R, so
// replica r of group g of any of them is element rix(g, r) = g*recw + r. A group's whole per-replica state is then
// NPL*R*4 contiguous bytes (252 B at R=7): a scattered group (the list and
// general kernels) costs 2-3 lines instead of one line per row, and a
// block stages its groups' records into LDS with coalesced loads. A lane's
// loads of one row still share one VGPR offset with immediate offsets r*4.
// raft_engine_create keeps Gp*recw*4 < 2^32.
constexpr int NPL = 9;   // rows per record
enum : int { PL_TERM = 0, PL_LAST, PL_COMMIT, PL_TSTART, PL_LTERM, PL_RS, PL_LMATCH, PL_LNEXT, PL_HWM };
// record pitch in words: NPL*R rounded up to 16 B (records stay 16-B aligned)
__host__ __device__ constexpr uint32_t recw_of(uint32_t R) { return (uint32_t(NPL) * R + 3u) & ~3u; }
template <int R>
__host__ __device__ constexpr uint32_t recw() { return recw_of(uint32_t(R)); }
template <int R>
__device__ __forceinline__ uint32_t rix(uint32_t g, int r) {
  return g * recw<R>() + uint32_t(r);
}
template <typename T>
__device__ __forceinline__ T& at(T* base, uint32_t idx) {
  using B = std::conditional_t<std::is_const_v<T>, const char, char>;
  return *reinterpret_cast<T*>(reinterpret_cast<B*>(base) + uint32_t(idx * uint32_t(sizeof(T))));
}
template <typename T, uint32_t S>
__device__ __forceinline__ T& at(Strided<T, S> base, uint32_t idx) {   // (32-bit byte offset, as above)
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base.p) + uint32_t(idx * S));
}

struct Trace {          // per-launch trace parameters (virtual clock + RNG)
  uint64_t seed;
  int64_t tick;
  int32_t now;          // tick * tick_seconds
  int32_t f_min, f_span, c_min, c_span;
  uint32_t iso_p, iso_min, iso_span;
  uint32_t iso_m, iso_l;  // x / iso_span = udiv_magic(x, iso_m, iso_l) (host-computed, exact for every u32 x)
  uint32_t iso_leader;  // EXT: a window isolates the lowest-id leader at its first tick
  int32_t secs;         // tick_seconds
  uint32_t period, entries;  // client event every `period` ticks, `entries` each
  // global client entries before the first tick of the current run of
  // consecutive raft_tick calls (no gap, no host mutation in between):
  // entries appended from there on are regenerable from the trace RNG
  // (k_fast.hip entry jobs), older ones are not
  uint64_t contig_q;
  // this tick's client entries and the client entries before it, computed by
  // the host (make_trace) or at_tick: the 64-bit divisions by `period` they
  // need were scalar code at the start of every wave (round 6)
  uint32_t n_tick;
  uint64_t eb_tick;
  __host__ __device__ __forceinline__ uint64_t entries_before_slow(int64_t t) const {
    return period && t > 0 ? uint64_t((t + int64_t(period) - 1) / int64_t(period)) * entries : 0u;
  }
  __host__ __device__ __forceinline__ uint32_t client_entries_slow(int64_t t) const {
    return (period && (t % int64_t(period)) == 0) ? entries : 0u;
  }
  __device__ __forceinline__ Trace at_tick(int64_t t) const {
    Trace x = *this;
    x.tick = t;
    x.now = int32_t(t * secs);
    x.n_tick = client_entries_slow(t);
    x.eb_tick = entries_before_slow(t);
    return x;
  }
  __device__ __forceinline__ uint32_t client_entries() const { return n_tick; }
  // Client entries of all ticks before t (ticks >= 0): the ring phase that
  // keeps every steady group's appends in the same slots (ring_phase()).
  __device__ __forceinline__ uint64_t entries_before(int64_t t) const {
    return t == tick ? eb_tick : entries_before_slow(t);
  }
};

// Exact u32 division by a launch constant d >= 1 (Granlund-Montgomery
// round-up with the add fix-up, as libdivide's branch-free u32 form): l =
// ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1; d = 1 is l = 0. One mulhi
// instead of the ~25-instruction runtime division.
__host__ __device__ __forceinline__ void udiv_magic_of(uint32_t d, uint32_t* m, uint32_t* l) {
  uint32_t ll = 0;
  while ((uint64_t(1) << ll) < d) ++ll;
  *l = ll;
  *m = ll ? uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << ll) - d)) / d + 1) : 0u;
}
__device__ __forceinline__ uint32_t udiv_magic(uint32_t x, uint32_t m, uint32_t l) {
  if (l == 0) return x;
  const uint32_t t = __umulhi(m, x);
  return (t + ((x - t) >> 1)) >> (l - 1);
}

// ------------------------------------------------------------------ RNG --
__host__ __device__ __forceinline__ uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
__host__ __device__ __forceinline__ uint64_t group_key(uint64_t seed, uint64_t gid) { return sm64(seed ^ sm64(gid)); }
__host__ __device__ __forceinline__ uint64_t rng_k(uint64_t key, uint32_t r, uint32_t stream, uint64_t tick) {
  return sm64(sm64(key ^ ((uint64_t(stream) << 32) | r)) ^ tick);
}

// VX (see M_VX): the value of a leader's client append that is the global
// client entry q (entry q mod E of client tick (q / E) * period; E entries
// per client tick), as the tick's client append draws it: value stream
// rng_k(key, r, ST_VALUE, tick), entry e = sm64(stream ^ e) >> 1 (rand.Int(),
// main.go:92). kv = sm64(key ^ (ST_VALUE << 32 | r)), the stream's key part.
__host__ __device__ __forceinline__ uint64_t vx_stream_key(uint64_t key, uint32_t r) {
  return sm64(key ^ ((uint64_t(ST_VALUE) << 32) | r));
}
__host__ __device__ __forceinline__ int64_t vx_value(uint64_t kv, uint64_t q, uint32_t E, uint32_t period) {
  const uint64_t qt = E == 1u ? q : q / E;
  const uint64_t qe = E == 1u ? 0u : q - qt * E;
  return int64_t(sm64(sm64(kv ^ (qt * period)) ^ qe) >> 1);
}

// Client values (rand.Int(), main.go:92 -> LogReq -> 327-329). A tick's
// client append of E entries by leader r of group g is described by one
// 64-bit value base vb: with the trace RNG (P.cv null) vb = rng_k(key, r,
// ST_VALUE, tick) and entry e is sm64(vb ^ e) >> 1; with staged values
// (raft_config.client_source RAFT_CLIENT_STAGED, P.cv) vb is the address of
// the group's entry-0 value of that tick in the caller's buffer and entry e is
// read at vb + e*G (every leader of the group appends the same request). The
// staged values are read once, when appended (non-temporal: they are not
// re-read, and must not push the per-group words out of the Infinity Cache).
__device__ __forceinline__ uint64_t cv_base(const DevPlanes& P, uint64_t key, uint32_t r, int64_t tick, uint32_t g) {
  if (P.cv) return uint64_t(reinterpret_cast<uintptr_t>(P.cv + uint64_t(tick - P.cv_t0) * P.cv_tstride + g));
  return rng_k(key, r, ST_VALUE, uint64_t(tick));
}
// stride: P.cv_stride when staged, 0 with the trace RNG
__device__ __forceinline__ int64_t cv_value(uint64_t vb, uint32_t e, uint64_t stride) {
  // (vb 0: a lane that appends nothing; its value is never used)
  if (stride) return vb ? __builtin_nontemporal_load(reinterpret_cast<const int64_t*>(uintptr_t(vb)) + uint64_t(e) * stride)
                        : 0;
  return int64_t(sm64(vb ^ uint64_t(e)) >> 1);
}
__device__ __forceinline__ uint64_t cv_stride(const DevPlanes& P) { return P.cv ? P.cv_stride : 0u; }

// Out-of-line RNG for the general kernels' unrolled per-replica code (the
// steady-state kernel inlines rng_k/sm64 directly).
__device__ __attribute__((noinline)) uint64_t rng_k_call(uint64_t key, uint32_t r, uint32_t stream, uint64_t tick) {
  return rng_k(key, r, stream, tick);
}
__device__ __attribute__((noinline)) int64_t entry_value(uint64_t vbase, uint32_t e, uint64_t stride) {   // main.go:92
  return cv_value(vbase, e, stride);
}

// Election timer duration min + (rng >> 32) % span (main.go:114, 194). Kept
// out of line: inlined into every unrolled handler copy, the 64-bit RNG gets
// speculated ahead of its branches and the general kernels run out of VGPRs.
__device__ __attribute__((noinline)) int timer_draw(uint64_t key, uint32_t r, uint32_t stream, int64_t tick, int mn,
                                                    int span) {
  const uint64_t h = rng_k(key, r, stream, uint64_t(tick));
  return mn + int(uint32_t(h >> 32) % uint32_t(span));
}

// --------------------------------------------------------------- CRC32C --
// EXT (config C5): CRC32C (Castagnoli, reflected) of an entry's payload =
// Term (4 B LE) || Value (8 B LE), slice-by-4 then slice-by-8 over the
// tables T[k][b] (T[0] = byte table, T[k][b] = T[k-1][b] >> 8 ^ T[0][T[k-1][b] & 255]),
// which may live in global memory or in LDS. Same definition as
// oracle_entry_crc() (bitwise reference, check value 0xE3069283).
__device__ __forceinline__ uint32_t crc_term_state(const uint32_t* T, int term) {
  const uint32_t c = 0xFFFFFFFFu ^ uint32_t(term);
  return T[768 + (c & 255)] ^ T[512 + ((c >> 8) & 255)] ^ T[256 + ((c >> 16) & 255)] ^ T[c >> 24];
}
__device__ __forceinline__ uint32_t crc_value_final(const uint32_t* T, uint32_t c, int64_t value) {
  const uint32_t lo = c ^ uint32_t(uint64_t(value)), hi = uint32_t(uint64_t(value) >> 32);
  return ~(T[1792 + (lo & 255)] ^ T[1536 + ((lo >> 8) & 255)] ^ T[1280 + ((lo >> 16) & 255)] ^ T[1024 + (lo >> 24)] ^
           T[768 + (hi & 255)] ^ T[512 + ((hi >> 8) & 255)] ^ T[256 + ((hi >> 16) & 255)] ^ T[hi >> 24]);
}
__device__ __forceinline__ uint32_t crc_entry(const uint32_t* T, int term, int64_t value) {
  return crc_value_final(T, crc_term_state(T, term), value);
}

// The followers' verification of one AppendEntries batch of n entries (value
// stream vb, the term's CRC state cs) against the leader's stamps, with the
// CRC computed once per entry: every follower receives the
// leader's bytes (main.go:148-149 appends what it received), so an unaltered
// copy has exactly the leader's stamp and needs no CRC; only the followers of
// `cm` receive an altered copy (EXT corruption: the batch's last value with
// bit 0 flipped), each checked against the leader's stamp of that entry.
// Returns the followers whose copy fails (a subset of cm).
__device__ __forceinline__ uint32_t crc_reject_mask(const uint32_t* T, uint32_t cs, uint64_t vb, uint64_t stride, int n,
                                                    uint32_t cm) {
  if (!cm || n <= 0) return 0u;
  const int64_t v = cv_value(vb, uint32_t(n - 1), stride);
  return crc_value_final(T, cs, v ^ 1) != crc_value_final(T, cs, v) ? cm : 0u;
}

// ------------------------------------------------- register-array helpers --
// Runtime-indexed access to a register array without letting LLVM fold the
// select chain into a dynamic GEP (which would demote the whole Group to
// scratch): each element is masked arithmetically and OR-ed (exclusive), and
// writes are unconditional selects per element.
template <int R>
__device__ __forceinline__ int sel(const int (&a)[R], int c) {
  int v = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) v |= a[i] & -int(c == i);
  return v;
}
template <int R>
__device__ __forceinline__ void put(int (&a)[R], int c, int v) {
#pragma unroll
  for (int i = 0; i < R; ++i) a[i] = (c == i) ? v : a[i];
}
// Per-replica array of one lane kept in LDS (general kernels): column
// `threadIdx.x` of a [R][256] int slab, so that consecutive lanes hit
// consecutive banks and a runtime replica index is one ds_read/ds_write
// instead of an R-way select chain in registers.
template <int R>
struct LArr {
  int* p;
  __device__ __forceinline__ int& operator[](int i) const { return p[i * 256]; }
};
template <int R>
__device__ __forceinline__ int sel(const LArr<R>& a, int c) { return a[c]; }
template <int R>
__device__ __forceinline__ void put(LArr<R>& a, int c, int v) { a[c] = v; }
// LDS ints one Group needs per lane (9 arrays of R)
template <int R>
constexpr int group_lds_ints() { return 9 * R; }

template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (N > 0) {
    static_for<N - 1>(f);
    f(std::integral_constant<int, N - 1>{});
  }
}

struct AEReq {          // AppendEntriesRequest (main.go:289-296), LeaderId implicit
  int term, prev_idx, prev_term, lc;
  int n;                // len(Logs)
  int corrupt;          // EXT: the last entry arrives with Value bit 0 flipped
};
struct AEResp { int term, match, ok; };  // AppendEntriesResponse (main.go:298-302)

// VX (see M_VX): writes group g's virtual suffix into its cut-off leader's
// ring column and drops the flag — the form's state as of the start of a tick
// whose client entries before it number Qb (entries_before(that tick)), so
// the suffix's last entry is the global client entry Qb - 1. Every reader
// other than the VX-aware fast paths runs this first. (RAFT only; never with
// payload CRC.)
template <int R>
__device__ __forceinline__ void vx_materialize(const DevPlanes& P, uint32_t g, uint64_t Qb, uint32_t E, uint32_t period,
                                               uint64_t seed) {
  const int meta = at(P.gmeta, g);
  if (!(meta & M_VX)) return;
  const int c = meta & 0xF;
  int xr = c, xlo = 0, xtop = 0, xterm = 0;
  if (meta & (M_LXS | M_SSYNC)) {   // LXS (the primary k ahead) or SXS (the stale leader xs = glx.dl)
    const SsRec s = P.gss[g];
    const LxRec x = P.glx[g];
    const bool lxs = (meta & M_LXS) != 0;
    xr = lxs ? c : x.dl;
    xlo = lxs ? s.last : at(P.lnext, rix<R>(g, xr)) - 1;
    xtop = s.last + x.k;
    xterm = lxs ? s.term : s.term - 1;
  } else {                          // ONESTALE, explicit rows: the other leader
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r != c && (at(P.rs, rix<R>(g, r)) & 3) == ROLE_L) xr = r;
    xlo = at(P.lnext, rix<R>(g, xr)) - 1;
    xtop = at(P.last, rix<R>(g, xr));
    xterm = at(P.term, rix<R>(g, xr));
  }
  const uint64_t tb = ring_tile(g, P.KP, R);
  const uint32_t rot = at(P.grot, g), rota = at(P.grota, g), rotb = at(P.grotb, g);
  const int sb = at(P.gsb, g), sb2 = at(P.gsb2, g);
  const uint64_t kv = vx_stream_key(group_key(seed, P.gbase + g), uint32_t(xr));
  const int lo = max(xlo, xtop - int(P.K));   // (older entries are out of every reader's window)
  for (int idx = lo + 1; idx <= xtop; ++idx) {
    const uint32_t o = ring_in_tile(g, R, ring_slot(idx, rot, rota, rotb, sb, sb2, P.kmask), uint32_t(xr));
    at(P.log_term + tb, o) = xterm;
    at(P.log_value + tb, o) = vx_value(kv, Qb - uint64_t(xtop - idx) - 1u, E, period);
  }
  at(P.gmeta, g) = uint16_t(meta & ~M_VX);
}

// SH (see ROT_SH): the live shared entries [max(shf, L-K+1), L] of group g
// (every log of length L: SSYNC, normal class) into all R replica columns.
// The caller clears ROT_SH in grot (or in its staged copy). Returns the
// number of entries copied.
template <int R>
__device__ __forceinline__ int sh_copy_back(const DevPlanes& P, uint32_t g, int L, int shf, uint32_t rot,
                                            uint32_t rota, uint32_t rotb, int sb, int sb2) {
  const uint64_t tb = ring_tile(g, P.KP, R), sb_t = sh_tile(g, P.KP);
  const int lo = max(shf, L - int(P.K) + 1), hi = L;
  for (int idx = lo; idx <= hi; ++idx) {
    const uint32_t slot = ring_slot(idx, rot, rota, rotb, sb, sb2, P.kmask);
    const uint32_t so = sh_in_tile(g, slot, P.sh_cs), o = ring_in_tile(g, R, slot, 0u);
    const int32_t t = at(P.sh_term + sb_t, so);
    const int64_t v = at(P.sh_value + sb_t, so);
    const uint32_t c = P.crc_on ? at(P.sh_crc + sb_t, so) : 0u;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      at(P.log_term + tb, o + uint32_t(r)) = t;
      at(P.log_value + tb, o + uint32_t(r)) = v;
      if (P.crc_on) at(P.log_crc + tb, o + uint32_t(r)) = c;
    }
  }
  return hi >= lo ? hi - lo + 1 : 0;
}
// ... reading every word from memory, writing the implied heartbeat time hb
// and clearing the bit (general kernels, one-pass kernel, the engine's flush).
// A group kept in shared form through a rejection (DevPlanes::sh_keep) may
// have explicit rows with one follower lagging: each column gets the shared
// entries of its own window [max(shf, last_r-K+1), last_r].
template <int R>
__device__ __forceinline__ void sh_materialize(const DevPlanes& P, uint32_t g, int32_t hb) {
  if (!P.sh) return;
  const uint32_t rot = at(P.grot, g);
  if (!(rot & ROT_SH)) return;
  const GSeg cw = P.gseg[g];
  const int sb = at(P.gsb, g);
  if (at(P.gmeta, g) & M_SSYNC) {
    sh_copy_back<R>(P, g, P.gss[g].last, cw.shf, rot, cw.rota, cw.rotb, sb, cw.sb2);
  } else {
    const uint64_t tb = ring_tile(g, P.KP, R), sb_t = sh_tile(g, P.KP);
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
      const int L = at(P.last, rix<R>(g, r));
      for (int idx = max(cw.shf, L - int(P.K) + 1); idx <= L; ++idx) {
        const uint32_t slot = ring_slot(idx, rot, cw.rota, cw.rotb, sb, cw.sb2, P.kmask);
        const uint32_t so = sh_in_tile(g, slot, P.sh_cs), o = ring_in_tile(g, R, slot, uint32_t(r));
        at(P.log_term + tb, o) = at(P.sh_term + sb_t, so);
        at(P.log_value + tb, o) = at(P.sh_value + sb_t, so);
        if (P.crc_on) at(P.log_crc + tb, o) = at(P.sh_crc + sb_t, so);
      }
    }
  }
  at(P.hb, g) = hb;   // (implied while shared: now of the last tick it was taken)
  at(P.grot, g) = uint16_t(rot & ~ROT_SH);
}

// Group context: the R replicas of one group, in registers. SEM selects the
// handler rules: SEM_REF = main.go bit for bit, SEM_RAFT = the EXT
// Raft-paper mode (same tick model and layout, see the r_* methods).
template <int R, int SEM = SEM_REF>
struct Group {
  // term, last, commit, dl (deadline), dur (timer duration), hw (RAFT:
  // high-water mark of each log; REF: unused) live in LDS (bind())
  LArr<R> term, last, commit, dl, dur, hw;
  // resident copies of the primary leader's MatchIndex / NextIndex rows and
  // of every replica's last-entry term (lmatch / lnext / lterm planes):
  // loaded once (rows lazily), written back once by store()
  LArr<R> pm, pn, ltm;
  uint32_t rows_m, rows_n;   // pm / pn hold the plane rows
  uint32_t rot, rot0;        // ring rotation (grot) now / as loaded
  uint32_t rota, rota0;      // previous segment's rotation (grota) now / as loaded
  int sb, sb0;               // segment boundary (gsb) now / as loaded
  uint32_t rotb;             // the segment before (grotb, gsb2; never changed by the general path)
  int sb2;
  uint32_t d_pm, d_pn, d_lt;
  uint32_t roles;       // 2 bits per replica
  uint32_t votes;       // 4 bits per replica: REF Voted (0/1), RAFT votedFor+1
  uint32_t known;       // deadline register valid
  uint32_t d_term, d_last, d_commit, d_dl, d_rs, d_hw;
  int primary, fault, meta0, hbt;
  uint32_t iso;         // EXT: replicas isolated during this tick
  uint32_t giso, giso0; // EXT leader-isolation victims (giso plane) now / as loaded
  uint32_t g;           // group index on this engine (lane)
  uint64_t key;
  int64_t tick;
  int32_t now;
  int st[NSTAT];
  // fast path for the entries appended by the client in this tick: the
  // follower copy regenerates them from the trace RNG instead of re-reading
  int cache_leader, cache_from, cache_term;
  uint64_t cache_vbase;

  __device__ __forceinline__ int role(int r) const { return int(roles >> (2 * r)) & 3; }
  __device__ __forceinline__ void set_role(int r, int v) {
    roles = (roles & ~(3u << (2 * r))) | (uint32_t(v) << (2 * r));
    d_rs |= 1u << r;
  }
  __device__ __forceinline__ int vote(int r) const { return int(votes >> (4 * r)) & 15; }
  __device__ __forceinline__ void set_vote(int r, int v) {
    votes = (votes & ~(15u << (4 * r))) | (uint32_t(v) << (4 * r));
    d_rs |= 1u << r;
  }
  __device__ __forceinline__ bool is_voted(int r) const { return vote(r) != 0; }
  __device__ __forceinline__ void set_voted(int r, bool v) { set_vote(r, v ? 1 : 0); }
  __device__ __forceinline__ void raise(int f) {
    if (!fault) fault = f;
  }
  __device__ __forceinline__ bool alive() const { return fault == 0; }
  __device__ __forceinline__ bool dropped(int a, int b) const { return ((iso >> a) | (iso >> b)) & 1u; }

  // ---------------------------------------------------------- load/store --
  // lds: a block's [6][R][256] int slab (shared by the lanes, column = lane)
  __device__ __forceinline__ void bind(int* lds) {
    int* b = lds + threadIdx.x;
    term.p = b; last.p = b + R * 256; commit.p = b + 2 * R * 256;
    dl.p = b + 3 * R * 256; dur.p = b + 4 * R * 256; hw.p = b + 5 * R * 256;
    pm.p = b + 6 * R * 256; pn.p = b + 7 * R * 256; ltm.p = b + 8 * R * 256;
  }
  __device__ __forceinline__ void begin(const DevPlanes& P, const Trace& T, uint32_t g_) {
    g = g_;
    key = group_key(T.seed, P.gbase + g);
    tick = T.tick;
    now = T.now;
    d_term = d_last = d_commit = d_dl = d_rs = d_hw = 0;
    d_pm = d_pn = d_lt = 0;
    rows_m = rows_n = 0;
    known = 0;
    iso = 0;
#pragma unroll
    for (int s = 0; s < NSTAT; ++s) st[s] = 0;
    cache_leader = -1;
    cache_from = 0; cache_term = 0; cache_vbase = 0;
    const int m = at(P.gmeta, g);
    meta0 = m;
    primary = m & 0xF;
    fault = (m >> 4) & 7;
    hbt = HB_NONE;
    rot = rot0 = at(P.grot, g);
    rota = rota0 = at(P.grota, g);
    sb = sb0 = at(P.gsb, g);
    rotb = at(P.grotb, g);
    sb2 = at(P.gsb2, g);
    giso = giso0 = at(P.giso, g);
  }
  // Per-tick reset of a group whose state stays resident across ticks
  // (general kernel catch-up): clock, counters, this tick's entry cache.
  __device__ __forceinline__ void next_tick(const Trace& T) {
    tick = T.tick;
    now = T.now;
    iso = 0;
#pragma unroll
    for (int s = 0; s < NSTAT; ++s) st[s] = 0;
    cache_leader = -1;
    cache_from = 0; cache_term = 0; cache_vbase = 0;
  }
  // Effective timer start: followers/candidates also count the last
  // steady-state heartbeat (hb), which resets every follower at once.
  __device__ __forceinline__ int eff_start(int ts, int r) const { return role(r) == ROLE_L ? ts : max(ts, hbt); }
  __device__ __forceinline__ void load(const DevPlanes& P, bool with_deadlines) {
    roles = 0; votes = 0;
    hbt = at(P.hb, g);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      term[r] = at(P.term, rix<R>(g, r));
      last[r] = at(P.last, rix<R>(g, r));
      commit[r] = at(P.commit, rix<R>(g, r));
      const uint32_t x = at(P.rs, rix<R>(g, r));
      roles |= (x & 3u) << (2 * r);
      votes |= ((x >> 2) & 15u) << (4 * r);
      dur[r] = int(x >> 6);
      hw[r] = (SEM == SEM_RAFT) ? at(P.hwm, rix<R>(g, r)) : 0;
      ltm[r] = at(P.lterm, rix<R>(g, r));
    }
#pragma unroll
    for (int r = 0; r < R; ++r) dl[r] = with_deadlines ? eff_start(at(P.tstart, rix<R>(g, r)), r) + dur[r] : 0;
    known = with_deadlines ? (1u << R) - 1u : 0u;
    // materialise the compressed state of an SSYNC group (written back by store)
    const LxRec x = (uses_glx(meta0) && primary < R) ? P.glx[g] : LxRec{0, 0};
    if ((meta0 & M_SSYNC) && primary < R) {
      const SsRec s = P.gss[g];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        term[r] = ss_term(s, r, meta0, x); last[r] = ss_last(s, r, primary, meta0, x);
        commit[r] = ss_commit(s, r, primary, meta0, x, commit[r]);
        ltm[r] = ss_term(s, r, meta0, x);
      }
      d_term = d_last = d_commit = d_lt = (1u << R) - 1u;
    }
    // materialise the rows the fast kernel kept implicit: MatchIndex = LastApplied
    // (RAFT also NextIndex = LastApplied+1 and high-water mark = LastApplied)
    if ((meta0 & M_MSYNC) && primary < R) {
      uint32_t peers = ((1u << R) - 1u) & ~(1u << primary);
      if (is_sxs(meta0)) peers &= ~(1u << x.dl);   // (SXS: the stale leader's row is explicit)
      rows_m = 1; d_pm = peers;
      if constexpr (SEM == SEM_RAFT) { rows_n = 1; d_pn = peers; }
#pragma unroll
      for (int p = 0; p < R; ++p) {
        if ((peers >> p) & 1u) {
          pm[p] = last[p];
          if constexpr (SEM == SEM_RAFT) pn[p] = last[p] + 1;
        } else if (p != primary) {   // explicit row (rows_m: pm holds every row)
          pm[p] = at(P.lmatch, rix<R>(g, p));
          if constexpr (SEM == SEM_RAFT) pn[p] = at(P.lnext, rix<R>(g, p));
        }
        if constexpr (SEM == SEM_RAFT) {   // max(plane, LastApplied) (HWX)
          if (hw[p] < last[p]) { hw[p] = last[p]; d_hw |= 1u << p; }
        }
      }
    }
  }
  // Also flushes the resident rows. next_phase: ring phase of the next tick to
  // be processed (entries_before(tick+1) mod K), taken by a group whose logs
  // are still empty (the fast kernel may append its first entry next).
  __device__ __forceinline__ void store(const DevPlanes& P, uint32_t next_phase) const {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if ((d_term >> r) & 1u) at(P.term, rix<R>(g, r)) = term[r];
      if ((d_last >> r) & 1u) at(P.last, rix<R>(g, r)) = last[r];
      if ((d_commit >> r) & 1u) at(P.commit, rix<R>(g, r)) = commit[r];
      if ((d_dl >> r) & 1u) at(P.tstart, rix<R>(g, r)) = dl[r] - dur[r];
      if ((d_rs >> r) & 1u)
        at(P.rs, rix<R>(g, r)) =
            int32_t(((roles >> (2 * r)) & 3u) | (((votes >> (4 * r)) & 15u) << 2) | (uint32_t(dur[r]) << 6));
      if (SEM == SEM_RAFT && ((d_hw >> r) & 1u)) at(P.hwm, rix<R>(g, r)) = hw[r];
      if ((d_lt >> r) & 1u) at(P.lterm, rix<R>(g, r)) = ltm[r];
      if ((d_pm >> r) & 1u) at(P.lmatch, rix<R>(g, r)) = pm[r];
      if (SEM == SEM_RAFT && ((d_pn >> r) & 1u)) at(P.lnext, rix<R>(g, r)) = pn[r];
    }
    {   // logs still empty: pick the phase of the next tick's first entry (the fast kernel may append it)
      bool empty = true;
#pragma unroll
      for (int r = 0; r < R; ++r) empty &= last[r] == 0 && (SEM != SEM_RAFT || hw[r] == 0);
      uint32_t rt = rot;
      int sbn = sb;
      if (empty && !fault) { rt = next_phase & P.kmask; sbn = 0; }
      if (rt != rot0) at(P.grot, g) = uint16_t(rt);
      if (sbn != sb0) at(P.gsb, g) = sbn;
      if (rota != rota0) at(P.grota, g) = uint16_t(rota);
      if (giso != giso0) at(P.giso, g) = uint8_t(giso);
    }
    // Primary placement (placement only; no state changes): the leader of the
    // highest term owns the coalesced MatchIndex / NextIndex planes, so that
    // a group whose newest leader is the active one (an older one cut off by
    // isolation) can take the steady-state kernel. The rows of the leader
    // that gives the planes up move to its xmatch / xnext rows.
    int pri = primary;
    if (!fault && ((roles >> 1) & ~roles & 0x5555u)) {
      int best = (pri < R && role(pri) == ROLE_L) ? pri : -1;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (role(r) == ROLE_L && (best < 0 || sel(term, r) > sel(term, best))) best = r;
      if (best != pri) {
#pragma unroll
        for (int p = 0; p < R; ++p) {
          const int a = at(P.lmatch, rix<R>(g, p));
          at(P.lmatch, rix<R>(g, p)) = at(prow(P.xmatch, best * R + p, P.Gp), g);
          if (pri < R) at(prow(P.xmatch, pri * R + p, P.Gp), g) = a;
          if constexpr (SEM == SEM_RAFT) {
            const int b = at(P.lnext, rix<R>(g, p));
            at(P.lnext, rix<R>(g, p)) = at(prow(P.xnext, best * R + p, P.Gp), g);
            if (pri < R) at(prow(P.xnext, pri * R + p, P.Gp), g) = b;
          }
        }
        pri = best;
      }
    }
    // DEFER and MSYNC are consumed by the general path; the class flags are recomputed
    const uint32_t others = roles & ~(3u << (2 * (pri & 15)));
    const bool led = pri < R && role(pri) == ROLE_L;
    const bool steady = led && others == 0u;
    // exactly one non-follower besides the primary: a candidate (ROLE_C = 1) ...
    const bool one = led && others != 0u && (others & (others - 1u)) == 0u;
    const bool onecand = one && (others & 0x5555u) != 0u;
    // ... or a leader (ROLE_L = 2) of a lower term (a stale leader still cut off)
    const int sx = one ? int(__builtin_ctz(others)) >> 1 : 0;
    const bool onestale = SEM == SEM_RAFT && one && (others & 0xAAAAu) != 0u && sel(term, sx) < sel(term, pri & 7);
    const int m = pri | (fault << 4) | (steady ? M_STEADY : 0) | (onecand ? M_ONECAND : 0) |
                  (onestale ? M_ONESTALE : 0) | (meta0 & M_DEFER);   // (DEFER: cleared by the window tail)
    if (m != meta0) at(P.gmeta, g) = uint16_t(m);
  }

  // Log ring of replica r: entry idx (1-based) at slot (idx-1) mod K.
  __device__ __forceinline__ uint32_t ring_off(const DevPlanes& P, int r, int idx) const {
    return ring_in_tile(g, R, ring_slot(idx, rot, rota, rotb, sb, sb2, P.kmask), uint32_t(r));
  }
  // Every log of the group is empty (RAFT: nothing above LastApplied either):
  // the ring holds no entry, so its rotation is free. Chosen so that the
  // entry appended at tick t lands in slot entries_before(t) mod K, the slot
  // every other steady group appends to at t (coalesced ring rows).
  __device__ __forceinline__ void align_ring(const DevPlanes& P, const Trace& T) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (last[r] != 0 || (SEM == SEM_RAFT && hw[r] != 0)) return;
    rot = uint32_t(T.entries_before(T.tick)) & P.kmask;
    sb = 0;
  }
  __device__ __forceinline__ int32_t& ring_term(const DevPlanes& P, int r, int idx) const {
    return at(P.log_term + ring_tile(g, P.KP, R), ring_off(P, r, idx));
  }
  __device__ __forceinline__ int64_t& ring_value(const DevPlanes& P, int r, int idx) const {
    return at(P.log_value + ring_tile(g, P.KP, R), ring_off(P, r, idx));
  }
  __device__ __forceinline__ uint32_t& ring_crc(const DevPlanes& P, int r, int idx) const {
    return at(P.log_crc + ring_tile(g, P.KP, R), ring_off(P, r, idx));
  }
  // EXT: is the AppendEntries delivered to replica p this tick corrupted?
  __device__ __forceinline__ int corrupted(const DevPlanes& P, int p) const {
    if (!P.crc_on || !P.corrupt_p) return 0;
    return (rng_k_call(key, uint32_t(p), ST_CORRUPT, uint64_t(tick)) & 0xFFFF) < P.corrupt_p;
  }
  // Timer of replica r (lazy: only read from HBM when a timeout check needs it).
  template <int Rp>
  __device__ __forceinline__ int deadline_of(const DevPlanes& P) {
    if (!((known >> Rp) & 1u)) {
      dl[Rp] = eff_start(at(P.tstart, rix<R>(g, Rp)), Rp) + dur[Rp];
      known |= 1u << Rp;
    }
    return dl[Rp];
  }

  // ------------------------------------------------------------ timers --
  __device__ __forceinline__ int draw(const Trace& T, int r, bool cand) const {
    return cand ? timer_draw(key, uint32_t(r), ST_TIMER_C, tick, T.c_min, T.c_span)
                : timer_draw(key, uint32_t(r), ST_TIMER_F, tick, T.f_min, T.f_span);
  }
  // FollowerRun entry: d = rand.Intn(20)+10, timer started (main.go:113-115).
  template <int Rp>
  __device__ __forceinline__ void enter_follower(const Trace& T) {
    set_role(Rp, ROLE_F);
    dur[Rp] = draw(T, Rp, false);
    dl[Rp] = now + dur[Rp];
    known |= 1u << Rp;
    d_dl |= 1u << Rp;
  }
  // CandidateRun entry: d = rand.Intn(4)+10 (main.go:194-195).
  __device__ __forceinline__ void enter_candidate(const Trace& T, int c) {
    set_role(c, ROLE_C);
    const int d = draw(T, c, true);
    put(dur, c, d);
    put(dl, c, now + d);
    known |= 1u << c;
    d_dl |= 1u << c;
  }
  template <int Rp>
  __device__ __forceinline__ void reset_timer() {   // timer.Reset(d)
    dl[Rp] = now + dur[Rp];
    known |= 1u << Rp;
    d_dl |= 1u << Rp;
  }
  // Log[idx].Term of replica r (1 <= idx <= its LastApplied): the last entry's
  // term is resident (ltm), so the common prevLogIndex == LastApplied check
  // costs no dependent HBM read; older entries come from the ring.
  __device__ __forceinline__ int term_at(const DevPlanes& P, int r, int idx) const {
    return idx == last[r] ? ltm[r] : ring_term(P, r, idx);
  }
  __device__ __forceinline__ void set_lterm(int r, int t) {   // Log[len-1].Term cache
    if (ltm[r] != t) { ltm[r] = t; d_lt |= 1u << r; }
  }
  template <int Rp>
  __device__ __forceinline__ void set_term(int t) {
    if (term[Rp] != t) { term[Rp] = t; d_term |= 1u << Rp; }
  }

  // Entries j0..n-1 of an AppendEntries into replica r's ring at base+1+j, in
  // batches of 4 whose loads are issued before their stores (the source is
  // the leader's ring or a host buffer, never r's own ring), so a catch-up of
  // n entries costs n/4 dependent memory round trips instead of n. Returns the
  // term of the last entry written.
  template <typename Src>
  __device__ __forceinline__ int copy_entries(const DevPlanes& P, int r, int base, int j0, int n, const Src& src) {
    int tl = 0;
    for (int j = j0; j < n; j += 4) {
      int t[4];
      int64_t v[4];
      uint32_t c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j + u < n) src.fetch(j + u, t[u], v[u], c[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (j + u >= n) break;
        ring_term(P, r, base + 1 + j + u) = t[u];
        ring_value(P, r, base + 1 + j + u) = v[u];
        if (P.crc_on) ring_crc(P, r, base + 1 + j + u) = c[u];
        tl = t[u];
      }
    }
    return tl;
  }

  // -------------------------------------------- AppendEntries receivers --
  // FollowerRun case AEReq (main.go:121-156). `src.fetch(j, t, v)` yields
  // Logs[j].
  template <int Rp, typename Src>
  __device__ __forceinline__ AEResp follower_ae(const DevPlanes& P, const AEReq& q, const Src& src) {
    AEResp res{term[Rp], last[Rp], 0};
    reset_timer<Rp>();                                        // 124-127
    if (q.term < term[Rp]) return res;                        // 129-133
    const int l = last[Rp];
    if (l > 0) {                                              // 135
      if (int64_t(l) + q.n < q.prev_idx) return res;          // 137-140
      if (q.prev_idx < 1 || q.prev_idx > l) { raise(F_PANIC_GETLOG); return res; }  // 142 -> 404
      if (q.prev_idx <= l - int(P.K)) { raise(F_RING_EVICTED); return res; }
      if (term_at(P, Rp, q.prev_idx) != q.prev_term) return res;                   // 142-145
    }
    if (int64_t(l) + q.n > I32MAX) { raise(F_OVERFLOW); return res; }
    // 148-149: append all Logs at the end (no truncation); only the last K
    // positions are kept in the ring.
    const int j0 = q.n > int(P.K) ? q.n - int(P.K) : 0;
    if (P.crc_on) {   // EXT: verify the payload that will be stored; a bad entry rejects the request
      for (int j = j0; j < q.n; ++j) {
        int t; int64_t v; uint32_t c;
        src.fetch(j, t, v, c);
        if (q.corrupt && j == q.n - 1) v ^= 1;
        if (crc_entry(P.crc_tab, t, v) != c) return res;
      }
    }
    const int tl = copy_entries(P, Rp, l, j0, q.n, src);
    const int nl = l + q.n;
    if (q.n) {
      last[Rp] = nl;
      d_last |= 1u << Rp;
      set_lterm(Rp, tl);
    }
    if (q.lc > commit[Rp]) {                                  // 151-152: min(LC, len(Log)+1)
      const int64_t cap = int64_t(nl) + 1;
      const int nc = int64_t(q.lc) < cap ? q.lc : int(cap);
      if (nc != commit[Rp]) { commit[Rp] = nc; d_commit |= 1u << Rp; }
    }
    set_term<Rp>(q.term);                                     // 155
    res.term = q.term; res.match = nl; res.ok = 1;            // 156
    return res;
  }
  // CandidateRun case AEReq (main.go:200-223).
  template <int Rp>
  __device__ __forceinline__ AEResp candidate_ae(const Trace& T, const AEReq& q) {
    AEResp res{term[Rp], last[Rp], 0};
    if (q.term >= term[Rp]) {                                 // 204
      res.ok = 1;                                             // 205-209 (nothing appended)
      set_voted(Rp, true);                                    // 211
      set_term<Rp>(q.term);                                   // 212
      enter_follower<Rp>(T);                                  // 210, 213-216
    }
    return res;
  }
  // LeaderRun case AEReq (main.go:309-326).
  template <int Rp>
  __device__ __forceinline__ AEResp leader_ae(const Trace& T, const AEReq& q) {
    AEResp res{term[Rp], 0, 0};
    if (q.term > term[Rp]) {                                  // 312
      res.ok = 1;                                             // 313-316 (MatchIndex 0)
      set_voted(Rp, false);                                   // 318
      set_term<Rp>(q.term);                                   // 319
      enter_follower<Rp>(T);                                  // 317, 320
      if (primary == Rp) primary = NO_PRIMARY;
    }
    return res;
  }
  // Run (main.go:98-109): the message goes to the receiver's current role.
  template <int Rp, typename Src>
  __device__ __forceinline__ AEResp deliver_ae(const DevPlanes& P, const Trace& T, const AEReq& q,
                                               const Src& src) {
    const int ro = role(Rp);
    if (ro == ROLE_F) return follower_ae<Rp>(P, q, src);
    if (ro == ROLE_C) return candidate_ae<Rp>(T, q);
    return leader_ae<Rp>(T, q);
  }

  // ---------------------------------------------- RequestVote receivers --
  template <int Rp>
  __device__ __forceinline__ int deliver_vr(const Trace& T, int rterm, int* resp_term) {
    const int ro = role(Rp);
    *resp_term = term[Rp];
    if (ro == ROLE_F) {                                       // main.go:157-170
      if (rterm < term[Rp] || is_voted(Rp)) return 0;         // 160-162
      reset_timer<Rp>();                                      // 164-167
      set_term<Rp>(rterm);                                    // 168
      set_voted(Rp, true);                                    // 169
      *resp_term = rterm;
      return 1;                                               // 170
    }
    if (ro == ROLE_C) {                                       // main.go:224-246
      if (rterm > term[Rp]) {                                 // 227-238
        set_voted(Rp, true);
        set_term<Rp>(rterm);
        enter_follower<Rp>(T);
        return 1;
      }
      reset_timer<Rp>();                                      // 243-246
      raise(F_DEADLOCK_VRES);                                 // 242: reply into its own VRes
      return 0;
    }
    raise(F_DEADLOCK_LEADER_VREQ);                            // main.go:308: no VReq case
    return 0;
  }

  // ------------------------------------------------------- node steps ----
  // CandidateRun default branch (main.go:253-284); c is a runtime id.
  __device__ __forceinline__ int candidate_round(const DevPlanes& P, const Trace& T, int c) {
    int count = 1;                                            // 255
    set_voted(c, true);                                       // 256
    const int ct = sel(term, c);
    static_for<R>([&](auto PI) {                              // 259-269
      constexpr int p = decltype(PI)::value;
      if (p == c || !alive() || dropped(c, p)) return;
      int rt;
      const int gr = deliver_vr<p>(T, ct, &rt);               // 264-265
      if (alive() && gr) { ++count; ++st[S_VOTES]; }          // 266-268
    });
    if (alive() && 2 * count > R) {                           // 273
      set_role(c, ROLE_L);                                    // 274
      // 275-282: MatchIndex 0 / NextIndex 1 for every peer
      if (primary == NO_PRIMARY) {
        primary = c;
#pragma unroll
        for (int p = 0; p < R; ++p)
          if (p != c) pm[p] = 0;
        rows_m = 1;
        d_pm |= ((1u << R) - 1u) & ~(1u << c);
      } else {
#pragma unroll
        for (int p = 0; p < R; ++p)
          if (p != c) at(prow(P.xmatch, c * R + p, P.Gp), g) = 0;
      }
      ++st[S_WON];
      return 1;
    }
    return 0;
  }

  // Commit rule (main.go:381-391): exact-value histogram over the peers'
  // MatchIndex (leader excluded); at most one value can hold a majority.
  __device__ __forceinline__ int commit_rule(const int (&m)[R], int c, int cm) {
#pragma unroll
    for (int p = 0; p < R; ++p) {
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < R; ++q) cnt += (q != c && m[q] == m[p]) ? 1 : 0;
      if (p != c && 2 * cnt > R && m[p] > cm) {               // 387
        st[S_COMMITTED] += m[p] - cm;
        cm = m[p];                                            // 389
      }
    }
    return cm;
  }

  // MatchIndex row of leader c: the primary leader's row lives in the
  // coalesced lmatch planes, any other concurrent leader's in xmatch.
  __device__ __forceinline__ void load_match(const DevPlanes& P, int c, int (&m)[R]) {
    if (primary == c) {
      if (!rows_m) {
#pragma unroll
        for (int p = 0; p < R; ++p) pm[p] = at(P.lmatch, rix<R>(g, p));
        rows_m = 1;
      }
#pragma unroll
      for (int p = 0; p < R; ++p) m[p] = (p != c) ? pm[p] : 0;
    } else {
#pragma unroll
      for (int p = 0; p < R; ++p) m[p] = (p != c) ? at(prow(P.xmatch, c * R + p, P.Gp), g) : 0;
    }
  }
  __device__ __forceinline__ void store_match(const DevPlanes& P, int c, const int (&m)[R], uint32_t dirty) {
    if (primary == c) {
      dirty &= ~(1u << c);
      if (!rows_m && dirty != (((1u << R) - 1u) & ~(1u << c))) {   // partial update: fetch the row first
#pragma unroll
        for (int p = 0; p < R; ++p) pm[p] = at(P.lmatch, rix<R>(g, p));
      }
      rows_m = 1;
#pragma unroll
      for (int p = 0; p < R; ++p)
        if ((dirty >> p) & 1u) pm[p] = m[p];
      d_pm |= dirty;
    } else {
#pragma unroll
      for (int p = 0; p < R; ++p)
        if (p != c && ((dirty >> p) & 1u)) at(prow(P.xmatch, c * R + p, P.Gp), g) = m[p];
    }
  }

  // LeaderRun default branch (main.go:332-391) for runtime leader id c.
  // Src builds the entry source for this leader.
  template <typename SrcF>
  __device__ __forceinline__ void leader_round(const DevPlanes& P, const Trace& T, int c, const SrcF& make_src) {
    const int lt = sel(term, c), ll = sel(last, c);
    const int lc = sel(commit, c);
    int m[R];
    uint32_t mdirty = 0;
    load_match(P, c, m);
    const auto src0 = make_src(c);
    static_for<R>([&](auto PI) {                              // 334-379
      constexpr int p = decltype(PI)::value;
      if (p == c || !alive()) return;
      if (dropped(c, p)) { ++st[S_AE_FAIL]; return; }
      AEReq q;
      q.term = lt; q.lc = lc;
      q.corrupt = corrupted(P, p);
      const int nxt = m[p] + 1;                               // NextIndex == MatchIndex + 1
      int from = 1;
      if (nxt <= ll) {                                        // 341
        if (nxt == 1) {                                       // 343-351: whole log
          q.n = ll; q.prev_idx = 0; q.prev_term = lt; from = 1;
        } else {                                              // 353-360
          if (nxt < 1 || m[p] > ll) { raise(F_PANIC_GETLOG); return; }
          if (m[p] <= ll - int(P.K)) { raise(F_RING_EVICTED); return; }
          q.prev_term = term_at(P, c, m[p]);                  // GetLog(MatchIndex).Term
          q.prev_idx = m[p]; q.n = ll - nxt + 1; from = nxt;
        }
      } else {                                                // 364-371: heartbeat
        q.n = 0; q.prev_idx = m[p]; q.prev_term = lt;
      }
      auto src = src0;
      src.from = from;
      const AEResp a = deliver_ae<p>(P, T, q, src);           // -> 373
      if (!alive()) return;
      if (a.ok) {                                             // 375-378
        if (a.match != m[p]) { m[p] = a.match; mdirty |= 1u << p; }
        ++st[S_AE_OK];
      } else {
        ++st[S_AE_FAIL];
      }
    });
    if (alive()) {
      const int nc = commit_rule(m, c, lc);
      if (nc != lc) { put(commit, c, nc); d_commit |= 1u << c; }
    }
    store_match(P, c, m, mdirty);
  }

  // Client append to leader c (main.go:327-329): Log += {Term, Value}; LastApplied++.
  __device__ __forceinline__ void client_append_value(const DevPlanes& P, int c, int64_t v) {
    const int l = sel(last, c);
    if (l >= I32MAX) { raise(F_OVERFLOW); return; }
    const int t = sel(term, c);
    ring_term(P, c, l + 1) = t;
    ring_value(P, c, l + 1) = v;
    if (P.crc_on) ring_crc(P, c, l + 1) = crc_entry(P.crc_tab, t, v);
    set_lterm(c, t);
    put(last, c, l + 1);
    d_last |= 1u << c;
    if (SEM == SEM_RAFT && l + 1 > sel(hw, c)) { put(hw, c, l + 1); d_hw |= 1u << c; }
  }

  // timer.C (main.go:171-177 follower -> candidate, 248-251 candidate Term++).
  __device__ __forceinline__ void timeout_fire(const Trace& T, int c) {
    const int t = sel(term, c);
    if (t >= I32MAX) { raise(F_OVERFLOW); return; }
    put(term, c, t + 1);
    d_term |= 1u << c;
    ++st[S_BUMPS];
    enter_candidate(T, c);
  }

  // =====================================================================
  // EXT RAFT-paper semantics (SEM_RAFT; Ongaro & Ousterhout, Figure 2), the
  // device twin of oracle/raft_oracle.c's r_* functions. Same tick model.
  // =====================================================================
  // A higher term in any RPC: adopt it, forget the vote, become a follower.
  template <int Rp>
  __device__ __forceinline__ void r_observe(const Trace& T, int t) {
    if (t <= term[Rp]) return;
    set_term<Rp>(t);
    set_vote(Rp, 0);
    if (role(Rp) != ROLE_F) {
      if (primary == Rp) primary = NO_PRIMARY;
      enter_follower<Rp>(T);
    }
  }
  __device__ __forceinline__ void r_observe_rt(const Trace& T, int c, int t) {   // runtime replica id
    if (t <= sel(term, c)) return;
    put(term, c, t);
    d_term |= 1u << c;
    set_vote(c, 0);
    if (role(c) != ROLE_F) {
      if (primary == c) primary = NO_PRIMARY;
      set_role(c, ROLE_F);
      const int d = draw(T, c, false);
      put(dur, c, d);
      put(dl, c, now + d);
      known |= 1u << c;
      d_dl |= 1u << c;
    }
  }
  __device__ __forceinline__ int lterm_of(const DevPlanes& P, int r, int l) const {
    return l > 0 ? ltm[r] : 0;
  }
  template <int Rp>
  __device__ __forceinline__ void r_grew(int nl) {   // the log reached length nl
    if (nl > hw[Rp]) { hw[Rp] = nl; d_hw |= 1u << Rp; }
  }

  template <int Rp>
  __device__ __forceinline__ int r_deliver_vr(const DevPlanes& P, const Trace& T, int t, int cand, int llast,
                                              int llterm, int* resp_term) {
    r_observe<Rp>(T, t);
    *resp_term = term[Rp];
    if (t < term[Rp]) return 0;
    const int mt = lterm_of(P, Rp, last[Rp]);
    const bool uptodate = llterm > mt || (llterm == mt && llast >= last[Rp]);
    const int v = vote(Rp);
    if ((v == 0 || v == cand + 1) && uptodate) {
      set_vote(Rp, cand + 1);
      reset_timer<Rp>();                          // granting a vote resets the election timer
      return 1;
    }
    return 0;
  }

  // On failure res.match is the hint H: the leader retries from min(next-1, H+1).
  // H = last (log too short), min(prevLogIndex-1, commitIndex) on a term
  // conflict (the committed prefix matches every later leader's log), or
  // prevLogIndex on an EXT payload CRC mismatch.
  template <int Rp, typename Src>
  __device__ __forceinline__ AEResp r_deliver_ae(const DevPlanes& P, const Trace& T, const AEReq& q,
                                                 const Src& src) {
    r_observe<Rp>(T, q.term);
    AEResp res{term[Rp], last[Rp], 0};
    if (q.term < term[Rp]) return res;
    if (role(Rp) == ROLE_L) return res;           // same-term second leader: cannot happen
    if (role(Rp) == ROLE_C) enter_follower<Rp>(T);
    reset_timer<Rp>();
    const int l = last[Rp];
    const int K = int(P.K);
    if (q.prev_idx > l) return res;               // log too short: hint = last
    if (q.prev_idx > 0) {
      if (q.prev_idx <= hw[Rp] - K) { raise(F_RING_EVICTED); return res; }
      if (term_at(P, Rp, q.prev_idx) != q.prev_term) {       // conflict: back off to the committed prefix
        res.match = q.prev_idx - 1 < commit[Rp] ? q.prev_idx - 1 : commit[Rp];
        return res;
      }
    }
    if (P.crc_on) {                               // EXT: verify what will be stored
      const int j0 = q.n > K ? q.n - K : 0;
      for (int j = j0; j < q.n; ++j) {
        int t; int64_t v; uint32_t c;
        src.fetch(j, t, v, c);
        if (q.corrupt && j == q.n - 1) v ^= 1;
        if (crc_entry(P.crc_tab, t, v) != c) { res.match = q.prev_idx; return res; }
      }
    }
    if (int64_t(q.prev_idx) + q.n > I32MAX) { raise(F_OVERFLOW); return res; }
    // skip entries already present, truncate at the first conflict, append the rest
    int j = 0;
    for (; j < q.n; ++j) {
      const int idx = q.prev_idx + 1 + j;
      if (idx > l) break;
      if (idx <= hw[Rp] - K) { raise(F_RING_EVICTED); return res; }
      int t; int64_t v; uint32_t c;
      src.fetch(j, t, v, c);
      if (term_at(P, Rp, idx) != t) break;       // conflict: entries from idx on are replaced
    }
    if (j < q.n) {
      const int tl = copy_entries(P, Rp, q.prev_idx, j, q.n, src);
      const int nl = q.prev_idx + q.n;
      if (nl != l) { last[Rp] = nl; d_last |= 1u << Rp; }
      set_lterm(Rp, tl);
      r_grew<Rp>(nl);
    }
    const int last_new = q.prev_idx + q.n;
    if (q.lc > commit[Rp]) {
      const int nc = q.lc < last_new ? q.lc : last_new;
      if (nc != commit[Rp]) { commit[Rp] = nc; d_commit |= 1u << Rp; }
    }
    res.term = term[Rp]; res.match = last_new; res.ok = 1;
    return res;
  }

  __device__ __forceinline__ int r_candidate_round(const DevPlanes& P, const Trace& T, int c) {
    int count = 1;                                // its own vote (votedFor = self since the timeout)
    const int ct = sel(term, c), cl = sel(last, c);
    const int clt = lterm_of(P, c, cl);
    bool stop = false;
    static_for<R>([&](auto PI) {
      constexpr int p = decltype(PI)::value;
      if (p == c || stop || !alive() || dropped(c, p)) return;
      int rt;
      const int gr = r_deliver_vr<p>(P, T, ct, c, cl, clt, &rt);
      if (!alive()) return;
      if (rt > ct) { r_observe_rt(T, c, rt); stop = true; return; }
      if (gr) { ++count; ++st[S_VOTES]; }
    });
    if (alive() && !stop && role(c) == ROLE_C && 2 * count > R) {
      set_role(c, ROLE_L);
      int m[R], nx[R];
#pragma unroll
      for (int p = 0; p < R; ++p) { m[p] = 0; nx[p] = cl + 1; }
      if (primary == NO_PRIMARY) primary = c;
      store_match(P, c, m, (1u << R) - 1u);
      store_next(P, c, nx, (1u << R) - 1u);
      ++st[S_WON];
      return 1;
    }
    return 0;
  }

  __device__ __forceinline__ void load_next(const DevPlanes& P, int c, int (&nx)[R]) {
    if (primary == c) {
      if (!rows_n) {
#pragma unroll
        for (int p = 0; p < R; ++p) pn[p] = at(P.lnext, rix<R>(g, p));
        rows_n = 1;
      }
#pragma unroll
      for (int p = 0; p < R; ++p) nx[p] = (p != c) ? pn[p] : 0;
    } else {
#pragma unroll
      for (int p = 0; p < R; ++p) nx[p] = (p != c) ? at(prow(P.xnext, c * R + p, P.Gp), g) : 0;
    }
  }
  __device__ __forceinline__ void store_next(const DevPlanes& P, int c, const int (&nx)[R], uint32_t dirty) {
    if (primary == c) {
      dirty &= ~(1u << c);
      if (!rows_n && dirty != (((1u << R) - 1u) & ~(1u << c))) {
#pragma unroll
        for (int p = 0; p < R; ++p) pn[p] = at(P.lnext, rix<R>(g, p));
      }
      rows_n = 1;
#pragma unroll
      for (int p = 0; p < R; ++p)
        if ((dirty >> p) & 1u) pn[p] = nx[p];
      d_pn |= dirty;
    } else {
#pragma unroll
      for (int p = 0; p < R; ++p)
        if (p != c && ((dirty >> p) & 1u)) at(prow(P.xnext, c * R + p, P.Gp), g) = nx[p];
    }
  }

  // commitIndex = the largest N held by a majority (leader included), only
  // if log[N].term == currentTerm.
  __device__ __forceinline__ int r_commit_rule(const DevPlanes& P, const int (&m)[R], int c, int cm) {
    const int ll = sel(last, c), lt = sel(term, c), lh = sel(hw, c);
    int v[R];
#pragma unroll
    for (int p = 0; p < R; ++p) v[p] = (p == c) ? ll : m[p];
    int N = -1;
#pragma unroll
    for (int p = 0; p < R; ++p) {   // the (R/2+1)-th largest value
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < R; ++q) cnt += v[q] >= v[p] ? 1 : 0;
      if (cnt >= R / 2 + 1 && v[p] > N) N = v[p];
    }
    if (N > cm) {
      if (N < 1 || N > ll) { raise(F_PANIC_GETLOG); return cm; }
      if (N <= lh - int(P.K)) { raise(F_RING_EVICTED); return cm; }
      if (term_at(P, c, N) == lt) {
        st[S_COMMITTED] += N - cm;
        return N;
      }
    }
    return cm;
  }

  template <typename SrcF>
  __device__ __forceinline__ void r_leader_round(const DevPlanes& P, const Trace& T, int c, const SrcF& make_src) {
    const int lt = sel(term, c), ll = sel(last, c), lc = sel(commit, c), lh = sel(hw, c);
    const int K = int(P.K);
    int m[R], nx[R];
    uint32_t dirty = 0;
    load_match(P, c, m);
    load_next(P, c, nx);
    const int pri = primary;   // row location of c as loaded (c may step down below)
    const auto src0 = make_src(c);
    bool stop = false;
    static_for<R>([&](auto PI) {
      constexpr int p = decltype(PI)::value;
      if (p == c || stop || !alive()) return;
      if (dropped(c, p)) { ++st[S_AE_FAIL]; return; }
      const int nxt = nx[p];
      if (nxt < 1 || nxt > ll + 1) { raise(F_PANIC_GETLOG); return; }
      if (nxt <= lh - K) { raise(F_RING_EVICTED); return; }
      AEReq q;
      q.term = lt; q.lc = lc;
      q.corrupt = corrupted(P, p);
      q.prev_idx = nxt - 1;
      q.prev_term = 0;
      if (q.prev_idx > 0) {
        if (q.prev_idx <= lh - K) { raise(F_RING_EVICTED); return; }
        q.prev_term = term_at(P, c, q.prev_idx);
      }
      q.n = ll - q.prev_idx;
      auto src = src0;
      src.from = nxt;
      const AEResp a = r_deliver_ae<p>(P, T, q, src);
      if (!alive()) return;
      if (a.term > lt) { r_observe_rt(T, c, a.term); ++st[S_AE_FAIL]; stop = true; return; }
      if (a.ok) {
        m[p] = a.match; nx[p] = a.match + 1; dirty |= 1u << p;
        ++st[S_AE_OK];
      } else {
        int nn = nx[p] - 1 < a.match + 1 ? nx[p] - 1 : a.match + 1;
        nn = nn < 1 ? 1 : nn;
        if (nn != nx[p]) { nx[p] = nn; dirty |= 1u << p; }
        ++st[S_AE_FAIL];
      }
    });
    if (alive() && !stop) {
      const int nc = r_commit_rule(P, m, c, lc);
      if (nc != lc) { put(commit, c, nc); d_commit |= 1u << c; }
    }
    // rows are written where they were read (c's rows are dead if it stepped down)
    const int keep = primary;
    primary = pri;
    store_match(P, c, m, dirty);
    store_next(P, c, nx, dirty);
    primary = keep;
  }

  __device__ __forceinline__ void r_timeout_fire(const Trace& T, int c) {
    const int t = sel(term, c);
    if (t >= I32MAX) { raise(F_OVERFLOW); return; }
    put(term, c, t + 1);
    d_term |= 1u << c;
    set_vote(c, c + 1);                            // votes for itself
    ++st[S_BUMPS];
    enter_candidate(T, c);
  }
};

// Entry source of a leader round inside the fused tick: entries appended by
// this tick's client event are regenerated from the trace RNG, older ones
// are read from the leader's ring. Held by value (no pointer to the
// register-resident Group, which would force it into scratch).
struct TickSrc {
  const int32_t* lt;
  const int64_t* lv;
  const uint32_t* lc;
  const uint32_t* tab;
  uint32_t crc_on;
  uint32_t R;          // replicas (ring layout)
  uint32_t g, KP, kmask, rot, rota, rotb;
  int sb, sb2;
  int leader, from;
  int cache_leader, cache_from, cache_term;
  uint64_t cache_vbase;
  uint64_t cv_stride;   // (cv_value: 0 = trace RNG)
  __device__ __forceinline__ void fetch(int j, int& t, int64_t& v, uint32_t& c) const {
    const int idx = from + j;
    c = 0;
    if (leader == cache_leader && idx >= cache_from) {
      t = cache_term;
      v = entry_value(cache_vbase, uint32_t(idx - cache_from), cv_stride);
      if (crc_on) c = crc_entry(tab, t, v);   // the leader's stamp of its own fresh entry
    } else {
      const uint64_t tb = ring_tile(g, KP, R);
      const uint32_t o = ring_in_tile(g, R, ring_slot(idx, rot, rota, rotb, sb, sb2, kmask), uint32_t(leader));
      t = at(lt + tb, o);
      v = at(lv + tb, o);
      if (crc_on) c = at(lc + tb, o);
    }
  }
};

// Entry source of a host-supplied AppendEntriesRequest (handler batch API);
// host payloads are stamped on ingest. Every term is staged; values and
// stamps only for Logs[skip..n), the last K (all that can land in the ring).
struct HostSrc {
  const int32_t* et;
  const int64_t* ev;
  const uint32_t* ec;
  uint64_t off, voff;
  uint32_t skip;
  int from;
  __device__ __forceinline__ void fetch(int j, int& t, int64_t& v, uint32_t& c) const {
    t = et[off + uint64_t(j)];
    if (uint32_t(j) < skip) { v = 0; c = 0; return; }
    const uint64_t k = voff + uint64_t(uint32_t(j) - skip);
    v = ev[k];
    c = ec[k];
  }
};

}  // namespace raftstep
