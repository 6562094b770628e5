/*
 * raftstep.h — C-ABI of the MI355X-native batched Raft step engine.
 *
 * This is the drop-in boundary for the hot path of eastwd/raft-sample:
 * the RequestVote / AppendEntries handlers and the leader commit logic of
 * main.go (FollowerRun main.go:111-180, CandidateRun main.go:193-287,
 * LeaderRun main.go:304-397). The reference has no exported API: its
 * handlers are inline `select` cases over `*Node` (main.go:14-39) and the
 * message structs (main.go:42-49, 182-191, 289-302). Each entry point below
 * names the reference code it replaces; INTEGRATION.md shows the cgo stub a
 * maintainer adds to main.go's package to call it.
 *
 * Rules of the ABI:
 *  - plain C types only; no torch / HIP types in any signature;
 *  - every function returns 0 on success or a negative errno-style code
 *    (RAFT_E*); the message is available from raft_last_error();
 *  - caller-owned host buffers are only borrowed for the duration of a call
 *    (cgo pointer rules: nothing is retained after return);
 *  - one engine = one GPU = one host thread at a time (not re-entrant).
 *
 * Semantics are the reference's ("REF") bit for bit,
 * including its quirks; where the reference would panic or deadlock the
 * group is frozen with a per-group fault code instead of killing the process.
 */
#ifndef RAFTSTEP_H
#define RAFTSTEP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RAFT_ABI_VERSION 6u
#define RAFT_MAX_REPLICAS 8u

/* Node.State (main.go:51-57). */
enum raft_role { RAFT_FOLLOWER = 0, RAFT_CANDIDATE = 1, RAFT_LEADER = 2 };

/* Per-group fault codes. The reference panics or blocks forever instead;
 * the engine freezes the group from that point on (no further state change). */
enum raft_fault {
  RAFT_F_NONE = 0,
  RAFT_F_PANIC_GETLOG = 1,        /* GetLog(i) out of range: main.go:142 -> 403-405 */
  RAFT_F_DEADLOCK_VRES = 2,       /* candidate answers a VoteRequest into its own VRes: main.go:242 */
  RAFT_F_DEADLOCK_LEADER_VREQ = 3,/* leader has no VReq case: main.go:308-332 */
  RAFT_F_RING_EVICTED = 4,        /* EXT: entry older than the ring depth K was needed */
  RAFT_F_OVERFLOW = 5             /* EXT: a term/index would leave int32 (Go int is 64-bit) */
};

/* REF = main.go bit for bit (the drop-in). RAFT = EXT mode with the
 * Raft-paper rules (votedFor, up-to-date check, truncate-on-conflict,
 * nextIndex backoff, majority commit with the current-term rule) on the same
 * tick model and layout, for churn workloads where REF faults (config C4). */
enum raft_semantics { RAFT_SEM_REF = 0, RAFT_SEM_RAFT = 1 };

/* Error codes (negative returns). */
#define RAFT_OK 0
#define RAFT_EINVAL (-22)
#define RAFT_ENOMEM (-12)
#define RAFT_ERANGE (-34)
#define RAFT_ETIMEDOUT (-110) /* a communicator did not complete in time (RAFTSTEP_COMM_TIMEOUT_S) */
#define RAFT_ENODEV (-19)
#define RAFT_EHIP (-1000)
#define RAFT_ERCCL (-2000)
#define RAFT_EINTERNAL (-3000)  /* an engine invariant failed its run-time check (a bug: report it) */

/* Statistics of one or more ticks (summed over groups, and over GPUs once a
 * communicator is attached). Index names: */
enum raft_stat {
  RAFT_STAT_COMMITTED = 0,      /* sum of leader CommitIndex advances (main.go:389) */
  RAFT_STAT_ELECTIONS_WON = 1,  /* candidate -> leader (main.go:273-282) */
  RAFT_STAT_TERM_BUMPS = 2,     /* election timeouts, Term++ (main.go:176, 250) */
  RAFT_STAT_AE_OK = 3,          /* AppendEntries answered Success:true */
  RAFT_STAT_AE_FAIL = 4,        /* AppendEntries answered false (or dropped, EXT) */
  RAFT_STAT_VOTES_GRANTED = 5,  /* VoteResponse vote:true */
  RAFT_STAT_FAULTS = 6,         /* groups that faulted during the tick(s) */
  RAFT_STAT_LEADER_GROUPS = 7,  /* groups with >=1 leader at the end of each tick (summed over ticks) */
  RAFT_NSTATS = 8
};
typedef struct raft_tick_stats { int64_t v[RAFT_NSTATS]; } raft_tick_stats;

/* Engine configuration. Zero-initialise, then set fields; see
 * raft_config_default(). Virtual time: one tick = tick_seconds virtual
 * seconds (the leader heartbeat period, main.go:394). */
typedef struct raft_config {
  uint32_t abi_version;        /* = RAFT_ABI_VERSION */
  uint32_t replicas;           /* R = len(Nodes), 1..8 (main.go:81 uses 3) */
  uint64_t groups;             /* independent Raft groups on this engine */
  uint64_t group_base;         /* global id of local group 0 (sharding across GPUs) */
  uint32_t ring_depth;         /* K: log entries kept per replica, power of two */
  uint32_t entries_per_tick;   /* E: client entries appended per client event (main.go:92) */
  uint32_t client_period;      /* ticks between client events; 0 = no client */
  uint32_t semantics;          /* enum raft_semantics */
  uint64_t seed;               /* trace seed (splitmix64 counter RNG) */
  int32_t tick_seconds;        /* 2 (main.go:394) */
  int32_t follower_timeout_min;   /* 10 s  (main.go:114: rand.Intn(20)+10) */
  int32_t follower_timeout_span;  /* 20    */
  int32_t candidate_timeout_min;  /* 10 s  (main.go:194: rand.Intn(4)+10) */
  int32_t candidate_timeout_span; /* 4     */
  uint32_t isolate_per_65536;  /* EXT: probability (x/65536) per 32-tick epoch that one replica is isolated */
  uint32_t isolate_min_ticks;  /* EXT: isolation length range, 1..32 */
  uint32_t isolate_max_ticks;
  int32_t device;              /* HIP device ordinal */
  uint32_t payload_crc;        /* EXT (config C5): stamp every entry with CRC32C(term||value), followers verify */
  uint32_t corrupt_per_65536;  /* EXT: probability that an AppendEntries' last entry arrives with a flipped bit */
  uint32_t isolate_leader;     /* EXT: 1 = an isolation window cuts off the group's leader at the window's first
                                  tick (the lowest-id Leader then; no leader: nobody), 0 = a hashed replica */
  uint32_t ticks_per_launch;   /* 1 (default; 0 reads as 1): one tick per kernel launch, every group's state read
                                  from and written back to HBM every tick (the metric's form).
                                  2..64: while the steady-state list skip holds (no isolation, no CRC), up to this
                                  many steady ticks run in one launch of the fused kernel (state kept in registers
                                  between them; results identical, not the §8(d) form) */
  uint32_t debug_flags;        /* RAFT_DEBUG_*; 0 in production */
  uint32_t client_source;      /* enum raft_client_source: where the client's values (main.go:92) come from */
  uint32_t reserved[2];        /* must be 0 */
} raft_config;

/* raft_config.client_source. The reference's client sends rand.Int() to
 * every node whose State is Leader (main.go:87-93 -> LogReq -> 327-329).
 *  RAFT_CLIENT_TRACE  (0): the values come from the seeded trace RNG on the
 *      device (splitmix64 keyed by seed, group, replica, tick, entry);
 *  RAFT_CLIENT_STAGED (1): the caller supplies them. Before raft_tick runs
 *      ticks [t0, t0+n) the caller stages n x E x G int64 values with
 *      raft_stage_values; every Leader of group g at tick t appends
 *      values[((t - t0) * E + e) * G + g] as its e-th entry of that tick (one
 *      client request per group and entry, sent to whichever replicas are
 *      leaders, like main.go:90-93). The engine never regenerates an entry in
 *      this mode: entries are read from the staged buffer when appended and
 *      from the rings afterwards. */
enum raft_client_source { RAFT_CLIENT_TRACE = 0, RAFT_CLIENT_STAGED = 1 };

/* raft_config.debug_flags */
#define RAFT_DEBUG_ALLOW_WRONG_RESULTS 1u  /* accept the timing-only environment knob RAFTSTEP_DIAG_LEAN, whose modes
                                              skip work and make results WRONG; without this flag
                                              raft_engine_create refuses it (RAFT_EINVAL) */

/* Canonical host view of engine state, group-major:
 *   per-replica arrays are indexed [g*R + r], match is [(g*R + leader)*R + peer],
 *   log arrays are [(g*R + r)*K + slot] where log index i (1-based) lives at
 *   slot (i-1) mod K and only i in (max(0,hwm-K), last] is meaningful (other
 *   slots read back as 0). match rows of replicas that are not leaders read
 *   back as 0. Any pointer may be NULL on store (field skipped). */
typedef struct raft_state_view {
  uint8_t* role;      /* Node.State (main.go:16) */
  uint8_t* voted;     /* REF: Node.Voted (main.go:20); RAFT: votedFor + 1 (0 = none) */
  int32_t* term;      /* Node.Term (main.go:19) */
  int32_t* last;      /* Node.LastApplied == len(Node.Log) (main.go:25, 148-149, 328-329) */
  int32_t* commit;    /* Node.CommitIndex (main.go:24) */
  int32_t* deadline;  /* election timer deadline, virtual seconds */
  int32_t* timeout;   /* current timer duration d, seconds (main.go:114, 194) */
  int32_t* match;     /* Node.MatchIndex (main.go:29); NextIndex == MatchIndex+1 (main.go:280-281, 376-377) */
  uint8_t* fault;     /* per group, enum raft_fault */
  int32_t* log_term;  /* Log.Term (main.go:47) */
  int64_t* log_value; /* Log.Value (main.go:48) */
  uint32_t* log_crc;  /* EXT: CRC32C of each ring entry (0 when payload_crc is off) */
  int32_t* next;      /* Node.NextIndex [(g*R + leader)*R + peer] (REF: match+1); 0 for non-leaders.
                         Optional on load: absent or 0 derives match+1 (REF ignores it) */
  int32_t* hwm;       /* [g*R + r] highest LastApplied ever (== last in REF); the ring holds (hwm-K, last].
                         Optional on load: absent or < last means last (REF ignores it) */
  uint8_t* iso_victim;/* per group, EXT leader-isolation mode: victims of the windows in flight, one nibble
                         per epoch parity (8 | replica, 0 = none). Optional on load (absent: 0) */
} raft_state_view;

typedef struct raft_engine raft_engine;

/* ---- lifecycle ---------------------------------------------------------- */
void raft_config_default(raft_config* cfg);
int raft_engine_create(const raft_config* cfg, raft_engine** out);
int raft_engine_destroy(raft_engine* e);
const char* raft_last_error(void);              /* thread-local message of the last failure */
int raft_engine_info(const raft_engine* e, raft_config* cfg_out, uint64_t* device_bytes);
/* Storage forms this engine uses (bit set = on; results are identical either
 * way): RAFT_FEATURE_SHARED_ENTRIES — the steady kernels store the entries
 * every replica of an in-step group holds alike once (shared ring, copied
 * back into the replica rings before any other reader); RAFT_FEATURE_
 * VIRTUAL_SUFFIXES — a cut-off leader's own entries are regenerated instead
 * of stored (RAFT leader isolation). */
#define RAFT_FEATURE_SHARED_ENTRIES 1u
#define RAFT_FEATURE_VIRTUAL_SUFFIXES 2u
int raft_engine_features(const raft_engine* e, uint32_t* flags);

/* NewNode x R for every group (main.go:59-76) followed by FollowerRun entry
 * (timer drawn, main.go:113-115) at virtual tick `tick0`. */
int raft_init_new_nodes(raft_engine* e, int64_t tick0);
/* Post-election state (KAT-1 generalised): replica `leader` (or a per-group
 * hashed replica when leader < 0) is Leader with Term 1, the others are
 * Followers with Term 1 and Voted, MatchIndex 0 / NextIndex 1, empty logs. */
int raft_init_steady(raft_engine* e, int32_t leader, int64_t tick0);

int raft_load_state(raft_engine* e, const raft_state_view* v);
int raft_store_state(raft_engine* e, raft_state_view* v);
/* The canonical view of groups [first_group, first_group + n_groups) only,
 * indexed by the local group (g - first_group) with the same per-group shapes
 * as raft_store_state; copies out only that slice of the device state, so a
 * slice of a multi-million-group engine can be compared with a CPU run of the
 * same groups (RAFT_ERANGE when the range leaves the engine). */
int raft_store_state_range(raft_engine* e, uint64_t first_group, uint64_t n_groups, raft_state_view* v);

/* ---- audit: digests, nodelog, checkpoints ---------------------------------
 * raft_state_digest: per-group 64-bit digest of the canonical view that
 * raft_store_state would return (splitmix64 chain keyed by the global group
 * id; words listed in oracle/raft_oracle.c oracle_state_digest), computed on
 * the device without copying the state out. `per_group` (u64[groups], may be
 * NULL) receives the digests, `total` (may be NULL) their wrapping sum, which
 * is independent of how groups are sharded over engines. */
int raft_state_digest(raft_engine* e, uint64_t* per_group, uint64_t* total);
/* nodelog (main.go:399-401) lines of every replica of one group:
 * "[Server<r>:<Term>:<CommitIndex>:<LastApplied>][<state>]\n". Returns the
 * number of bytes written (NUL-terminated when it fits) or a negative code;
 * RAFT_ERANGE if `cap` is too small. */
int raft_nodelog(raft_engine* e, uint64_t group, char* buf, size_t cap);
/* Checkpoint = the canonical view of every group plus the engine's config,
 * written to / read from a file (header + fields + CRC32C trailer). The
 * persistent Node fields of main.go:18-21 (Term, Voted, Log) and the volatile
 * ones (22-29) survive a save/load round trip bit for bit. Loading checks
 * replicas / groups / ring depth / semantics / payload_crc against the
 * engine's config (RAFT_EINVAL on mismatch, on a bad magic/version or CRC). */
int raft_checkpoint_save(raft_engine* e, const char* path);
int raft_checkpoint_load(raft_engine* e, const char* path);

/* ---- the tick (the metric path) -----------------------------------------
 * Advances every group by `nticks` ticks starting at virtual tick
 * `first_tick`. One tick per kernel launch (config.ticks_per_launch = 1, the
 * default; see there for the fused steady form); per tick and group, in order:
 *   1. client append to leaders (main.go:87-93 -> 327-329),
 *   2. replicas in ascending id: leader replication round + commit
 *      (main.go:332-391) / candidate vote round (main.go:253-284), every
 *      message delivered through the receiver's handler,
 *   3. election timers that expired, in (deadline, id) order, each followed
 *      at once by the new candidate's vote round (main.go:171-177, 248-251).
 * `out` (may be NULL) receives the stats summed over the ticks. */
int raft_tick(raft_engine* e, int64_t first_tick, uint32_t nticks, raft_tick_stats* out);
/* RAFT_CLIENT_STAGED engines: the client values of ticks [first_tick,
 * first_tick + nticks), laid out [nticks][E][G] int64 (E = entries_per_tick,
 * G = groups of this engine, indexed by the local group; the value stream of
 * main.go:92, one request per group, tick and entry, LogReq at main.go:327-329).
 * Copied into HBM (the host buffer is only borrowed for the call); replaces
 * whatever was staged before. raft_tick then accepts calls whose ticks lie
 * inside the staged range (RAFT_EINVAL otherwise). RAFT_EINVAL on a
 * RAFT_CLIENT_TRACE engine. */
int raft_stage_values(raft_engine* e, int64_t first_tick, uint32_t nticks, const int64_t* values);
/* Per-tick statistics of the last raft_tick call that asked for stats: record
 * t (0 <= t < nticks of that call) holds tick first_tick+t, summed over groups
 * and, with a communicator, over GPUs (the 64-B record the all-reduce carries). */
int raft_tick_records(raft_engine* e, uint32_t nticks, raft_tick_stats* per_tick);
int raft_sync(raft_engine* e);

/* ---- message-level handlers (drop-in for the select cases) --------------
 * Batched: element i is applied to group reqs[i].group; all groups of one
 * batch must be distinct (RAFT_EINVAL otherwise). `now_tick` is the virtual
 * time used for timer resets / redraws. */
typedef struct raft_log_entry { int64_t term; int64_t value; } raft_log_entry; /* Log (main.go:46-49) */

typedef struct raft_ae_req {     /* AppendEntriesRequest (main.go:289-296) */
  uint64_t group;
  uint32_t to;                   /* receiving replica */
  uint32_t leader_id;            /* LeaderId (routing only) */
  int64_t term;                  /* Term */
  int64_t prev_log_index;        /* PrevLogIndex */
  int64_t prev_log_term;         /* PrevLogTerm */
  int64_t leader_commit;         /* LeaderCommit */
  uint64_t entries_offset;       /* Logs = entries[entries_offset .. +n_entries) */
  uint64_t n_entries;
} raft_ae_req;
typedef struct raft_ae_resp {    /* AppendEntriesResponse (main.go:298-302) */
  int64_t term;
  int64_t match_index;
  int32_t success;
  int32_t fault;                 /* enum raft_fault raised while handling (0 = none) */
} raft_ae_resp;
/* FollowerRun case AEReq (main.go:121-156), CandidateRun case AEReq
 * (main.go:200-223), LeaderRun case AEReq (main.go:309-326), dispatched on
 * the receiver's State like Run (main.go:98-109). */
int raft_append_entries_batch(raft_engine* e, int64_t now_tick, const raft_ae_req* reqs, size_t n,
                              const raft_log_entry* entries, size_t n_entries_total, raft_ae_resp* out);

typedef struct raft_vote_req {   /* VoteRequest (main.go:182-187) */
  uint64_t group;
  uint32_t to;
  uint32_t candidate_id;         /* CandidateId (routing only) */
  int64_t term;
  int64_t last_log_index;        /* never read by the reference (main.go:185-186, 264) */
  int64_t last_log_term;
} raft_vote_req;
typedef struct raft_vote_resp {  /* VoteResponse (main.go:188-191) */
  int64_t term;
  int32_t vote_granted;
  int32_t fault;
} raft_vote_resp;
/* FollowerRun case VReq (main.go:157-170), CandidateRun case VReq
 * (main.go:224-246); a leader has no VReq case (main.go:308) -> fault. */
int raft_request_vote_batch(raft_engine* e, int64_t now_tick, const raft_vote_req* reqs, size_t n,
                            raft_vote_resp* out);

/* Whole-node steps, batched over distinct groups. LEADER_ROUND and
 * CANDIDATE_ROUND honour the config's EXT isolation windows at now_tick
 * (messages to or from an isolated replica are dropped), like raft_tick. */
enum raft_op_kind {
  RAFT_OP_CLIENT_APPEND = 1,   /* LeaderRun case LogReq (main.go:327-329); arg = Value */
  RAFT_OP_LEADER_ROUND = 2,    /* LeaderRun default: AE to each peer + commit (main.go:332-391) */
  RAFT_OP_CANDIDATE_ROUND = 3, /* CandidateRun default: vote round + tally (main.go:253-284) */
  RAFT_OP_TIMEOUT = 4,         /* timer.C: follower -> candidate / candidate Term++ (main.go:171-177, 248-251) */
  RAFT_OP_LEADER_COMMIT = 5    /* commit rule alone (main.go:381-391) */
};
typedef struct raft_group_op {
  uint64_t group;
  uint32_t replica;
  uint32_t kind;
  int64_t arg;
} raft_group_op;
typedef struct raft_op_result {
  int32_t status;   /* 0 applied; RAFT_EINVAL if the replica's State does not run this step */
  int32_t fault;    /* group fault code after the op */
  int64_t value;    /* CommitIndex after LEADER_ROUND/LEADER_COMMIT; 1 if elected by CANDIDATE_ROUND */
} raft_op_result;
int raft_group_ops_batch(raft_engine* e, int64_t now_tick, const raft_group_op* ops, size_t n,
                         raft_op_result* out);

/* ---- multi-GPU statistics (RCCL over xGMI) -------------------------------
 * Groups shard by id (config.group_base); the only collective is the sum of
 * tick statistics. raft_tick reduces per-tick records on the device (NSTAT
 * int64 = 64 B per tick) and all-reduces them: in a call that runs list or
 * general kernels, once per general-kernel window on a second HIP stream
 * (ordered by an event, overlapping the following ticks); the call's last sum,
 * and the only one of a steady call (list skipped), on the engine stream at
 * the end of the call. Rank 0 creates the id and distributes it out of band.
 * raft_comm_init and every wait on a call with a communicator are bounded by
 * RAFTSTEP_COMM_TIMEOUT_S seconds (default 300): a missing rank or ranks that
 * disagree end in RAFT_ETIMEDOUT with a message (an all-reduce timeout also
 * aborts the communicator and poisons the engine), never in a hang. */
int raft_comm_unique_id(uint8_t id_out[128]);
int raft_comm_init(raft_engine* e, int nranks, int rank, const uint8_t id[128]);
/* All-reduce `stats` (in/out) over the communicator (sum); no-op without one. */
int raft_comm_allreduce_stats(raft_engine* e, raft_tick_stats* stats);
/* Ranks of the attached communicator as RCCL reports them (ncclCommCount /
 * ncclCommUserRank; 1 / 0 without one) and the number of per-window stats
 * all-reduces raft_tick has issued on the engine's comm stream so far. */
int raft_comm_info(raft_engine* e, int32_t* nranks, int32_t* rank, uint64_t* allreduces);

/* ---- instrumentation -----------------------------------------------------
 * mode 1: the steady-state tick kernel is timed by events attached to its
 *         dispatches (hipExtLaunchKernel): in a call that runs the lean (or
 *         fused) kernel alone, one pair spanning the call's back-to-back
 *         launches (start on the first, stop on the last: the kernels run as
 *         in an unprofiled call); otherwise a pair on every dispatch
 *         (kernel-exact, ~5-9 us of wall time between launches);
 * mode 2: one event pair on the engine stream around all launches of each
 *         raft_tick call (no per-launch cost; includes the general kernel and
 *         launch gaps, so it upper-bounds the tick kernel's duration);
 * mode 3: as mode 1 for the second pass of the two-pass tick (the list
 *         kernel over the groups the lean steady-state kernel passed on);
 * mode 0: off. raft_profile_read() syncs and returns the summed milliseconds
 * and the number of tick launches covered. */
int raft_profile_enable(raft_engine* e, int mode);
int raft_profile_read(raft_engine* e, double* total_ms, uint64_t* launches);

/* ---- diagnostics: tick-class coverage ------------------------------------
 * raft_diag_enable(e, 1) zeroes and starts the device lane-class counters:
 * for every tick, the lanes (groups) of the steady-state (lean) kernel and of
 * the full fast-path body (the list kernel, or the one-pass kernel) that took
 * each class of tick. raft_diag_read copies out n <= RAFT_DIAG_COUNTERS
 * counters (indices below) and zeroes them. Counting costs one ballot and
 * atomic per wave and class; off by default. */
#define RAFT_DIAG_DEVICE_COUNTERS 64u
#define RAFT_DIAG_COUNTERS 72u
enum raft_diag_counter {
  /* lean kernel (first pass of the two-pass tick) */
  RAFT_DIAG_LEAN_LANES = 10,          /* groups looked at */
  RAFT_DIAG_LEAN_SKIPPED = 0,         /* deferred to the general kernel or frozen by a fault */
  RAFT_DIAG_LEAN_SSYNC = 18,          /* compressed steady ticks taken */
  RAFT_DIAG_LEAN_LXS = 19,            /* cut-off leader appending alone (LXS) taken */
  RAFT_DIAG_LEAN_THREE_SEG = 20,      /* ring segment switch while the previous segment stays live */
  RAFT_DIAG_LEAN_LXS_WHOLE_ROW = 21,  /* LXS ticks written as whole ring rows */
  RAFT_DIAG_LEAN_HWX = 22,            /* steady ticks of a group with a truncated log in step (HWX) */
  RAFT_DIAG_LEAN_PASSED = 23,         /* groups passed on to the list kernel */
  RAFT_DIAG_LEAN_FORCED = 24,         /* groups passed by raft_debug_force_pass */
  RAFT_DIAG_LEAN_SXS = 25,            /* new leader replicating while the stale one is cut off (SXS) taken */
  RAFT_DIAG_LEAN_SXS_STALE_IN_ROW = 26,/* ... with the stale leader's entry inside the common ring row */
  RAFT_DIAG_LEAN_SXS_VX = 27,         /* SXS ticks whose stale leader holds a virtual suffix (whole rows) */
  RAFT_DIAG_LIST_RETURN_VX = 28,      /* stale leaders' returns with a virtual suffix (no entry copy) */
  RAFT_DIAG_LIST_LXS_VX = 29,         /* LXS entered with a virtual suffix */
  RAFT_DIAG_LEAN_SH = 30,             /* steady ticks whose entries went to the shared ring (SH) */
  RAFT_DIAG_LIST_SH_COPIED = 31,      /* groups in shared form whose entries the list kernel copied back */
  RAFT_DIAG_LIST_SH_ENTRIES = 1,      /* ... the shared entries it copied */
  RAFT_DIAG_LIST_LAG_CATCHUP = 6,     /* REF + CRC: a follower that rejected a corrupted copy caught up (list kernel) */
  RAFT_DIAG_LIST_SH_KEPT = 7,         /* REF + CRC: listed groups that kept their shared form (no copy-back) */
  RAFT_DIAG_LEAN_SWITCH = 5,          /* ring segment switches */
  /* full fast-path body (list kernel / one-pass kernel): 32 + bit */
  RAFT_DIAG_LIST_LANES = 42,          /* groups looked at */
  RAFT_DIAG_LIST_DEFERRED = 33,       /* deferred to the general kernel this tick */
  RAFT_DIAG_LIST_ISOLATION = 34,      /* an isolation window over the group */
  RAFT_DIAG_LIST_SWITCH = 37,         /* ring segment switches */
  RAFT_DIAG_LIST_QUIET = 48,          /* quiet leaderless ticks */
  RAFT_DIAG_LIST_ISOLATED_LEADER = 49,/* cut-off leader appending alone */
  RAFT_DIAG_LIST_SSYNC = 50,          /* ticks ending in the compressed steady state */
  RAFT_DIAG_LIST_ELECTION = 51,       /* a follower's election while the leader is cut off */
  RAFT_DIAG_LIST_FIRST_ROUND = 52,    /* a new leader's first round (fresh rows) */
  RAFT_DIAG_LIST_RETURN = 53,         /* the stale leader's return (step-down + catch-up) */
  RAFT_DIAG_LIST_RETURN_TRUNC = 54,   /* ... with its log truncated */
  RAFT_DIAG_LIST_STALE = 55,          /* new leader replicating while the stale one is cut off */
  RAFT_DIAG_LIST_HWX = 56,            /* truncated logs in step */
  RAFT_DIAG_LIST_THREE_SEG = 57,      /* ring segment switch while the previous segment stays live */
  RAFT_DIAG_LIST_ISOLATED_REPLICA = 58,/* one isolated follower / candidate */
  RAFT_DIAG_LIST_TIMER_FIRE = 59,     /* the isolated replica's election timer fired */
  RAFT_DIAG_LIST_WINDOW_START = 60,   /* a leader-isolation window decided on the fast path */
  RAFT_DIAG_LIST_SXS_MATERIALISED = 61,/* SXS groups taken by the full body (explicit form rebuilt) */
  RAFT_DIAG_LIST_SXS_ENTERED = 62,    /* ticks ending in the SXS compressed form */
  RAFT_DIAG_LIST_STALE_MOVED = 63,    /* segment switch that moved a stale leader's entries (placement only) */
  /* host counters since the last read */
  RAFT_DIAG_TICKS = 64,
  RAFT_DIAG_TICKS_LIST_SKIPPED = 65,  /* ticks run by the lean kernel alone (steady-state list skip) */
  RAFT_DIAG_GENERAL_LAUNCHES = 66
};
int raft_diag_enable(raft_engine* e, int on);
int raft_diag_read(raft_engine* e, uint64_t* counters, uint32_t n);
/* Test knob: the lean kernel passes `group` (< 0: none) to the list kernel at
 * every tick instead of taking it. Results are unchanged while the list kernel
 * runs; in a list-skipping call the group's tick is lost, which the engine
 * detects (RAFT_EINTERNAL, engine poisoned until its state is replaced). */
int raft_debug_force_pass(raft_engine* e, int64_t group);
/* Debugging: the raw per-group words of one group (gmeta, giso, hb, the
 * compressed record gss[4], glx[2], grot, grota, gsb, grotb, gsb2). */
#define RAFT_DEBUG_GROUP_WORDS 14u
int raft_debug_group_words(raft_engine* e, uint64_t group, int32_t* out, uint32_t n);
/* Timing diagnostics (results WRONG while non-zero): replaces the engine's
 * kernel diagnostic mode (RAFTSTEP_DIAG_LEAN's bits) from the next call on,
 * e.g. after a settle; RAFT_EINVAL unless the engine was created with
 * debug_flags RAFT_DEBUG_ALLOW_WRONG_RESULTS. 0 restores exact ticks (the
 * state is then whatever the diagnostic ticks left). */
int raft_debug_diag_mode(raft_engine* e, uint32_t mode);
/* Measurement: the steady lean kernel's byte mix and access shape (per
 * element 20 B read in one round trip, 20 B of record + heartbeat and R ring
 * entries of 12 B written as whole rows; 20 + 20 + 12 R bytes) over `elems`
 * fresh elements on `device`, no Raft state: one untimed pass, then `reps`
 * back-to-back passes between HIP events. Returns the mean pass time and the
 * bytes per pass (bench.py: the device's sustained rate for that pattern). */
#define RAFT_PROBE_PLAIN_RING 1u    /* plain (write-back) ring stores instead of non-temporal ones */
#define RAFT_PROBE_NT_RECORD 2u     /* non-temporal record / heartbeat stores */
#define RAFT_PROBE_NO_HEARTBEAT 4u  /* no heartbeat store (a group in shared form): 16 B written + ring */
int raft_stream_probe(int device, uint32_t replicas, uint64_t elems, uint32_t reps, uint32_t flags,
                      double* us_per_pass, double* bytes_per_pass);

#ifdef __cplusplus
}
#endif
#endif /* RAFTSTEP_H */
