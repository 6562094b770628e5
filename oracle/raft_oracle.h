/*
 * raft_oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the
 * reference's Raft handlers (eastwd/raft-sample main.go), used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
 * The product (libraftstep.so) never links, loads or calls this code.
 *
 * PARITY UNPINNED by reference outputs: the reference is Go-only, no Go
 * toolchain exists in the build container or on the GPU box (SURVEY.md
 * §8(c)), and the reference ships no tests, fixtures or golden vectors. The
 * oracle is instead pinned by the hand-derived known-answer tests of
 * SURVEY.md Appendix B (tests/kat_cases.py via tests/test_oracle_kat.py),
 * each derived from the main.go text; tests/golden/ freezes the trace
 * definition (RNG vectors, oracle-generated traces).
 *
 * State is array-of-structs, one group at a time, logs are growable
 * arrays like Go slices (main.go:148, 328) with int64 terms/indices like
 * Go's int; the engine's int32 range is enforced with RAFT_F_OVERFLOW at
 * the same points so that both agree.
 */
#ifndef RAFT_ORACLE_H
#define RAFT_ORACLE_H
#include "../include/raftstep.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle oracle;

oracle* oracle_create(const raft_config* cfg);
void oracle_destroy(oracle* o);
void oracle_init_new_nodes(oracle* o, int64_t tick0);
void oracle_init_steady(oracle* o, int32_t leader, int64_t tick0);
int oracle_load_state(oracle* o, const raft_state_view* v);
void oracle_store_state(const oracle* o, raft_state_view* v);
/* Runs nticks ticks; groups are split into nthreads contiguous ranges, each
 * run by its own pthread through all ticks (groups are independent). */
void oracle_tick(oracle* o, int64_t first_tick, uint32_t nticks, int nthreads, raft_tick_stats* out);
/* RAFT_CLIENT_STAGED: client values of ticks [first_tick, +nticks), [nticks][E][G]
 * over the oracle's groups (raft_stage_values' layout); 0 or -22. */
int oracle_stage_values(oracle* o, int64_t first_tick, uint32_t nticks, const int64_t* values);
int oracle_append_entries(oracle* o, int64_t now_tick, const raft_ae_req* reqs, size_t n,
                          const raft_log_entry* entries, raft_ae_resp* out);
int oracle_request_vote(oracle* o, int64_t now_tick, const raft_vote_req* reqs, size_t n,
                        raft_vote_resp* out);
int oracle_group_ops(oracle* o, int64_t now_tick, const raft_group_op* ops, size_t n,
                     raft_op_result* out);
/* The trace RNG (for golden-vector tests). */
uint64_t oracle_rng(uint64_t seed, uint64_t gid, uint32_t replica, uint32_t stream, uint64_t tick);
uint64_t oracle_client_value(uint64_t seed, uint64_t gid, uint32_t replica, uint64_t tick, uint32_t e);
int32_t oracle_timer_draw(const raft_config* cfg, uint64_t gid, uint32_t replica, int role, uint64_t tick);
int oracle_isolated(const raft_config* cfg, uint64_t gid, uint32_t replica, int64_t tick);
/* Leader replica of raft_init_steady (leader < 0: hashed per group). */
uint32_t oracle_steady_leader(const raft_config* cfg, uint64_t gid, int32_t leader);
/* EXT CRC32C (Castagnoli) and the entry stamp CRC32C(term_le32 || value_le64). */
uint32_t oracle_crc32c(const uint8_t* p, size_t n);
uint32_t oracle_entry_crc(int64_t term, int64_t value);
int oracle_corrupted(const raft_config* cfg, uint64_t gid, uint32_t replica, int64_t tick);
/* State digest, same definition as raft_state_digest (per group + wrapping sum). */
void oracle_state_digest(const oracle* o, uint64_t* per_group, uint64_t* total);
/* nodelog-format dump of one group (main.go:399-401), for debugging. */
int oracle_nodelog(const oracle* o, uint64_t group, char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
