// raftnode.hpp — C++ host-side mirror of eastwd/raft-sample's Go node API,
// implemented over the C-ABI (include/raftstep.h). Go is not available in
// this image, so this is the host layer above the boundary in the
// reference's compiled-language spirit: the same type names, fields and
// handler entry points as main.go, with a Node being a (group, replica) view
// onto a GPU engine. Nothing here computes Raft state.
//
//   main.go                                   here
//   type Node struct (14-39)                  raft::Node (view) + raft::Engine (storage)
//   type Log / NewLogRequest (42-49)          raft::Log / raft::NewLogRequest
//   type State (51-57)                        raft::State
//   VoteRequest/VoteResponse (182-191)        raft::VoteRequest / raft::VoteResponse
//   AppendEntriesRequest/Response (289-302)   raft::AppendEntriesRequest / ...Response
//   FollowerRun/CandidateRun/LeaderRun cases  Node::OnAppendEntries / OnRequestVote / OnNewLog
//   LeaderRun default (332-391)               Node::LeaderRound
//   CandidateRun default (253-284)            Node::CandidateRound
//   timer.C (171-177, 248-251)                Node::OnTimeout
//   nodelog (399-401)                         Node::nodelog
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/raftstep.h"

namespace raft {

enum class State : uint8_t { Follower = RAFT_FOLLOWER, Candidate = RAFT_CANDIDATE, Leader = RAFT_LEADER };
inline const char* to_string(State s) {
  return s == State::Follower ? "follower" : s == State::Candidate ? "candidate" : "leader";
}

struct Log { int64_t Term = 0; int64_t Value = 0; };
struct NewLogRequest { int64_t Value = 0; };
struct VoteRequest { int64_t Term = 0; uint32_t CandidateId = 0; int64_t LastLogIndex = 0; int64_t LastLogTerm = 0; };
struct VoteResponse { int64_t Term = 0; bool vote = false; int fault = 0; };
struct AppendEntriesRequest {
  int64_t Term = 0;
  uint32_t LeaderId = 0;
  std::vector<Log> Logs;
  int64_t LeaderCommit = 0, PrevLogIndex = 0, PrevLogTerm = 0;
};
struct AppendEntriesResponse { int64_t Term = 0; bool Success = false; int64_t MatchIndex = 0; int fault = 0; };

class Error : public std::runtime_error {
 public:
  Error(int code, const std::string& what) : std::runtime_error(what), code(code) {}
  int code;
};
inline void check(int rc, const char* where) {
  if (rc != 0) throw Error(rc, std::string(where) + ": " + raft_last_error());
}

// Owns one raft_engine (one GPU, many groups).
class Engine {
 public:
  explicit Engine(const raft_config& cfg) : cfg_(cfg) { check(raft_engine_create(&cfg_, &h_), "raft_engine_create"); }
  ~Engine() { if (h_) raft_engine_destroy(h_); }
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;
  raft_engine* handle() const { return h_; }
  const raft_config& config() const { return cfg_; }
  void NewNodes(int64_t tick0) { check(raft_init_new_nodes(h_, tick0), "raft_init_new_nodes"); }
  raft_tick_stats Tick(int64_t first, uint32_t n) {
    raft_tick_stats s{};
    check(raft_tick(h_, first, n, &s), "raft_tick");
    return s;
  }

  // Snapshot of every group's state (canonical group-major arrays).
  struct Snapshot {
    uint32_t R = 0, K = 0;
    std::vector<uint8_t> role, voted, fault;
    std::vector<int32_t> term, last, commit, deadline, timeout, match, log_term;
    std::vector<int64_t> log_value;
    std::vector<uint32_t> log_crc;
  };
  Snapshot Store() const {
    Snapshot s;
    const uint64_t G = cfg_.groups, R = cfg_.replicas, K = cfg_.ring_depth;
    s.R = uint32_t(R); s.K = uint32_t(K);
    s.role.resize(G * R); s.voted.resize(G * R); s.fault.resize(G);
    s.term.resize(G * R); s.last.resize(G * R); s.commit.resize(G * R); s.deadline.resize(G * R);
    s.timeout.resize(G * R); s.match.resize(G * R * R); s.log_term.resize(G * R * K); s.log_value.resize(G * R * K);
    s.log_crc.resize(G * R * K);
    raft_state_view v{s.role.data(), s.voted.data(), s.term.data(), s.last.data(), s.commit.data(),
                      s.deadline.data(), s.timeout.data(), s.match.data(), s.fault.data(),
                      s.log_term.data(), s.log_value.data(), s.log_crc.data(), nullptr, nullptr, nullptr};
    check(raft_store_state(h_, &v), "raft_store_state");
    return s;
  }

 private:
  raft_config cfg_;
  raft_engine* h_ = nullptr;
};

// A Raft node: replica `replica` of group `group` on an engine. The handler
// methods are the bodies of main.go's select cases, dispatched on the node's
// current State exactly like Run (main.go:98-109).
class Node {
 public:
  Node(Engine& e, uint64_t group, uint32_t replica, std::string id)
      : Id(std::move(id)), e_(&e), group_(group), replica_(replica) {}

  std::string Id;
  uint32_t replica() const { return replica_; }
  uint64_t group() const { return group_; }

  // case r := <-n.AEReq (main.go:121-156, 200-223, 309-326)
  AppendEntriesResponse OnAppendEntries(int64_t now_tick, const AppendEntriesRequest& r) {
    raft_ae_req q{};
    q.group = group_; q.to = replica_; q.leader_id = r.LeaderId; q.term = r.Term;
    q.prev_log_index = r.PrevLogIndex; q.prev_log_term = r.PrevLogTerm; q.leader_commit = r.LeaderCommit;
    q.entries_offset = 0; q.n_entries = r.Logs.size();
    std::vector<raft_log_entry> ents(r.Logs.size());
    for (size_t i = 0; i < r.Logs.size(); ++i) ents[i] = raft_log_entry{r.Logs[i].Term, r.Logs[i].Value};
    raft_ae_resp out{};
    check(raft_append_entries_batch(e_->handle(), now_tick, &q, 1, ents.data(), ents.size(), &out),
          "raft_append_entries_batch");
    return AppendEntriesResponse{out.term, out.success != 0, out.match_index, out.fault};
  }
  // case r := <-n.VReq (main.go:157-170, 224-246)
  VoteResponse OnRequestVote(int64_t now_tick, const VoteRequest& r) {
    raft_vote_req q{};
    q.group = group_; q.to = replica_; q.candidate_id = r.CandidateId; q.term = r.Term;
    q.last_log_index = r.LastLogIndex; q.last_log_term = r.LastLogTerm;
    raft_vote_resp out{};
    check(raft_request_vote_batch(e_->handle(), now_tick, &q, 1, &out), "raft_request_vote_batch");
    return VoteResponse{out.term, out.vote_granted != 0, out.fault};
  }
  // case req := <-n.LogReq (main.go:327-329); false if this node is not the leader
  bool OnNewLog(int64_t now_tick, const NewLogRequest& req) { return op(now_tick, RAFT_OP_CLIENT_APPEND, req.Value).status == 0; }
  // LeaderRun default branch (main.go:332-391); returns CommitIndex
  int64_t LeaderRound(int64_t now_tick) { return op(now_tick, RAFT_OP_LEADER_ROUND, 0).value; }
  // CandidateRun default branch (main.go:253-284); returns true if elected
  bool CandidateRound(int64_t now_tick) { return op(now_tick, RAFT_OP_CANDIDATE_ROUND, 0).value != 0; }
  // <-timer.C (main.go:171-177, 248-251)
  void OnTimeout(int64_t now_tick) { op(now_tick, RAFT_OP_TIMEOUT, 0); }

  // nodelog (main.go:399-401) from a snapshot
  std::string nodelog(const Engine::Snapshot& s, const std::string& message) const {
    const uint64_t i = group_ * s.R + replica_;
    return "[" + Id + ":" + std::to_string(s.term[i]) + ":" + std::to_string(s.commit[i]) + ":" +
           std::to_string(s.last[i]) + "][" + to_string(State(s.role[i])) + "]" + message;
  }

 private:
  raft_op_result op(int64_t now_tick, uint32_t kind, int64_t arg) {
    raft_group_op q{group_, replica_, kind, arg};
    raft_op_result out{};
    check(raft_group_ops_batch(e_->handle(), now_tick, &q, 1, &out), "raft_group_ops_batch");
    return out;
  }
  Engine* e_;
  uint64_t group_;
  uint32_t replica_;
};

}  // namespace raft
