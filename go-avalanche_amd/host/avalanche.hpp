// avalanche.hpp — C++ host mirror of go-avalanche's Processor API, running on
// the MI355X engine behind the C ABI (include/avhip.h).
//
// The reference is Go (package avalanche); no Go toolchain exists in this
// image, so the host side above the C ABI is C++ with the same names,
// argument meaning and error behaviour:
//   Processor::AddTargetToReconcile  processor.go:45-58   -> av_add_targets
//   Processor::RegisterVotes         processor.go:61-122  -> av_register_votes
//   Processor::IsAccepted            processor.go:125-130 -> av_is_accepted
//   Processor::GetConfidence         processor.go:133-140 -> av_get_confidence (throws where Go panics)
//   Processor::GetInvsForNextPoll    processor.go:144-170 -> av_get_invs
//   Processor::GetRound              processor.go:40-42   -> av_get_round (per-node field, av_set_round)
// A Processor is a view (engine, node) over one batched Engine, so N
// Processors share one HBM-resident state and one batched round driver
// (Network::RunRounds = the example's poll loop for every node at once).
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "avhip.h"

namespace avalanche {
namespace gpu {

// avalanche.go:8-22
constexpr int kFinalizationScore = AV_FINALIZATION_SCORE;
constexpr int kMaxElementPoll = AV_MAX_ELEMENT_POLL;

using NodeID = int64_t;       // avalanche.go:25
constexpr NodeID NoNode = -1; // avalanche.go:28
using Hash = int64_t;         // avalanche.go:71 (Go int, 64-bit)

// avalanche.go:42-56
enum class Status : int { Invalid = AV_STATUS_INVALID, Rejected = AV_STATUS_REJECTED,
                          Accepted = AV_STATUS_ACCEPTED, Finalized = AV_STATUS_FINALIZED };

struct StatusUpdate {  // avalanche.go:59-62
  Hash hash;
  Status status;
  bool operator==(const StatusUpdate& o) const { return hash == o.hash && status == o.status; }
};

struct Inv {  // avalanche.go:65-68
  std::string target_type;
  Hash target_hash;
};

// avalanche.go:74-91
class Target {
 public:
  virtual ~Target() = default;
  virtual Hash GetHash() const = 0;
  virtual std::string Type() const = 0;
  virtual bool IsAccepted() const = 0;
  virtual int64_t Score() const = 0;
  virtual bool IsValid() const = 0;
};

// vote.go:4-22
class Vote {
 public:
  Vote(uint32_t err, Hash hash) : err_(err), hash_(hash) {}
  Hash GetHash() const { return hash_; }
  uint32_t GetError() const { return err_; }

 private:
  uint32_t err_;
  Hash hash_;
};
inline Vote NewVote(uint32_t err, Hash hash) { return Vote(err, hash); }

// response.go:5-25
class Response {
 public:
  Response() = default;
  Response(int64_t round, uint32_t cooldown, std::vector<Vote> votes)
      : round_(round), cooldown_(cooldown), votes_(std::move(votes)) {}
  const std::vector<Vote>& GetVotes() const { return votes_; }
  int64_t GetRound() const { return round_; }
  uint32_t GetCooldown() const { return cooldown_; }

 private:
  int64_t round_ = 0;
  uint32_t cooldown_ = 0;
  std::vector<Vote> votes_;
};
inline Response NewResponse(int64_t round, uint32_t cooldown, std::vector<Vote> votes) {
  return Response(round, cooldown, std::move(votes));
}

// net.go:11-31
class Connman {
 public:
  void AddNode(NodeID id);
  std::vector<NodeID> NodesIDs() const;

 private:
  std::vector<NodeID> nodes_;
};

class Error : public std::runtime_error {
 public:
  Error(int code, const std::string& msg) : std::runtime_error(msg), code(code) {}
  int code;
};

// Thrown where the reference panics (processor.go:136).
class VoteRecordNotFound : public Error {
 public:
  VoteRecordNotFound() : Error(AV_ERR_NOT_FOUND, "VoteRecord not found") {}
};

struct EngineOptions {
  int64_t n_nodes = 2;
  int64_t n_targets = 1024;  // hash catalog capacity (target slots)
  int32_t k = 8;
  uint64_t seed = 0xA7A1A9C4ull;
  int32_t peer_mode = AV_PEERS_RANDOM;
  uint32_t byz_threshold = 0;
  int32_t device = 0;
};

// One HBM-resident network of VoteRecords + the Hash -> target-slot catalog.
class Engine {
 public:
  explicit Engine(const EngineOptions& opt);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  av_engine* handle() const { return h_; }
  const EngineOptions& options() const { return opt_; }
  // slot of a hash, or -1; Intern assigns a slot on first use (-1 if full)
  int64_t Find(Hash h) const;
  int64_t Intern(const Target& t);
  Hash HashOf(int64_t slot) const { return hashes_[slot]; }
  const std::string& TypeOf(int64_t slot) const { return types_[slot]; }
  // Push Target::IsValid() of every catalogued target whose value changed
  // (isWorthyPolling is evaluated dynamically: processor.go:185-187).
  void SyncValidity();
  // Batched rounds for every node (the hot path).
  void RunRounds(int32_t rounds);
  int64_t Round() const;
  std::vector<uint64_t> FetchUpdates();
  // One node's StatusUpdates of one round, in the reference's append order (processor.go:94,111).
  using Deliver = std::function<void(int64_t round, NodeID node, const std::vector<StatusUpdate>& updates)>;
  // `rounds` batched rounds, every round's StatusUpdates handed to deliver node by node: round r + 1
  // computes while round r's compact stream is copied (av_fetch_compact_async / _wait) and decoded.
  void Rounds(int32_t rounds, const Deliver& deliver);
  // Walk a compact StatusUpdate stream (include/avhip.h av_compact_header) in place: Hash through
  // the catalog (a slot never interned is its own Hash).
  void DecodeCompact(const void* stream, int64_t bytes, const Deliver& deliver) const;

 private:
  EngineOptions opt_;
  av_engine* h_ = nullptr;
  std::unordered_map<Hash, int64_t> slot_of_;
  std::vector<Hash> hashes_;
  std::vector<std::string> types_;
  std::vector<const Target*> targets_;
  std::vector<int8_t> valid_;
};

// processor.go:12-25 — one node's Processor, a view over the shared Engine.
class Processor {
 public:
  Processor(std::shared_ptr<Engine> engine, NodeID node, Connman* connman = nullptr);

  int64_t GetRound() const;                                                              // :40-42
  // the reference test's `p.round++` (avalanche_test.go:302): Processor.round
  // is a field only its owner changes
  void SetRound(int64_t round);
  bool AddTargetToReconcile(const Target& t);                                            // :45-58
  bool RegisterVotes(NodeID id, const Response& resp, std::vector<StatusUpdate>* updates);  // :61-122
  bool IsAccepted(const Target& t) const;                                                // :125-130
  uint16_t GetConfidence(const Target& t) const;                                         // :133-140
  std::vector<Inv> GetInvsForNextPoll() const;                                           // :144-170
  NodeID getSuitableNodeToQuery() const;                                                 // :173-182

 private:
  std::shared_ptr<Engine> engine_;
  NodeID node_;
  Connman* connman_;
};

}  // namespace gpu
}  // namespace avalanche
