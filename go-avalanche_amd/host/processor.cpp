// processor.cpp — C++ mirror of go-avalanche's Processor over the C ABI.
#include <algorithm>
#include <cstring>

#include "avalanche.hpp"

namespace avalanche {
namespace gpu {
namespace {

void check(int rc) {
  if (rc == AV_OK) return;
  if (rc == AV_ERR_NOT_FOUND) throw VoteRecordNotFound();
  throw Error(rc, std::string(av_strerror(rc)) + ": " + av_last_error());
}

}  // namespace

void Connman::AddNode(NodeID id) {
  if (std::find(nodes_.begin(), nodes_.end(), id) == nodes_.end()) nodes_.push_back(id);
}

std::vector<NodeID> Connman::NodesIDs() const { return nodes_; }

Engine::Engine(const EngineOptions& opt) : opt_(opt) {
  av_config c;
  av_config_init(&c);
  c.n_nodes = opt.n_nodes;
  c.n_targets = opt.n_targets;
  c.k = opt.k;
  c.seed = opt.seed;
  c.peer_mode = opt.peer_mode;
  c.byz_threshold = opt.byz_threshold;
  c.device = opt.device;
  check(av_create(&c, &h_));
}

Engine::~Engine() {
  if (h_) av_destroy(h_);
}

int64_t Engine::Find(Hash h) const {
  auto it = slot_of_.find(h);
  return it == slot_of_.end() ? -1 : it->second;
}

int64_t Engine::Intern(const Target& t) {
  const Hash h = t.GetHash();
  int64_t s = Find(h);
  if (s >= 0) {
    targets_[s] = &t;  // the latest Target object answers IsValid()
    return s;
  }
  if ((int64_t)hashes_.size() >= opt_.n_targets) return -1;
  s = (int64_t)hashes_.size();
  slot_of_[h] = s;
  hashes_.push_back(h);
  types_.push_back(t.Type());
  targets_.push_back(&t);
  valid_.push_back(1);  // engine slots start valid
  return s;
}

void Engine::SyncValidity() {
  for (size_t s = 0; s < targets_.size(); ++s) {
    const int8_t v = targets_[s]->IsValid() ? 1 : 0;
    if (v != valid_[s]) {
      check(av_set_valid(h_, (int64_t)s, v));
      valid_[s] = v;
    }
  }
}

void Engine::RunRounds(int32_t rounds) {
  SyncValidity();
  check(av_run_rounds(h_, rounds));
}

int64_t Engine::Round() const {
  int64_t r = 0;
  check(av_round_index(h_, &r));
  return r;
}

std::vector<uint64_t> Engine::FetchUpdates() {
  int64_t n = 0;
  check(av_updates_count(h_, &n));
  std::vector<uint64_t> out((size_t)std::max<int64_t>(n, 1));
  check(av_fetch_updates(h_, out.data(), (int64_t)out.size(), &n));
  out.resize((size_t)n);
  return out;
}

void Engine::Rounds(int32_t rounds, const Deliver& deliver) {
  SyncValidity();
  std::vector<int64_t> pend;
  auto drain = [&](int64_t t) {
    const void* s = nullptr;
    int64_t n = 0;
    check(av_fetch_compact_wait(h_, t, &s, &n));
    DecodeCompact(s, n, deliver);
  };
  for (int32_t r = 0; r < rounds; ++r) {
    check(av_run_rounds(h_, 1));
    int64_t t = 0;
    check(av_fetch_compact_async(h_, &t));  // waits for the round, encodes, starts the copy
    pend.push_back(t);
    if (pend.size() >= 2) {  // the previous round's stream landed while this round ran
      drain(pend.front());
      pend.erase(pend.begin());
    }
  }
  for (int64_t t : pend) drain(t);
}

void Engine::DecodeCompact(const void* stream, int64_t bytes, const Deliver& deliver) const {
  av_compact_header h;
  if (bytes < (int64_t)sizeof(h)) throw Error(AV_ERR_INVALID_ARG, "compact stream shorter than its header");
  std::memcpy(&h, stream, sizeof(h));
  if (h.magic != AV_COMPACT_MAGIC || h.bytes != bytes) throw Error(AV_ERR_INVALID_ARG, "not a compact stream");
  const auto* base = static_cast<const uint8_t*>(stream);
  const uint64_t n_idx = (uint64_t)h.n_rounds * (uint64_t)h.chunks + 1;
  const auto* idx = reinterpret_cast<const uint64_t*>(base + sizeof(h));
  const uint8_t* g = base + sizeof(h) + n_idx * 16;
  const uint32_t tb = (uint32_t)h.target_bits, cw = (uint32_t)h.code_bytes, tmask = (1u << tb) - 1u;
  std::vector<StatusUpdate> ups;
  for (uint64_t j = 0; j + 1 < n_idx; ++j) {
    const int64_t round = h.log_base + (int64_t)(j / (uint64_t)h.chunks);
    for (uint64_t at = idx[2 * j]; at < idx[2 * j + 2];) {
      uint32_t node = 0, cnt = 0;
      std::memcpy(&node, g + at, 4);
      std::memcpy(&cnt, g + at + 4, 4);
      ups.resize(cnt);
      for (uint32_t i = 0; i < cnt; ++i) {
        uint32_t code = 0;
        std::memcpy(&code, g + at + 8 + (size_t)i * cw, cw);  // little-endian 2- or 4-byte code
        const int64_t slot = h.target_base + (int64_t)((code >> 2) & tmask);
        ups[i].hash = slot < (int64_t)hashes_.size() ? hashes_[(size_t)slot] : (Hash)slot;
        ups[i].status = (Status)(code & 3u);
      }
      deliver(round, (NodeID)node, ups);
      at += 8 + (((uint64_t)cnt * cw + 3) & ~3ull);
    }
  }
}

Processor::Processor(std::shared_ptr<Engine> engine, NodeID node, Connman* connman)
    : engine_(std::move(engine)), node_(node), connman_(connman) {}

int64_t Processor::GetRound() const {
  int64_t r = 0;
  check(av_get_round(engine_->handle(), node_, &r));
  return r;
}

void Processor::SetRound(int64_t round) { check(av_set_round(engine_->handle(), node_, round)); }

bool Processor::AddTargetToReconcile(const Target& t) {
  if (!t.IsValid()) return false;  // processor.go:46-48
  const int64_t s = engine_->Intern(t);
  if (s < 0) return false;  // catalog full: no slot for a new hash
  engine_->SyncValidity();
  const uint8_t acc = t.IsAccepted() ? 1 : 0;
  uint8_t added = 0;
  check(av_add_targets(engine_->handle(), node_, &s, &acc, 1, &added));
  return added != 0;
}

bool Processor::RegisterVotes(NodeID /*id*/, const Response& resp, std::vector<StatusUpdate>* updates) {
  // validation against outstanding queries is disabled in the reference
  // (`if false`, processor.go:63-90), so RegisterVotes always returns true.
  engine_->SyncValidity();
  const auto& votes = resp.GetVotes();
  std::vector<int64_t> slots(votes.size());
  std::vector<uint32_t> errs(votes.size());
  for (size_t i = 0; i < votes.size(); ++i) {
    slots[i] = engine_->Find(votes[i].GetHash());  // unknown hash -> skipped (:95-99)
    errs[i] = votes[i].GetError();
  }
  std::vector<int32_t> status(votes.size(), -1);
  check(av_register_votes(engine_->handle(), node_, slots.data(), errs.data(), (int64_t)votes.size(),
                          status.data()));
  for (size_t i = 0; i < votes.size(); ++i)
    if (status[i] >= 0) updates->push_back({votes[i].GetHash(), static_cast<Status>(status[i])});
  return true;
}

bool Processor::IsAccepted(const Target& t) const {
  const int64_t s = engine_->Find(t.GetHash());
  if (s < 0) return false;
  int32_t out = 0;
  check(av_is_accepted(engine_->handle(), node_, s, &out));
  return out != 0;
}

uint16_t Processor::GetConfidence(const Target& t) const {
  const int64_t s = engine_->Find(t.GetHash());
  if (s < 0) throw VoteRecordNotFound();
  uint16_t out = 0;
  check(av_get_confidence(engine_->handle(), node_, s, &out));
  return out;
}

std::vector<Inv> Processor::GetInvsForNextPoll() const {
  engine_->SyncValidity();
  std::vector<int64_t> slots(kMaxElementPoll);
  int64_t n = 0;
  check(av_get_invs(engine_->handle(), node_, slots.data(), (int64_t)slots.size(), &n));
  std::vector<Inv> invs;
  invs.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i) invs.push_back({engine_->TypeOf(slots[i]), engine_->HashOf(slots[i])});
  return invs;
}

NodeID Processor::getSuitableNodeToQuery() const {
  if (!connman_) return NoNode;
  auto ids = connman_->NodesIDs();
  if (ids.empty()) return NoNode;
  return *std::min_element(ids.begin(), ids.end());  // lowest id after sort (processor.go:173-182)
}

}  // namespace gpu
}  // namespace avalanche
