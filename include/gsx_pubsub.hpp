// gsx_pubsub.hpp — host-side mirror of the reference's peer-scoring interface
// (package pubsub: score.go, score_params.go) over the C ABI of gsx.h.
//
// The reference is Go and no Go toolchain exists in this image, so the host
// side above the C ABI is this header-only C++ layer.  Names, argument
// meaning and error behaviour follow the reference:
//   PeerScoreParams / TopicScoreParams / PeerScoreThresholds  score_params.go:12-148
//   validate()                                                  score_params.go:34-268
//   ScoreParameterDecay[WithBase]                               score_params.go:277-287
//   newPeerScore + the RawTracer / router methods of peerScore score.go:180-974
// Peer ids and topics are strings as in Go; the scorer's clock is injected
// (the reference reads time.Now(); score.go:501,636,657,711,839).
#pragma once

#include <cmath>
#include <cstring>
#include <cstdint>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "gsx.h"

namespace pubsub {

using Duration = int64_t;  // time.Duration, nanoseconds
constexpr Duration Nanosecond = 1, Microsecond = 1000, Millisecond = 1000000, Second = 1000000000,
                   Minute = 60 * Second, Hour = 60 * Minute;

struct Error {
    int code = 0;
    std::string msg;
    explicit operator bool() const { return code != 0; }
};

struct TopicScoreParams {  // score_params.go:98-148
    double TopicWeight = 0;
    double TimeInMeshWeight = 0;
    Duration TimeInMeshQuantum = 0;
    double TimeInMeshCap = 0;
    double FirstMessageDeliveriesWeight = 0, FirstMessageDeliveriesDecay = 0, FirstMessageDeliveriesCap = 0;
    double MeshMessageDeliveriesWeight = 0, MeshMessageDeliveriesDecay = 0;
    double MeshMessageDeliveriesCap = 0, MeshMessageDeliveriesThreshold = 0;
    Duration MeshMessageDeliveriesWindow = 0, MeshMessageDeliveriesActivation = 0;
    double MeshFailurePenaltyWeight = 0, MeshFailurePenaltyDecay = 0;
    double InvalidMessageDeliveriesWeight = 0, InvalidMessageDeliveriesDecay = 0;

    gsx_topic_score_params c() const {
        gsx_topic_score_params p{};
        p.topic_weight = TopicWeight;
        p.time_in_mesh_weight = TimeInMeshWeight;
        p.time_in_mesh_quantum_ns = TimeInMeshQuantum;
        p.time_in_mesh_cap = TimeInMeshCap;
        p.first_message_deliveries_weight = FirstMessageDeliveriesWeight;
        p.first_message_deliveries_decay = FirstMessageDeliveriesDecay;
        p.first_message_deliveries_cap = FirstMessageDeliveriesCap;
        p.mesh_message_deliveries_weight = MeshMessageDeliveriesWeight;
        p.mesh_message_deliveries_decay = MeshMessageDeliveriesDecay;
        p.mesh_message_deliveries_cap = MeshMessageDeliveriesCap;
        p.mesh_message_deliveries_threshold = MeshMessageDeliveriesThreshold;
        p.mesh_message_deliveries_window_ns = MeshMessageDeliveriesWindow;
        p.mesh_message_deliveries_activation_ns = MeshMessageDeliveriesActivation;
        p.mesh_failure_penalty_weight = MeshFailurePenaltyWeight;
        p.mesh_failure_penalty_decay = MeshFailurePenaltyDecay;
        p.invalid_message_deliveries_weight = InvalidMessageDeliveriesWeight;
        p.invalid_message_deliveries_decay = InvalidMessageDeliveriesDecay;
        return p;
    }
    Error validate() const {  // score_params.go:200-268
        const gsx_topic_score_params p = c();
        if (gsx_validate_topic_params(&p) != 0) return {GSX_EINVAL, "invalid topic score parameters"};
        return {};
    }
};

struct PeerScoreParams {  // score_params.go:53-96
    std::map<std::string, TopicScoreParams> Topics;
    double TopicScoreCap = 0;
    std::function<double(const std::string&)> AppSpecificScore;
    double AppSpecificWeight = 0;
    double IPColocationFactorWeight = 0;
    int IPColocationFactorThreshold = 0;
    std::vector<std::string> IPColocationFactorWhitelist;  // IPs, resolved from the CIDRs by the caller
    double BehaviourPenaltyWeight = 0, BehaviourPenaltyThreshold = 0, BehaviourPenaltyDecay = 0;
    Duration DecayInterval = 0;
    double DecayToZero = 0;
    Duration RetainScore = 0;

    gsx_peer_score_params c() const {
        gsx_peer_score_params p{};
        p.topic_score_cap = TopicScoreCap;
        p.app_specific_weight = AppSpecificWeight;
        p.app_specific_score_set = AppSpecificScore ? 1 : 0;
        p.ip_colocation_factor_threshold = IPColocationFactorThreshold;
        p.ip_colocation_factor_weight = IPColocationFactorWeight;
        p.behaviour_penalty_weight = BehaviourPenaltyWeight;
        p.behaviour_penalty_threshold = BehaviourPenaltyThreshold;
        p.behaviour_penalty_decay = BehaviourPenaltyDecay;
        p.decay_interval_ns = DecayInterval;
        p.decay_to_zero = DecayToZero;
        p.retain_score_ns = RetainScore;
        return p;
    }
    Error validate() const {  // score_params.go:151-198
        for (const auto& kv : Topics)
            if (Error e = kv.second.validate()) return {e.code, "invalid score parameters for topic " + kv.first};
        const gsx_peer_score_params p = c();
        if (gsx_validate_peer_params(&p) != 0) return {GSX_EINVAL, "invalid peer score parameters"};
        return {};
    }
};

struct PeerScoreThresholds {  // score_params.go:12-32
    double GossipThreshold = 0, PublishThreshold = 0, GraylistThreshold = 0, AcceptPXThreshold = 0,
           OpportunisticGraftThreshold = 0;
    Error validate() const {
        gsx_thresholds t{GossipThreshold, PublishThreshold, GraylistThreshold, AcceptPXThreshold,
                         OpportunisticGraftThreshold};
        if (gsx_validate_thresholds(&t) != 0) return {GSX_EINVAL, "invalid peer score thresholds"};
        return {};
    }
};

inline double ScoreParameterDecayWithBase(Duration decay, Duration base, double decayToZero) {
    return gsx_score_parameter_decay_with_base(decay, base, decayToZero);
}
inline double ScoreParameterDecay(Duration decay) { return gsx_score_parameter_decay(decay); }

// Reject reasons, tracer.go:28-38
inline const std::map<std::string, int32_t>& reject_reasons() {
    static const std::map<std::string, int32_t> m = {
        {"blacklisted peer", GSX_REJECT_BLACKLISTED_PEER},
        {"blacklisted source", GSX_REJECT_BLACKLISTED_SOURCE},
        {"missing signature", GSX_REJECT_MISSING_SIGNATURE},
        {"unexpected signature", GSX_REJECT_UNEXPECTED_SIGNATURE},
        {"unexpected auth info", GSX_REJECT_UNEXPECTED_AUTH_INFO},
        {"invalid signature", GSX_REJECT_INVALID_SIGNATURE},
        {"validation queue full", GSX_REJECT_VALIDATION_QUEUE_FULL},
        {"validation throttled", GSX_REJECT_VALIDATION_THROTTLED},
        {"validation failed", GSX_REJECT_VALIDATION_FAILED},
        {"validation ignored", GSX_REJECT_VALIDATION_IGNORED},
        {"self originated message", GSX_REJECT_SELF_ORIGIN},
    };
    return m;
}
const std::string RejectBlacklstedPeer = "blacklisted peer", RejectBlacklistedSource = "blacklisted source",
                  RejectMissingSignature = "missing signature", RejectUnexpectedSignature = "unexpected signature",
                  RejectUnexpectedAuthInfo = "unexpected auth info", RejectInvalidSignature = "invalid signature",
                  RejectValidationQueueFull = "validation queue full",
                  RejectValidationThrottled = "validation throttled", RejectValidationFailed = "validation failed",
                  RejectValidationIgnored = "validation ignored", RejectSelfOrigin = "self originated message";

// The scorer's view of a pubsub Message (pubsub.go Message): id = msgID(msg).
struct Message {
    std::string ID;
    std::string Topic;
    std::string ReceivedFrom;
};

// Clock injected where the reference reads time.Now().
struct Clock {
    int64_t now = 1700000000LL * Second;
    int64_t Now() const { return now; }
    void Sleep(Duration d) { now += d; }
};

// One router's peerScore (score.go:64-86) on the GPU engine.  The peer
// universe (ids and their IPs: getIPs, score.go:977-1017) is fixed at
// construction; the topic universe is params.Topics plus `extra_topics`.
class PeerScore {
   public:
    PeerScore(PeerScoreParams params, const std::vector<std::string>& peers,
              const std::map<std::string, std::vector<std::string>>& peer_ips = {}, Clock* clock = nullptr,
              const std::vector<std::string>& extra_topics = {}, int device = 0)
        : params_(std::move(params)), clock_(clock ? clock : &own_clock_) {
        for (const auto& kv : params_.Topics) topic_index(kv.first, true);
        for (const auto& t : extra_topics) topic_index(t, true);
        if (topics_.empty()) topic_index("", true);
        gsx_config cfg{};
        cfg.n_topics = (uint32_t)topics_.size();
        cfg.device = device;
        check(gsx_create(&cfg, &e_), "gsx_create");
        const gsx_peer_score_params pp = params_.c();
        check(gsx_set_peer_params(e_, &pp), "gsx_set_peer_params");
        for (const auto& kv : params_.Topics) {
            const gsx_topic_score_params tp = kv.second.c();
            check(gsx_set_topic_params(e_, topics_.at(kv.first), &tp), "gsx_set_topic_params");
        }
        // one observer (node 0), peers are nodes 1..K
        const uint32_t K = (uint32_t)peers.size();
        std::vector<int64_t> row_ptr(K + 2, (int64_t)K);
        row_ptr[0] = 0;
        std::vector<int32_t> col(K);
        std::vector<uint32_t> ips(2 * (K + 1), GSX_NO_IP);
        std::unordered_map<std::string, uint32_t> ip_ids;
        for (uint32_t i = 0; i < K; ++i) {
            peers_[peers[i]] = i;
            ids_.push_back(peers[i]);
            col[i] = (int32_t)(i + 1);
            auto it = peer_ips.find(peers[i]);
            if (it == peer_ips.end()) continue;
            for (size_t k = 0; k < it->second.size() && k < 2; ++k)
                ips[2 * (i + 1) + k] = ip_ids.emplace(it->second[k], (uint32_t)ip_ids.size()).first->second;
        }
        check(gsx_load_overlay(e_, K + 1, row_ptr.data(), col.data(), nullptr, ips.data()), "gsx_load_overlay");
        std::vector<uint32_t> wl;
        for (const auto& ip : params_.IPColocationFactorWhitelist) {
            auto it = ip_ids.find(ip);
            if (it != ip_ids.end()) wl.push_back(it->second);
        }
        check(gsx_set_ip_whitelist(e_, wl.data(), wl.size()), "gsx_set_ip_whitelist");
        app_.assign(K, 0.0);
    }
    ~PeerScore() { gsx_destroy(e_); }
    PeerScore(const PeerScore&) = delete;
    PeerScore& operator=(const PeerScore&) = delete;

    // ---- router interface -------------------------------------------------------
    double Score(const std::string& p) {  // score.go:247-256
        auto it = peers_.find(p);
        if (it == peers_.end()) return 0;
        sync_app(it->second);  // score() calls AppSpecificScore(p) for p only (:320)
        double s = 0;
        check(gsx_score(e_, it->second, &s), "gsx_score");
        return s;
    }
    // Score(p) of every peer one RPC asks about (AcceptFrom :589, the Publish
    // targets :960-989): one flush, one re-score and one copy (gsx_score_many).
    // Unknown peers score 0, as in Score.
    std::vector<double> ScoreMany(const std::vector<std::string>& ps) {
        std::vector<uint64_t> idx;
        std::vector<size_t> at;
        idx.reserve(ps.size());
        for (size_t i = 0; i < ps.size(); ++i) {
            auto it = peers_.find(ps[i]);
            if (it == peers_.end()) continue;
            sync_app(it->second);
            idx.push_back(it->second);
            at.push_back(i);
        }
        std::vector<double> got(idx.size()), out(ps.size(), 0.0);
        check(gsx_score_many(e_, idx.data(), idx.size(), got.data()), "gsx_score_many");
        for (size_t k = 0; k < at.size(); ++k) out[at[k]] = got[k];
        return out;
    }
    void AddPenalty(const std::string& p, int count) { event(GSX_EV_PENALTY, p, "", count); }  // :384-398
    Error SetTopicScoreParams(const std::string& topic, const TopicScoreParams& p) {  // :194-234
        uint32_t t = topic_index(topic, false);
        if (t == NO_TOPIC) return {GSX_ERANGE, "no topic slot for " + topic};
        const gsx_topic_score_params tp = p.c();
        int rc = gsx_set_topic_params(e_, t, &tp);
        if (rc) return {rc, gsx_last_error(e_)};
        params_.Topics[topic] = p;
        return {};
    }
    void refreshScores() {  // :497-558 (no AppSpecificScore call: Score(p) reads p's when it scores)
        check(gsx_refresh(e_, clock_->Now()), "gsx_refresh");
    }
    void gcDeliveryRecords() { check(gsx_gc_deliveries(e_, clock_->Now()), "gsx_gc_deliveries"); }  // :580-585

    // ---- RawTracer (score.go:588-830) ---------------------------------------------------
    void AddPeer(const std::string& p, const std::string& /*proto*/) { event(GSX_EV_ADD_PEER, p); }
    void RemovePeer(const std::string& p) {
        auto it = peers_.find(p);
        if (it != peers_.end()) sync_app(it->second);  // RemovePeer evaluates score(p) (:615)
        event(GSX_EV_REMOVE_PEER, p);
    }
    void Graft(const std::string& p, const std::string& topic) { event(GSX_EV_GRAFT, p, topic); }
    void Prune(const std::string& p, const std::string& topic) { event(GSX_EV_PRUNE, p, topic); }
    void ValidateMessage(const Message& m) { trace(gsx_trace_validate, m); }
    void DeliverMessage(const Message& m) { trace(gsx_trace_deliver, m); }
    void DuplicateMessage(const Message& m) { trace(gsx_trace_duplicate, m); }
    void RejectMessage(const Message& m, const std::string& reason) {
        auto it = peers_.find(m.ReceivedFrom);
        if (it == peers_.end()) return;
        check(gsx_trace_reject(e_, it->second, msg_id(m.ID), topic_or_unscored(m.Topic), reject_reasons().at(reason),
                               clock_->Now()),
              "gsx_trace_reject");
    }

    // internals the reference's tests reach into (ps.peerStats[p].topics[t].x)
    double topicCounter(const std::string& p, const std::string& topic, const char* field) {
        const size_t K = ids_.size(), T = topics_.size();
        std::vector<double> a(K * T);
        gsx_state_view v{};
        const std::string f = field;
        if (f == "firstMessageDeliveries") v.first_message_deliveries = a.data();
        else if (f == "meshMessageDeliveries") v.mesh_message_deliveries = a.data();
        else if (f == "meshFailurePenalty") v.mesh_failure_penalty = a.data();
        else if (f == "invalidMessageDeliveries") v.invalid_message_deliveries = a.data();
        else throw std::invalid_argument(f);
        check(gsx_export_state(e_, &v), "gsx_export_state");
        return a[topics_.at(topic) * K + peers_.at(p)];
    }
    gsx_engine* engine() { return e_; }

   private:
    static constexpr uint32_t NO_TOPIC = 0xFFFFFFFFu;

    static void check(int rc, const char* what) {
        if (rc != 0) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
    }
    uint32_t topic_index(const std::string& t, bool create) {
        auto it = topics_.find(t);
        if (it != topics_.end()) return it->second;
        if (!create) return NO_TOPIC;
        const uint32_t i = (uint32_t)topics_.size();
        topics_[t] = i;
        return i;
    }
    // a topic outside the universe is unscored: route it to a topic index that
    // never has params (or drop the call, which is the same no-op)
    uint32_t topic_or_unscored(const std::string& t) {
        const uint32_t i = topic_index(t, false);
        return i == NO_TOPIC ? GSX_MAX_TOPICS : i;
    }
    uint64_t msg_id(const std::string& id) {
        return msgs_.emplace(id, (uint64_t)msgs_.size()).first->second;
    }
    void event(uint32_t kind, const std::string& p, const std::string& topic = "", int64_t arg = 0) {
        auto it = peers_.find(p);
        if (it == peers_.end()) return;  // unknown peer: a no-op in the reference too
        gsx_event ev{kind, topic.empty() ? 0u : topic_or_unscored(topic), it->second, clock_->Now(), arg};
        check(gsx_apply_events(e_, &ev, 1), "gsx_apply_events");
    }
    void trace(int (*fn)(gsx_engine*, uint64_t, uint64_t, uint32_t, int64_t), const Message& m) {
        auto it = peers_.find(m.ReceivedFrom);
        if (it == peers_.end()) return;
        check(fn(e_, it->second, msg_id(m.ID), topic_or_unscored(m.Topic), clock_->Now()), "gsx_trace");
    }
    static bool same(double a, double b) { return a == b && std::signbit(a) == std::signbit(b); }
    // AppSpecificScore(p) is called at score time (:320), for the scored peer
    // only: a changed value is one GSX_EV_APP_SCORE event (the engine then
    // re-scores that observer's row); an unchanged one leaves the engine's
    // scores, and their host copy, valid.  The first call takes every peer's.
    void sync_app(uint32_t i) {
        if (!params_.AppSpecificScore) return;
        if (!app_synced_) {
            sync_app_all();
            return;
        }
        const double a = params_.AppSpecificScore(ids_[i]);
        if (same(a, app_[i])) return;
        app_[i] = a;
        int64_t bits;
        std::memcpy(&bits, &a, sizeof bits);
        gsx_event ev{GSX_EV_APP_SCORE, 0u, i, clock_->Now(), bits};
        check(gsx_apply_events(e_, &ev, 1), "gsx_apply_events");
    }
    void sync_app_all() {  // a snapshot of every peer's (construction, inspection)
        if (!params_.AppSpecificScore) return;
        bool changed = !app_synced_;
        for (size_t i = 0; i < ids_.size(); ++i) {
            const double a = params_.AppSpecificScore(ids_[i]);
            changed |= !same(a, app_[i]);
            app_[i] = a;
        }
        if (changed) check(gsx_set_app_scores(e_, app_.data(), app_.size()), "gsx_set_app_scores");
        app_synced_ = true;
    }

    PeerScoreParams params_;
    Clock own_clock_;
    Clock* clock_;
    gsx_engine* e_ = nullptr;
    std::unordered_map<std::string, uint32_t> peers_;
    std::vector<std::string> ids_;
    std::map<std::string, uint32_t> topics_;
    std::unordered_map<std::string, uint64_t> msgs_;
    std::vector<double> app_;
    bool app_synced_ = false;
};

}  // namespace pubsub
