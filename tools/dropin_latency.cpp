// dropin_latency.cpp — per-call latency of the drop-in scorer (one router's
// peerScore on the GPU engine through include/gsx_pubsub.hpp), the path a cgo
// shim inside one gossipsub router would take.  Prints one
// JSON object.  The router's call pattern per RPC (gossipsub.go:589 AcceptFrom
// -> Score; pubsub.go pushMsg -> ValidateMessage / DeliverMessage /
// DuplicateMessage; gossipsub.go:960-989 Publish -> Score per target) mixes
// tracer calls and Score(); each leg below times one such pattern.
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "../include/gsx_pubsub.hpp"

using namespace pubsub;
using Clk = std::chrono::steady_clock;

static long app_calls = 0;  // AppSpecificScore closure calls (score.go:320: one per score(p))

static double us_since(Clk::time_point t0, int n) {
    return std::chrono::duration<double, std::micro>(Clk::now() - t0).count() / n;
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? std::atoi(argv[1]) : 1000;  // connected peers of the router
    const int N = argc > 2 ? std::atoi(argv[2]) : 2000;  // calls per leg
    PeerScoreParams p;
    p.AppSpecificScore = [](const std::string&) {
        ++app_calls;
        return 0.0;
    };
    p.DecayInterval = Second;
    p.DecayToZero = 0.01;
    p.IPColocationFactorWeight = -10;
    p.IPColocationFactorThreshold = 1;
    p.BehaviourPenaltyWeight = -10;
    p.BehaviourPenaltyDecay = 0.99;
    TopicScoreParams t;  // gossipsub_spam_test.go:636-654
    t.TopicWeight = 0.25;
    t.TimeInMeshWeight = 0.0027;
    t.TimeInMeshQuantum = Second;
    t.TimeInMeshCap = 3600;
    t.FirstMessageDeliveriesWeight = 0.664;
    t.FirstMessageDeliveriesDecay = 0.9916;
    t.FirstMessageDeliveriesCap = 1500;
    t.MeshMessageDeliveriesWeight = -0.25;
    t.MeshMessageDeliveriesDecay = 0.97;
    t.MeshMessageDeliveriesCap = 400;
    t.MeshMessageDeliveriesThreshold = 100;
    t.MeshMessageDeliveriesActivation = 30 * Second;
    t.MeshMessageDeliveriesWindow = 5 * Minute;
    t.MeshFailurePenaltyWeight = -0.25;
    t.MeshFailurePenaltyDecay = 0.997;
    t.InvalidMessageDeliveriesWeight = -99;
    t.InvalidMessageDeliveriesDecay = 0.9994;
    p.Topics["t"] = t;
    std::vector<std::string> peers;
    std::map<std::string, std::vector<std::string>> ips;
    for (int i = 0; i < K; ++i) {
        peers.push_back("peer-" + std::to_string(i));
        ips[peers.back()] = {"10.0." + std::to_string(i % 200) + ".1"};
    }
    Clock clk;
    PeerScore ps(p, peers, ips, &clk);
    for (auto& q : peers) ps.AddPeer(q, "/meshsub/1.1.0");
    for (int i = 0; i < 6; ++i) ps.Graft(peers[i], "t");
    volatile double sink = 0;
    for (int i = 0; i < 50; ++i) sink += ps.Score(peers[i % K]);  // warm-up (first launches)

    auto t0 = Clk::now();
    for (int i = 0; i < N; ++i) sink += ps.Score(peers[i % K]);
    const double score_cached = us_since(t0, N);

    t0 = Clk::now();
    for (int i = 0; i < N; ++i) ps.DeliverMessage(Message{"m" + std::to_string(i), "t", peers[i % K]});
    const double deliver = us_since(t0, N);

    const long app0 = app_calls;
    t0 = Clk::now();
    for (int i = 0; i < N; ++i) {
        ps.DeliverMessage(Message{"x" + std::to_string(i), "t", peers[i % K]});
        sink += ps.Score(peers[(i * 7) % K]);
    }
    const double deliver_then_score = us_since(t0, N);
    const double app_per_score = (double)(app_calls - app0) / N;

    t0 = Clk::now();
    for (int i = 0; i < N; ++i) {  // one RPC: AcceptFrom, then the message, then Publish to the mesh
        sink += ps.Score(peers[i % K]);
        const Message m{"y" + std::to_string(i), "t", peers[i % K]};
        ps.ValidateMessage(m);
        ps.DeliverMessage(m);
        for (int j = 0; j < 6; ++j) sink += ps.Score(peers[j]);
    }
    const double rpc = us_since(t0, N);

    std::vector<std::string> targets(peers.begin(), peers.begin() + 6);
    t0 = Clk::now();
    for (int i = 0; i < N; ++i) {  // the same RPC with the batched call: AcceptFrom, message, one ScoreMany
        sink += ps.Score(peers[i % K]);
        const Message m{"z" + std::to_string(i), "t", peers[i % K]};
        ps.ValidateMessage(m);
        ps.DeliverMessage(m);
        for (double v : ps.ScoreMany(targets)) sink += v;
    }
    const double rpc_many = us_since(t0, N);

    const int R = N / 10 > 0 ? N / 10 : 1;
    t0 = Clk::now();
    for (int i = 0; i < R; ++i) {
        clk.Sleep(Second);
        ps.refreshScores();
    }
    const double refresh = us_since(t0, R);
    std::printf(
        "{\"peers\": %d, \"calls_per_leg\": %d, \"score_unchanged_us\": %.3f, \"deliver_message_us\": %.3f, "
        "\"deliver_then_score_us\": %.3f, \"app_score_calls_per_score\": %.2f, "
        "\"rpc_accept_deliver_publish6_us\": %.3f, \"rpc_accept_deliver_publish6_many_us\": %.3f, "
        "\"refresh_scores_us\": %.3f, \"sink\": %g}\n",
        K, N, score_cached, deliver, deliver_then_score, app_per_score, rpc, rpc_many, refresh, (double)sink);
    return 0;
}
