// score_test.cpp — the reference's score_test.go, restated over the C++ mirror
// (include/gsx_pubsub.hpp) of the peer-scoring interface, so the parity tests
// read like the reference's own.  time.Sleep becomes a simulated clock; the
// values asserted are the reference's.  Runs on the GPU engine via the C ABI.
#include <cmath>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "../../include/gsx_pubsub.hpp"

using namespace pubsub;

static int failures = 0;
#define FATALF(...)                          \
    do {                                     \
        std::printf("    FAIL: " __VA_ARGS__); \
        std::printf("\n");                   \
        ++failures;                          \
        return;                              \
    } while (0)

static Message makeTestMessage(int i, const std::string& topic, const std::string& from) {
    return Message{"msg-" + std::to_string(i), topic, from};
}

static PeerScoreParams base_params() {
    PeerScoreParams p;
    p.AppSpecificScore = [](const std::string&) { return 0.0; };
    return p;
}

static const std::string mytopic = "mytopic";

static void TestScoreTimeInMesh() {  // score_test.go:13-50
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 0.5;
    tsp.TimeInMeshWeight = 1;
    tsp.TimeInMeshQuantum = Millisecond;
    tsp.TimeInMeshCap = 3600;
    params.Topics[mytopic] = tsp;
    Clock clk;
    PeerScore ps(params, {"A"}, {}, &clk);
    ps.AddPeer("A", "myproto");
    if (ps.Score("A") != 0) FATALF("expected score to start at zero");
    ps.Graft("A", mytopic);
    Duration elapsed = tsp.TimeInMeshQuantum * 200;
    clk.Sleep(elapsed);
    ps.refreshScores();
    double aScore = ps.Score("A");
    double expected = tsp.TopicWeight * tsp.TimeInMeshWeight * double(elapsed / tsp.TimeInMeshQuantum);
    if (aScore < expected) FATALF("Score: %f. Expected >= %f", aScore, expected);
}

static void TestScoreTimeInMeshCap() {  // score_test.go:52-84
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 0.5;
    tsp.TimeInMeshWeight = 1;
    tsp.TimeInMeshQuantum = Millisecond;
    tsp.TimeInMeshCap = 10;
    params.Topics[mytopic] = tsp;
    Clock clk;
    PeerScore ps(params, {"A"}, {}, &clk);
    ps.AddPeer("A", "myproto");
    ps.Graft("A", mytopic);
    clk.Sleep(tsp.TimeInMeshQuantum * 40);
    ps.refreshScores();
    double aScore = ps.Score("A");
    double expected = tsp.TopicWeight * tsp.TimeInMeshWeight * tsp.TimeInMeshCap;
    double variance = 0.5;
    if (!(aScore > expected * (1 - variance) && aScore < expected * (1 + variance)))
        FATALF("Score: %f. Expected %f +- %f", aScore, expected, variance * expected);
}

static void first_deliveries(double decay, double cap, const char* name) {  // score_test.go:86-215
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 1;
    tsp.FirstMessageDeliveriesWeight = 1;
    tsp.FirstMessageDeliveriesDecay = decay;
    tsp.FirstMessageDeliveriesCap = cap;
    tsp.TimeInMeshQuantum = Second;
    params.Topics[mytopic] = tsp;
    PeerScore ps(params, {"A"});
    ps.AddPeer("A", "myproto");
    ps.Graft("A", mytopic);
    const int nMessages = 100;
    for (int i = 0; i < nMessages; i++) {
        Message msg = makeTestMessage(i, mytopic, "A");
        ps.ValidateMessage(msg);
        ps.DeliverMessage(msg);
    }
    ps.refreshScores();
    double aScore = ps.Score("A");
    double expected;
    if (decay != 1.0)
        expected = tsp.TopicWeight * tsp.FirstMessageDeliveriesWeight * tsp.FirstMessageDeliveriesDecay * double(nMessages);
    else if (cap < nMessages)
        expected = tsp.TopicWeight * tsp.FirstMessageDeliveriesWeight * tsp.FirstMessageDeliveriesCap;
    else
        expected = tsp.TopicWeight * tsp.FirstMessageDeliveriesWeight * double(nMessages);
    if (aScore != expected) FATALF("%s Score: %.17g. Expected %.17g", name, aScore, expected);
    if (decay != 1.0) {
        for (int i = 0; i < 10; i++) {
            ps.refreshScores();
            expected *= tsp.FirstMessageDeliveriesDecay;
        }
        aScore = ps.Score("A");
        if (aScore != expected) FATALF("%s Score: %.17g. Expected %.17g", name, aScore, expected);
    }
}
static void TestScoreFirstMessageDeliveries() { first_deliveries(1.0, 2000, "FirstMessageDeliveries"); }
static void TestScoreFirstMessageDeliveriesCap() { first_deliveries(1.0, 50, "FirstMessageDeliveriesCap"); }
static void TestScoreFirstMessageDeliveriesDecay() { first_deliveries(0.9, 2000, "FirstMessageDeliveriesDecay"); }

static void TestScoreMeshMessageDeliveries() {  // score_test.go:217-308
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 1;
    tsp.MeshMessageDeliveriesWeight = -1;
    tsp.MeshMessageDeliveriesActivation = Second;
    tsp.MeshMessageDeliveriesWindow = 10 * Millisecond;
    tsp.MeshMessageDeliveriesThreshold = 20;
    tsp.MeshMessageDeliveriesCap = 100;
    tsp.MeshMessageDeliveriesDecay = 1.0;
    tsp.FirstMessageDeliveriesWeight = 0;
    tsp.TimeInMeshQuantum = Second;
    params.Topics[mytopic] = tsp;
    Clock clk;
    std::vector<std::string> peers = {"A", "B", "C"};
    PeerScore ps(params, peers, {}, &clk);
    for (auto& p : peers) {
        ps.AddPeer(p, "myproto");
        ps.Graft(p, mytopic);
    }
    ps.refreshScores();
    for (auto& p : peers)
        if (ps.Score(p) < 0) FATALF("expected no mesh delivery penalty before activation time");
    clk.Sleep(tsp.MeshMessageDeliveriesActivation);
    const int nMessages = 100;
    for (int i = 0; i < nMessages; i++) {
        Message msg = makeTestMessage(i, mytopic, "A");
        ps.ValidateMessage(msg);
        ps.DeliverMessage(msg);
        msg.ReceivedFrom = "B";
        ps.DuplicateMessage(msg);
    }
    clk.Sleep(tsp.MeshMessageDeliveriesWindow + 20 * Millisecond);  // the time.AfterFunc duplicates from C
    for (int i = 0; i < nMessages; i++) {
        Message msg = makeTestMessage(i, mytopic, "C");
        ps.DuplicateMessage(msg);
    }
    ps.refreshScores();
    double a = ps.Score("A"), b = ps.Score("B"), c = ps.Score("C");
    if (a < 0) FATALF("Expected non-negative score for peer A, got %f", a);
    if (b < 0) FATALF("Expected non-negative score for peer B, got %f", b);
    double penalty = tsp.MeshMessageDeliveriesThreshold * tsp.MeshMessageDeliveriesThreshold;
    double expected = tsp.TopicWeight * tsp.MeshMessageDeliveriesWeight * penalty;
    if (c != expected) FATALF("Score: %f. Expected %f", c, expected);
}

static void TestScoreMeshMessageDeliveriesDecay() {  // score_test.go:310-369
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 1;
    tsp.MeshMessageDeliveriesWeight = -1;
    tsp.MeshMessageDeliveriesActivation = 0;
    tsp.MeshMessageDeliveriesWindow = 10 * Millisecond;
    tsp.MeshMessageDeliveriesThreshold = 20;
    tsp.MeshMessageDeliveriesCap = 100;
    tsp.MeshMessageDeliveriesDecay = 0.9;
    tsp.FirstMessageDeliveriesWeight = 0;
    tsp.TimeInMeshQuantum = Second;
    params.Topics[mytopic] = tsp;
    Clock clk;
    PeerScore ps(params, {"A"}, {}, &clk);
    ps.AddPeer("A", "myproto");
    ps.Graft("A", mytopic);
    const int nMessages = 40;
    for (int i = 0; i < nMessages; i++) {
        Message msg = makeTestMessage(i, mytopic, "A");
        ps.ValidateMessage(msg);
        ps.DeliverMessage(msg);
    }
    clk.Sleep(Millisecond);
    ps.refreshScores();
    if (ps.Score("A") < 0) FATALF("Expected non-negative score for peer A");
    double decayed = double(nMessages) * tsp.MeshMessageDeliveriesDecay;
    for (int i = 0; i < 20; i++) {
        ps.refreshScores();
        decayed *= tsp.MeshMessageDeliveriesDecay;
    }
    double deficit = tsp.MeshMessageDeliveriesThreshold - decayed;
    double expected = tsp.TopicWeight * tsp.MeshMessageDeliveriesWeight * (deficit * deficit);
    double a = ps.Score("A");
    if (a != expected) FATALF("Score: %.17g. Expected %.17g", a, expected);
}

static void TestScoreMeshFailurePenalty() {  // score_test.go:371-450
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 1;
    tsp.MeshFailurePenaltyWeight = -1;
    tsp.MeshFailurePenaltyDecay = 1.0;
    tsp.MeshMessageDeliveriesActivation = 0;
    tsp.MeshMessageDeliveriesWindow = 10 * Millisecond;
    tsp.MeshMessageDeliveriesThreshold = 20;
    tsp.MeshMessageDeliveriesCap = 100;
    tsp.MeshMessageDeliveriesDecay = 1.0;
    tsp.TimeInMeshQuantum = Second;
    params.Topics[mytopic] = tsp;
    Clock clk;
    PeerScore ps(params, {"A", "B"}, {}, &clk);
    for (auto p : {"A", "B"}) {
        ps.AddPeer(p, "myproto");
        ps.Graft(p, mytopic);
    }
    for (int i = 0; i < 100; i++) {
        Message msg = makeTestMessage(i, mytopic, "A");
        ps.ValidateMessage(msg);
        ps.DeliverMessage(msg);
    }
    clk.Sleep(Millisecond);
    ps.refreshScores();
    if (ps.Score("A") != 0) FATALF("expected peer A to have score 0.0");
    if (ps.Score("B") != 0) FATALF("expected peer B to have score 0.0");
    ps.Prune("B", mytopic);
    ps.refreshScores();
    if (ps.Score("A") != 0) FATALF("expected peer A to have score 0.0");
    double penalty = tsp.MeshMessageDeliveriesThreshold * tsp.MeshMessageDeliveriesThreshold;
    double expected = tsp.TopicWeight * tsp.MeshFailurePenaltyWeight * penalty;
    if (ps.Score("B") != expected) FATALF("Score: %f. Expected %f", ps.Score("B"), expected);
}

static void invalid_deliveries(double decay) {  // score_test.go:452-534
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 1;
    tsp.TimeInMeshQuantum = Second;
    tsp.InvalidMessageDeliveriesWeight = -1;
    tsp.InvalidMessageDeliveriesDecay = decay;
    params.Topics[mytopic] = tsp;
    PeerScore ps(params, {"A"});
    ps.AddPeer("A", "myproto");
    ps.Graft("A", mytopic);
    const int nMessages = 100;
    for (int i = 0; i < nMessages; i++) ps.RejectMessage(makeTestMessage(i, mytopic, "A"), RejectInvalidSignature);
    ps.refreshScores();
    double expected;
    if (decay == 1.0)
        expected = tsp.TopicWeight * tsp.InvalidMessageDeliveriesWeight * double(nMessages * nMessages);
    else
        expected = tsp.TopicWeight * tsp.InvalidMessageDeliveriesWeight *
                   std::pow(tsp.InvalidMessageDeliveriesDecay * double(nMessages), 2);
    if (ps.Score("A") != expected) FATALF("Score: %.17g. Expected %.17g", ps.Score("A"), expected);
    if (decay != 1.0) {
        for (int i = 0; i < 10; i++) {
            ps.refreshScores();
            expected *= std::pow(tsp.InvalidMessageDeliveriesDecay, 2);
        }
        if (ps.Score("A") != expected) FATALF("Score: %.17g. Expected %.17g", ps.Score("A"), expected);
    }
}
static void TestScoreInvalidMessageDeliveries() { invalid_deliveries(1.0); }
static void TestScoreInvalidMessageDeliveriesDecay() { invalid_deliveries(0.9); }

static void TestScoreRejectMessageDeliveries() {  // score_test.go:536-666
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 1;
    tsp.TimeInMeshQuantum = Second;
    tsp.InvalidMessageDeliveriesWeight = -1;
    tsp.InvalidMessageDeliveriesDecay = 1.0;
    params.Topics[mytopic] = tsp;
    Clock clk;
    PeerScore ps(params, {"A", "B"}, {}, &clk);
    ps.AddPeer("A", "myproto");
    ps.AddPeer("B", "myproto");
    Message msg = makeTestMessage(0, mytopic, "A"), msg2 = makeTestMessage(0, mytopic, "B");
    ps.RejectMessage(msg, RejectBlacklstedPeer);
    ps.RejectMessage(msg, RejectBlacklistedSource);
    ps.RejectMessage(msg, RejectValidationQueueFull);
    if (ps.Score("A") != 0) FATALF("Score: %f. Expected 0", ps.Score("A"));
    auto clear_records = [&] {  // ps.deliveries.head.expire = time.Now(); gc()
        clk.Sleep(121 * Second);
        ps.gcDeliveryRecords();
    };
    ps.ValidateMessage(msg);
    ps.RejectMessage(msg, RejectValidationThrottled);
    ps.DuplicateMessage(msg2);
    if (ps.Score("A") != 0 || ps.Score("B") != 0) FATALF("throttled: expected 0, 0");
    clear_records();
    ps.ValidateMessage(msg);
    ps.RejectMessage(msg, RejectValidationIgnored);
    ps.DuplicateMessage(msg2);
    if (ps.Score("A") != 0 || ps.Score("B") != 0) FATALF("ignored: expected 0, 0");
    clear_records();
    ps.ValidateMessage(msg);
    ps.RejectMessage(msg, RejectValidationFailed);
    ps.DuplicateMessage(msg2);
    if (ps.Score("A") != -1.0) FATALF("Score: %f. Expected -1", ps.Score("A"));
    if (ps.Score("B") != -1.0) FATALF("Score: %f. Expected -1", ps.Score("B"));
    clear_records();
    ps.ValidateMessage(msg);
    ps.DuplicateMessage(msg2);
    ps.RejectMessage(msg, RejectValidationFailed);
    if (ps.Score("A") != -4.0) FATALF("Score: %f. Expected -4", ps.Score("A"));
    if (ps.Score("B") != -4.0) FATALF("Score: %f. Expected -4", ps.Score("B"));
}

static void TestScoreApplicationScore() {  // score_test.go:668-694
    double appScoreValue = 0;
    PeerScoreParams params;
    params.AppSpecificScore = [&](const std::string&) { return appScoreValue; };
    params.AppSpecificWeight = 0.5;
    PeerScore ps(params, {"A"});
    ps.AddPeer("A", "myproto");
    ps.Graft("A", mytopic);
    for (int i = -100; i < 100; i++) {
        appScoreValue = double(i);
        ps.refreshScores();
        double expected = double(i) * params.AppSpecificWeight;
        if (ps.Score("A") != expected) FATALF("expected peer score to equal app-specific score %f, got %f", expected, ps.Score("A"));
    }
}

static void ip_colocation(bool whitelist) {  // score_test.go:696-803
    auto params = base_params();
    params.IPColocationFactorThreshold = 1;
    params.IPColocationFactorWeight = -1;
    if (whitelist) params.IPColocationFactorWhitelist = {"2.3.4.5"};  // the IPs inside 2.3.0.0/16
    std::vector<std::string> peers = {"A", "B", "C", "D"};
    PeerScore ps(params, peers,
                 {{"A", {"1.2.3.4"}}, {"B", {"2.3.4.5"}}, {"C", {"2.3.4.5", "3.4.5.6"}}, {"D", {"2.3.4.5"}}});
    for (auto& p : peers) {
        ps.AddPeer(p, "myproto");
        ps.Graft(p, mytopic);
    }
    ps.refreshScores();
    if (ps.Score("A") != 0) FATALF("expected peer A to have score 0.0, got %f", ps.Score("A"));
    int nShared = 3;
    int ipSurplus = nShared - params.IPColocationFactorThreshold;
    double expected = whitelist ? 0.0 : params.IPColocationFactorWeight * double(ipSurplus * ipSurplus);
    for (auto p : {"B", "C", "D"})
        if (ps.Score(p) != expected) FATALF("Score: %f. Expected %f", ps.Score(p), expected);
}
static void TestScoreIPColocation() { ip_colocation(false); }
static void TestScoreIPColocationWhitelist() { ip_colocation(true); }

static void TestScoreBehaviourPenalty() {  // score_test.go:805-859
    PeerScoreParams params;
    params.AppSpecificScore = [](const std::string&) { return 0.0; };
    params.BehaviourPenaltyWeight = -1;
    params.BehaviourPenaltyDecay = 0.99;
    PeerScore ps(params, {"A"});
    ps.AddPenalty("A", 1);  // on a peer without stats
    if (ps.Score("A") != 0) FATALF("expected peer score to be 0");
    ps.AddPeer("A", "myproto");
    if (ps.Score("A") != 0) FATALF("expected peer score to be 0");
    ps.AddPenalty("A", 1);
    if (ps.Score("A") != -1) FATALF("expected peer score to be -1, got %f", ps.Score("A"));
    ps.AddPenalty("A", 1);
    if (ps.Score("A") != -4) FATALF("expected peer score to be -4, got %f", ps.Score("A"));
    ps.refreshScores();
    if (ps.Score("A") != -3.9204) FATALF("expected peer score to be -3.9204, got %.17g", ps.Score("A"));
}

static void TestScoreRetention() {  // score_test.go:861-903
    PeerScoreParams params;
    params.AppSpecificScore = [](const std::string&) { return -1000.0; };
    params.AppSpecificWeight = 1.0;
    params.RetainScore = Second;
    Clock clk;
    PeerScore ps(params, {"A"}, {}, &clk);
    ps.AddPeer("A", "myproto");
    ps.Graft("A", mytopic);
    double expected = -1000;
    ps.refreshScores();
    if (ps.Score("A") != expected) FATALF("Score: %f. Expected %f", ps.Score("A"), expected);
    ps.RemovePeer("A");
    Duration delay = params.RetainScore / Duration(2);
    clk.Sleep(delay);
    ps.refreshScores();
    if (ps.Score("A") != expected) FATALF("Score: %f. Expected %f", ps.Score("A"), expected);
    clk.Sleep(delay + 50 * Millisecond);
    ps.refreshScores();
    if (ps.Score("A") != 0) FATALF("Score: %f. Expected 0.0", ps.Score("A"));
}

static void TestScoreRecapTopicParams() {  // score_test.go:905-1000
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 1;
    tsp.MeshMessageDeliveriesWeight = -1;
    tsp.MeshMessageDeliveriesActivation = Second;
    tsp.MeshMessageDeliveriesWindow = 10 * Millisecond;
    tsp.MeshMessageDeliveriesThreshold = 20;
    tsp.MeshMessageDeliveriesCap = 100;
    tsp.MeshMessageDeliveriesDecay = 1.0;
    tsp.FirstMessageDeliveriesWeight = 10;
    tsp.FirstMessageDeliveriesDecay = 1.0;
    tsp.FirstMessageDeliveriesCap = 100;
    tsp.TimeInMeshQuantum = Second;
    params.Topics[mytopic] = tsp;
    PeerScore ps(params, {"A", "B"});
    for (auto p : {"A", "B"}) {
        ps.AddPeer(p, "myproto");
        ps.Graft(p, mytopic);
    }
    for (int i = 0; i < 100; i++) {
        Message msg = makeTestMessage(i, mytopic, "A");
        ps.ValidateMessage(msg);
        ps.DeliverMessage(msg);
        msg.ReceivedFrom = "B";
        ps.DuplicateMessage(msg);
    }
    if (ps.topicCounter("A", mytopic, "firstMessageDeliveries") != 100) FATALF("expected 100 FirstMessageDeliveries for peerA");
    if (ps.topicCounter("B", mytopic, "meshMessageDeliveries") != 100) FATALF("expected 100 MeshMessageDeliveries for peerB");
    TopicScoreParams n = tsp;
    n.MeshMessageDeliveriesCap = 50;
    n.FirstMessageDeliveriesCap = 50;
    if (Error err = ps.SetTopicScoreParams(mytopic, n)) FATALF("%s", err.msg.c_str());
    if (ps.topicCounter("A", mytopic, "firstMessageDeliveries") != 50) FATALF("expected 50 FirstMessageDeliveries for peerA");
    if (ps.topicCounter("B", mytopic, "meshMessageDeliveries") != 50) FATALF("expected 50 MeshMessageDeliveries for peerB");
}

static void TestScoreResetTopicParams() {  // score_test.go:1002-1062
    auto params = base_params();
    TopicScoreParams tsp;
    tsp.TopicWeight = 1;
    tsp.TimeInMeshQuantum = Second;
    tsp.InvalidMessageDeliveriesWeight = -1;
    tsp.InvalidMessageDeliveriesDecay = 1.0;
    params.Topics[mytopic] = tsp;
    PeerScore ps(params, {"A"});
    ps.AddPeer("A", "myproto");
    for (int i = 0; i < 100; i++) {
        Message msg = makeTestMessage(i, mytopic, "A");
        ps.ValidateMessage(msg);
        ps.RejectMessage(msg, RejectValidationFailed);
    }
    if (ps.Score("A") != -10000) FATALF("expected a -10000 score, but got %f instead", ps.Score("A"));
    TopicScoreParams n = tsp;
    n.InvalidMessageDeliveriesWeight = -10;
    if (Error err = ps.SetTopicScoreParams(mytopic, n)) FATALF("%s", err.msg.c_str());
    if (ps.Score("A") != -100000) FATALF("expected a -100000 score, but got %f instead", ps.Score("A"));
}

static void TestScoreParameterDecay() {  // score_params_test.go:323-328
    double decay1hr = ScoreParameterDecay(Hour);
    if (decay1hr != .9987216039048303) FATALF("expected .9987216039048303, got %.17g", decay1hr);
}

int main() {
    struct {
        const char* name;
        void (*fn)();
    } tests[] = {
        {"TestScoreTimeInMesh", TestScoreTimeInMesh},
        {"TestScoreTimeInMeshCap", TestScoreTimeInMeshCap},
        {"TestScoreFirstMessageDeliveries", TestScoreFirstMessageDeliveries},
        {"TestScoreFirstMessageDeliveriesCap", TestScoreFirstMessageDeliveriesCap},
        {"TestScoreFirstMessageDeliveriesDecay", TestScoreFirstMessageDeliveriesDecay},
        {"TestScoreMeshMessageDeliveries", TestScoreMeshMessageDeliveries},
        {"TestScoreMeshMessageDeliveriesDecay", TestScoreMeshMessageDeliveriesDecay},
        {"TestScoreMeshFailurePenalty", TestScoreMeshFailurePenalty},
        {"TestScoreInvalidMessageDeliveries", TestScoreInvalidMessageDeliveries},
        {"TestScoreInvalidMessageDeliveriesDecay", TestScoreInvalidMessageDeliveriesDecay},
        {"TestScoreRejectMessageDeliveries", TestScoreRejectMessageDeliveries},
        {"TestScoreApplicationScore", TestScoreApplicationScore},
        {"TestScoreIPColocation", TestScoreIPColocation},
        {"TestScoreIPColocationWhitelist", TestScoreIPColocationWhitelist},
        {"TestScoreBehaviourPenalty", TestScoreBehaviourPenalty},
        {"TestScoreRetention", TestScoreRetention},
        {"TestScoreRecapTopicParams", TestScoreRecapTopicParams},
        {"TestScoreResetTopicParams", TestScoreResetTopicParams},
        {"TestScoreParameterDecay", TestScoreParameterDecay},
    };
    for (auto& t : tests) {
        const int before = failures;
        try {
            t.fn();
        } catch (const std::exception& ex) {
            std::printf("    FAIL: exception %s\n", ex.what());
            ++failures;
        }
        std::printf("%s %s\n", failures == before ? "ok  " : "FAIL", t.name);
    }
    std::printf("%d failure(s)\n", failures);
    return failures ? 1 : 0;
}
