// gsx_device.h — device-side data layout shared by the HIP kernels and the
// host engine.  Everything here is MI355X (gfx950) code; there is no other
// target.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsx {

// Per-topic parameters as the kernels read them (TopicScoreParams,
// score_params.go:98-148), plus the `scored` bit that stands for
// `ps.params.Topics[topic]` existing (score.go:269-273, 520-524).
struct DevTopicParams {
    double topic_weight;
    double w1, cap1;  // P1 weight / cap
    int64_t q1;       // TimeInMeshQuantum (ns)
    double w2, d2, cap2;
    double w3, d3, cap3, thr3;
    int64_t win3, act3;  // window, activation (ns)
    double w3b, d3b;
    double w4, d4;
    int32_t scored;
    int32_t pad;
};

// Global parameters (PeerScoreParams, score_params.go:53-96) passed by value.
struct DevPeerParams {
    double topic_score_cap;
    double w5;
    double w6;
    int64_t thr6;
    double w7, thr7, d7;
    double decay_to_zero;
    int64_t retain_ns;
};

// Pointers to the structure-of-arrays state in HBM.  Record arrays are
// topic-major, element [t * rs + p] with the row stride rs = n_pairs rounded
// up to a multiple of 64 (every topic row starts 512-B aligned for f64).
struct DevState {
    double* fmd;
    double* mmd;
    double* mfp;
    double* imd;
    int64_t* graft;
    int64_t* mtime;
    uint8_t* rflags;
    uint8_t* pflags;
    int64_t* expire;
    double* bp;
    const double* app;
    const uint32_t* ipg;  // 2 per pair: (observer, ip) group id | WL bit, or NONE
    uint32_t* ipcount;    // per group: number of present pairs carrying it
    double* score;
    const DevTopicParams* tp;
    uint64_t n_pairs;
    uint64_t rs;
    uint32_t n_topics;
};

constexpr uint8_t REC_IN_MESH = 0x01;
constexpr uint8_t REC_ACTIVE = 0x02;
constexpr uint8_t PAIR_PRESENT = 0x01;
constexpr uint8_t PAIR_CONNECTED = 0x02;
constexpr uint32_t IPG_NONE = 0xFFFFFFFFu;
constexpr uint32_t IPG_WL = 0x80000000u;  // whitelisted IP: counted, never penalised

// Sorted-by-observer event batch for the event kernel.
struct DevEvent {
    uint32_t kind;
    uint32_t topic;
    uint64_t pair;
    int64_t now_ns;
    int64_t arg;
};

}  // namespace gsx

// launchers (gsx_kernels.hip)
namespace gsx {
hipError_t launch_purge(const DevState& s, int64_t now, hipStream_t st);
hipError_t launch_refresh_score(const DevState& s, const DevPeerParams& pp, int64_t now, bool refresh,
                                hipStream_t st);
hipError_t launch_apply_events(const DevState& s, const DevPeerParams& pp, const DevEvent* ev,
                               const uint32_t* group_off, uint32_t n_groups, hipStream_t st);
hipError_t launch_recap(const DevState& s, uint32_t topic, double cap2, double cap3, hipStream_t st);
hipError_t launch_rebuild_ipcount(const DevState& s, uint32_t n_groups_ip, hipStream_t st);

struct DevSynthSpec {
    uint64_t seed;
    int64_t now;
    double fmd_max, mmd_max, mfp_max, imd_max;
    double p_in_mesh;
    int64_t graft_window;
    double bp_max, p_disc, p_abs;
    int64_t expire_jitter;
    uint32_t sybil_first;
};
hipError_t launch_synthesize(const DevState& s, const int32_t* col, const DevSynthSpec& spec, hipStream_t st);
}  // namespace gsx
