// gsx_ops.h — device functions shared by the kernels: the scorer's arithmetic
// (score.go), its tracer updates, and the canonical RNG.  Header-only so every
// kernel file inlines them.  gfx950 only.
#pragma once

#include "gsx_device.h"

namespace gsx {

// ---- score() pieces (score.go:258-381) --------------------------------------

// P6, ipColocationFactor (score.go:337-381) from the per-(observer, IP) count
// of present pairs (the size of ps.peerIPs[ip]).
__device__ __forceinline__ double ip_colocation(const DevState& s, const DevPeerParams& pp, uint64_t p) {
    const uint2 g = reinterpret_cast<const uint2*>(s.ipg)[p];
    double result = 0.0;
    const uint32_t gs[2] = {g.x, g.y};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t id = gs[k];
        if (id == IPG_NONE || (id & IPG_WL)) continue;  // no IP / whitelisted (:346-367)
        const int64_t peers_in_ip = (int64_t)s.ipcount[id];
        if (peers_in_ip > pp.thr6) {
            const double surpluss = (double)(peers_in_ip - pp.thr6);
            result += surpluss * surpluss;
        }
    }
    return result;
}

// The per-pair tail of score(): topic cap, P5, P6, P7 (score.go:315-332).
__device__ __forceinline__ double score_tail(const DevState& s, const DevPeerParams& pp, uint64_t p, double score,
                                             double bp) {
    if (pp.topic_score_cap > 0 && score > pp.topic_score_cap) score = pp.topic_score_cap;
    const double p5 = s.app[p];
    score += p5 * pp.w5;
    // With w6 == 0 the term is +-0 and score (never -0) is unchanged: skip the gather.
    if (pp.w6 != 0.0) {
        const double p6 = ip_colocation(s, pp, p);
        score += p6 * pp.w6;
    }
    if (bp > pp.thr7) {
        const double excess = bp - pp.thr7;
        const double p7 = excess * excess;
        score += p7 * pp.w7;
    }
    return score;
}

// One topic's contribution, score.go:276-311.
__device__ __forceinline__ double topic_score(const DevTopicParams& tp, uint8_t fl, int64_t mesh_time, double fmd,
                                              double mmd, double mfp, double imd) {
    double ts = 0.0;
    if (fl & REC_IN_MESH) {  // P1, integer Duration division (:280)
        double p1 = (double)(mesh_time / tp.q1);
        if (p1 > tp.cap1) p1 = tp.cap1;
        ts += p1 * tp.w1;
    }
    const double p2 = fmd;  // P2
    ts += p2 * tp.w2;
    if (fl & REC_ACTIVE) {  // P3
        if (mmd < tp.thr3) {
            const double deficit = tp.thr3 - mmd;
            const double p3 = deficit * deficit;
            ts += p3 * tp.w3;
        }
    }
    const double p3b = mfp;  // P3b
    ts += p3b * tp.w3b;
    const double p4 = (imd * imd);  // P4
    ts += p4 * tp.w4;
    return ts * tp.topic_weight;
}

// meshTime of a stored record: FRESH (grafted, not refreshed since) -> 0,
// else the value the last refresh computed (score.go:544-546).
__device__ __forceinline__ int64_t mesh_time_of(const DevState& s, uint8_t fl, uint64_t p, uint32_t t) {
    if (!(fl & REC_IN_MESH) || (fl & REC_FRESH)) return 0;
    const int64_t graft = reinterpret_cast<const int64_t*>(s.rec)[rec_index(p, t, s.n_topics, GRAFT)];
    return s.last_refresh - graft;
}

// score(p) from the stored state, no refresh (RemovePeer, score.go:615).
__device__ __forceinline__ double eval_pair(const DevState& s, const DevPeerParams& pp, uint64_t p) {
    if (!(s.pflags[p] & PAIR_PRESENT)) return 0.0;
    double score = 0.0;
    for (uint32_t t = 0; t < s.n_topics; ++t) {
        const DevTopicParams& tp = s.tp[t];
        if (!tp.scored) continue;
        const uint8_t fl = s.rflags[flag_index(p, t, s.n_topics)];
        const size_t b = rec_index(p, t, s.n_topics, FMD);
        score += topic_score(tp, fl, mesh_time_of(s, fl, p, t), s.rec[b], s.rec[b + MMD * TILE],
                             s.rec[b + MFP * TILE], s.rec[b + IMD * TILE]);
    }
    return score_tail(s, pp, p, score, s.bp[p]);
}

// k steps of "x = x + 1; if x > cap { x = cap }" (score.go:925-938, 970-973),
// bit for bit, in O(log k): x only ever grows until it is capped, and it
// stays capped, so the result is min(cap, k sequential +1s); within one
// binade [2^e, 2^(e+1)) with 0 <= e <= 52 adding an integer is exact, so only
// the step that crosses into the next binade rounds.  Below 1 (and in the
// never-reached range >= 2^52) the steps are taken one by one.
__device__ __forceinline__ double add_ones_capped(double x, uint32_t k, double cap) {
    while (k && !(x >= 1.0 && x < 4503599627370496.0)) {  // [1, 2^52)
        x = x + 1;
        --k;
        if (x > cap) return cap;
    }
    while (k) {
        const unsigned long long bits = (unsigned long long)__double_as_longlong(x);
        const double top = __longlong_as_double((long long)((((bits >> 52) & 0x7FF) + 1) << 52));  // 2^(e+1)
        const double gap = top - x;  // exact (Sterbenz)
        const double s = ceil(gap) - 1;  // steps that stay below top
        if (s >= (double)k) {
            x = x + (double)k;
            k = 0;
        } else {
            x = x + s;
            k -= (uint32_t)s;
            x = x + 1;  // the crossing step rounds
            --k;
        }
        if (x > cap) return cap;
        if (!(x < 4503599627370496.0))
            while (k) {
                x = x + 1;
                --k;
                if (x > cap) return cap;
            }
    }
    return x > cap ? cap : x;
}

// x *= decay; x = 0 if x < DecayToZero   (score.go:527-542, 553-556)
__device__ __forceinline__ double decay(double x, double d, double dtz) {
    x *= d;
    return x < dtz ? 0.0 : x;
}

// ---- tracer updates (score.go:588-974) -----------------------------------------

__device__ __forceinline__ void ipcount_add(const DevState& s, uint64_t p, int delta) {
    const uint2 g = reinterpret_cast<const uint2*>(s.ipg)[p];
    if (g.x != IPG_NONE) s.ipcount[g.x & ~IPG_WL] += (uint32_t)delta;
    if (g.y != IPG_NONE && g.y != g.x) s.ipcount[g.y & ~IPG_WL] += (uint32_t)delta;
}

__device__ __forceinline__ bool scored_topic(const DevState& s, uint64_t p, uint32_t topic) {
    return (s.pflags[p] & PAIR_PRESENT) && topic < s.n_topics && s.tp[topic].scored;
}

__device__ inline void ev_add_peer(const DevState& s, uint64_t p) {  // AddPeer :588-602
    const uint8_t st = s.pflags[p];
    if (!(st & PAIR_PRESENT)) {  // new peerStats{topics: {}}
        for (uint32_t t = 0; t < s.n_topics; ++t) {
            const size_t b = rec_index(p, t, s.n_topics, FMD);
            for (int f = 0; f < NFIELD; ++f) s.rec[b + f * TILE] = 0.0;
            s.rflags[flag_index(p, t, s.n_topics)] = 0;
        }
        s.bp[p] = 0.0;
        s.expire[p] = 0;
        ipcount_add(s, p, +1);  // setIPs
    }
    s.pflags[p] = PAIR_PRESENT | PAIR_CONNECTED;
}

__device__ inline void ev_remove_peer(const DevState& s, const DevPeerParams& pp, uint64_t p, int64_t now) {  // :604-637
    const uint8_t st = s.pflags[p];
    if (!(st & PAIR_PRESENT)) return;
    if (eval_pair(s, pp, p) > 0) {  // positive score: forget the peer
        ipcount_add(s, p, -1);
        s.pflags[p] = 0;
        return;
    }
    for (uint32_t t = 0; t < s.n_topics; ++t) {
        const DevTopicParams& tp = s.tp[t];
        if (!tp.scored) continue;
        const size_t b = rec_index(p, t, s.n_topics, FMD);
        const size_t fi = flag_index(p, t, s.n_topics);
        s.rec[b + FMD * TILE] = 0.0;
        const uint8_t fl = s.rflags[fi];
        const double threshold = tp.thr3;
        const double mmd = s.rec[b + MMD * TILE];
        if ((fl & REC_IN_MESH) && (fl & REC_ACTIVE) && mmd < threshold) {
            const double deficit = threshold - mmd;
            s.rec[b + MFP * TILE] = s.rec[b + MFP * TILE] + deficit * deficit;
        }
        s.rflags[fi] = fl & ~(REC_IN_MESH | REC_FRESH);
    }
    s.pflags[p] = PAIR_PRESENT;
    s.expire[p] = now + pp.retain_ns;
}

__device__ inline void ev_graft(const DevState& s, uint64_t p, uint32_t topic, int64_t now) {  // :642-660
    if (!scored_topic(s, p, topic)) return;
    reinterpret_cast<int64_t*>(s.rec)[rec_index(p, topic, s.n_topics, GRAFT)] = now;
    s.rflags[flag_index(p, topic, s.n_topics)] = REC_IN_MESH | REC_FRESH;  // meshTime = 0, not active
}

__device__ inline void ev_prune(const DevState& s, uint64_t p, uint32_t topic) {  // :662-684
    if (!scored_topic(s, p, topic)) return;
    const size_t b = rec_index(p, topic, s.n_topics, FMD);
    const size_t fi = flag_index(p, topic, s.n_topics);
    const uint8_t fl = s.rflags[fi];
    const double threshold = s.tp[topic].thr3;
    const double mmd = s.rec[b + MMD * TILE];
    if ((fl & REC_ACTIVE) && mmd < threshold) {
        const double deficit = threshold - mmd;
        s.rec[b + MFP * TILE] = s.rec[b + MFP * TILE] + deficit * deficit;
    }
    s.rflags[fi] = fl & ~(REC_IN_MESH | REC_FRESH);
}

__device__ inline void ev_first(const DevState& s, uint64_t p, uint32_t topic) {  // :912-939
    if (!scored_topic(s, p, topic)) return;
    const DevTopicParams& tp = s.tp[topic];
    const size_t b = rec_index(p, topic, s.n_topics, FMD);
    double f = s.rec[b + FMD * TILE] + 1;
    if (f > tp.cap2) f = tp.cap2;
    s.rec[b + FMD * TILE] = f;
    if (!(s.rflags[flag_index(p, topic, s.n_topics)] & REC_IN_MESH)) return;
    double m = s.rec[b + MMD * TILE] + 1;
    if (m > tp.cap3) m = tp.cap3;
    s.rec[b + MMD * TILE] = m;
}

__device__ inline void ev_mesh(const DevState& s, uint64_t p, uint32_t topic) {  // :944-974 (window checked by caller)
    if (!scored_topic(s, p, topic)) return;
    if (!(s.rflags[flag_index(p, topic, s.n_topics)] & REC_IN_MESH)) return;
    const size_t b = rec_index(p, topic, s.n_topics, MMD);
    double m = s.rec[b] + 1;
    if (m > s.tp[topic].cap3) m = s.tp[topic].cap3;
    s.rec[b] = m;
}

__device__ inline void ev_invalid(const DevState& s, uint64_t p, uint32_t topic) {  // :894-907
    if (!scored_topic(s, p, topic)) return;
    const size_t b = rec_index(p, topic, s.n_topics, IMD);
    s.rec[b] = s.rec[b] + 1;
}

__device__ inline void ev_penalty(const DevState& s, uint64_t p, int64_t count) {  // AddPenalty :384-398
    if (!(s.pflags[p] & PAIR_PRESENT)) return;
    s.bp[p] = s.bp[p] + (double)count;
}

// ---- counters --------------------------------------------------------------------
// Sums NV per-thread counters over a 256-thread block (wave shuffles, then
// LDS across the four waves) and adds each non-zero total to its global
// counter with ONE atomic per block.  Same-address atomics serialise at the
// memory side, so kernels that own counters run grid-stride over a bounded
// grid (COUNTER_GRID blocks) and reach this once per block, every thread.
constexpr unsigned COUNTER_GRID = 2048;

template <int NV>
__device__ __forceinline__ void block_count(unsigned long long (&v)[NV], unsigned long long* stats,
                                            const uint32_t (&slot)[NV]) {
    __shared__ unsigned long long part[NV][4];
#pragma unroll
    for (int i = 0; i < NV; ++i)
        for (int off = 32; off > 0; off >>= 1) v[i] += __shfl_down(v[i], off, 64);
    const unsigned wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) part[i][wave] = v[i];
    __syncthreads();
    if (threadIdx.x < NV) {
        const unsigned i = threadIdx.x;
        const unsigned long long t = part[i][0] + part[i][1] + part[i][2] + part[i][3];
        if (t) atomicAdd(&stats[slot[i]], t);
    }
}

// Appends to a shared list with ONE atomic per wave: the active lanes with
// `take` get consecutive slots in lane order (-> the lane's slot; callable in
// divergent code: the ballot and the broadcast see the active lanes only).  A
// per-lane atomicAdd on one counter serialises every append of the grid at
// one L2 channel.
__device__ __forceinline__ uint32_t wave_append(uint32_t* ctr, bool take) {
    const uint64_t b = __ballot(take);
    if (b == 0) return 0;
    const uint32_t lane = __lane_id();
    const int leader = __ffsll((long long)b) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(b));
    base = (uint32_t)__shfl((int)base, leader, 64);
    return base + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
}

// ---- canonical RNG ---------------------------------------------
__host__ __device__ __forceinline__ uint64_t smix(uint64_t z) {  // SplitMix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t h4(uint64_t seed, uint64_t tag, uint64_t a, uint64_t b) {
    return smix(seed + 0x9E3779B97F4A7C15ull * (1ull + smix(tag ^ smix(a ^ smix(b)))));
}
// math/rand's Int31n over Int31 draws h(seed, tag, vertex, base | k), standing
// in for the router's global rand source (gossipsub.go:1890-1895).
struct Rng {
    uint64_t seed, tag, vertex, base;
    uint32_t k;
    __host__ __device__ int32_t int31() { return (int32_t)(h4(seed, tag, vertex, base | k++) >> 33); }
    __host__ __device__ int32_t int31n(int32_t n) {
        if ((n & (n - 1)) == 0) return int31() & (n - 1);
        const int32_t max = (int32_t)((1u << 31) - 1 - (1u << 31) % (uint32_t)n);
        int32_t v = int31();
        while (v > max) v = int31();
        return v % n;
    }
    // shufflePeers: for i, j = Intn(i+1), swap
    template <typename T>
    __device__ void shuffle(T* a, int n) {
        for (int i = 0; i < n; ++i) {
            const int j = int31n(i + 1);
            const T x = a[i];
            a[i] = a[j];
            a[j] = x;
        }
    }
};

}  // namespace gsx
