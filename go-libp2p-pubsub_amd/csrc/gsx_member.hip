// Topic membership: who has joined which topic (gs.mesh /
// gs.p.topics), the fanout of publishers that have not joined
// (gossipsub.go:981-998, 1517-1554) and Join / Leave (:1015-1082).
//
// Every kernel here is one lane per node or per (node, topic) entry, walking
// the node's own row; candidate lists are staged in `scratch` over the row's
// own pair range (each row belongs to one lane of a launch), shuffled with
// the canonical draws and truncated, as getPeers does (:1852-1872).
#include "gsx_device.h"
#include "gsx_ops.h"

namespace gsx {

namespace {

// getPeers' candidates of (v, t) into scratch[r0 ..): mesh-capable topic
// peers, not direct, score >= ref, optionally not in v's fanout; returns count
__device__ int member_candidates(const DevState& s, const HbState& h, uint32_t* scratch, int64_t r0, int64_t r1,
                                 uint32_t t, double ref, bool skip_fanout) {
    int n = 0;
    for (int64_t r = r0; r < r1; ++r) {
        const uint8_t ef = h.eflags[r];
        if ((s.pflags[r] & (PAIR_PRESENT | PAIR_CONNECTED)) != (PAIR_PRESENT | PAIR_CONNECTED)) continue;
        if (!topic_peer(h.psub, (uint64_t)r, t) || !(ef & EDGE_GOSSIPSUB) || (ef & EDGE_DIRECT)) continue;
        if (skip_fanout && ((h.fanout[r] >> t) & 1)) continue;
        if (!(s.score[r] >= ref)) continue;
        scratch[r0 + n++] = (uint32_t)(r - r0);
    }
    return n;
}

__device__ void set_fanout_bits(const HbState& h, const uint32_t* scratch, int64_t r0, int k, uint32_t t) {
    for (int i = 0; i < k; ++i) {
        uint64_t* w = h.fanout + r0 + scratch[r0 + i];
        *w = *w | (1ull << t);
    }
}

}  // namespace

__global__ __launch_bounds__(256) void k_psub(const int32_t* __restrict__ col, const uint64_t* __restrict__ sub,
                                              uint64_t* __restrict__ psub, uint64_t n) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x; r < n; r += (uint64_t)gridDim.x * 256u)
        psub[r] = sub[(uint32_t)col[r]];
}

// Publish at a source that has not joined t (:981-998): an empty fanout is
// filled with getPeers(D) of non-direct peers with score >= PublishThreshold
// (draws h(seed, 10, source, t << 24 | k)); lastpub = now.
__global__ __launch_bounds__(64) void k_fanout_pick(DevState s, HbState h, const uint32_t* __restrict__ sources,
                                                    uint32_t n_src, uint32_t t, int64_t now, uint64_t seed,
                                                    double thr, uint32_t* scratch) {
    for (uint32_t i = blockIdx.x * 64u + threadIdx.x; i < n_src; i += gridDim.x * 64u) {
        const uint32_t v = sources[i];
        const int64_t r0 = h.row_ptr[v], r1 = h.row_ptr[v + 1];
        bool empty = true;
        for (int64_t r = r0; r < r1 && empty; ++r) empty = !((h.fanout[r] >> t) & 1);
        if (empty) {
            int n = member_candidates(s, h, scratch, r0, r1, t, thr, false);
            Rng g{seed, TAG_FANOUT, (uint64_t)v, (uint64_t)t << 24, 0};
            g.shuffle(scratch + r0, n);
            if (n > h.gp.d) n = h.gp.d;
            set_fanout_bits(h, scratch, r0, n, t);
            if (n > 0) h.fan_has[v] |= 1ull << t;
        }
        h.lastpub[(size_t)v * s.n_topics + t] = now;
    }
}

// The heartbeat's fanout of topic t (:1517-1554), after every joined topic's
// maintenance: expiry after FanoutTTL, peers no longer in the topic or below
// PublishThreshold (heartbeat-start scores) dropped, topped up to D with the
// draws h(seed, 8, node, tick << 32 | t << 24 | 1 << 23 | k); the node's
// fanout gossip continues the same stream (rngk).
__global__ __launch_bounds__(64) void k_hb_fanout(DevState s, HbState h, uint32_t t, int64_t ttl, uint32_t* scratch) {
    const uint32_t T = s.n_topics;
    for (uint32_t v = blockIdx.x * 64u + threadIdx.x; v < h.n_nodes; v += gridDim.x * 64u) {
        const int64_t r0 = h.row_ptr[v], r1 = h.row_ptr[v + 1];
        int64_t* lp = h.lastpub + (size_t)v * T + t;
        if (*lp != 0 && *lp + ttl < h.now) {
            for (int64_t r = r0; r < r1; ++r) h.fanout[r] &= ~(1ull << t);
            h.fan_has[v] &= ~(1ull << t);
            *lp = 0;
        }
        if (!((h.fan_has[v] >> t) & 1)) continue;
        int have = 0;
        for (int64_t r = r0; r < r1; ++r) {
            if (!((h.fanout[r] >> t) & 1)) continue;
            const bool in = (s.pflags[r] & (PAIR_PRESENT | PAIR_CONNECTED)) == (PAIR_PRESENT | PAIR_CONNECTED) &&
                            topic_peer(h.psub, (uint64_t)r, t);
            if (!in || s.score[r] < h.publish_threshold) h.fanout[r] &= ~(1ull << t);
            else ++have;
        }
        Rng g{h.seed, TAG_HEARTBEAT, (uint64_t)h.node_lo + v, (h.tick << 32) | ((uint64_t)t << 24) | (1ull << 23), 0};
        if (have < h.gp.d) {
            int n = member_candidates(s, h, scratch, r0, r1, t, h.publish_threshold, true);
            g.shuffle(scratch + r0, n);
            if (n > h.gp.d - have) n = h.gp.d - have;
            set_fanout_bits(h, scratch, r0, n, t);
        }
        h.rngk[(size_t)t * h.n_nodes + v] = g.k;
    }
}

// Join / Leave of (node, topic) entries, one lane each; the host launches
// the entries of one node in separate launches (they share the node's row).
// Join (:1015-1064): the mesh from the fanout (negative scores dropped,
// topped up to D) or getPeers(D); each mesh peer gets tracer.Graft and a
// GRAFT.  Leave (:1066-1082): each mesh peer gets tracer.Prune and a PRUNE.
// The subscriptions themselves were announced by the host before.
__global__ __launch_bounds__(64) void k_join(DevState s, HbState h, const uint32_t* __restrict__ nodes,
                                             const uint32_t* __restrict__ topics, uint32_t n, uint32_t leave,
                                             uint32_t* scratch) {
    uint64_t grafts = 0, prunes = 0;
    for (uint32_t i = blockIdx.x * 64u + threadIdx.x; i < n; i += gridDim.x * 64u) {
        const uint32_t v = nodes[i], t = topics[i];
        const int64_t r0 = h.row_ptr[v], r1 = h.row_ptr[v + 1];
        if (leave) {
            for (int64_t r = r0; r < r1; ++r) {
                if (!((s.pflags[r] & PAIR_PRESENT) && (s.rflags[flag_index(r, t, s.n_topics)] & REC_IN_MESH))) continue;
                ev_prune(s, (uint64_t)r, t);
                atomicOr((unsigned long long*)&h.ctl[2 * (size_t)r + 1], 1ull << t);
                const uint32_t q = h.rev[r];
                if (q != NO_PAIR && !(q & HALO)) h.inbox[q] = 1;
                h.dirty[r] = 1;
                ++prunes;
            }
            continue;
        }
        Rng g{h.seed, TAG_JOIN, (uint64_t)v, (uint64_t)t << 24, 0};
        const int D = h.gp.d;
        if ((h.fan_has[v] >> t) & 1) {
            int have = 0;
            for (int64_t r = r0; r < r1; ++r) {
                if (!((h.fanout[r] >> t) & 1)) continue;
                if (s.score[r] < 0) h.fanout[r] &= ~(1ull << t);
                else ++have;
            }
            if (have < D) {
                int k = member_candidates(s, h, scratch, r0, r1, t, 0.0, true);
                g.shuffle(scratch + r0, k);
                if (k > D - have) k = D - have;
                set_fanout_bits(h, scratch, r0, k, t);
            }
        } else {
            int k = member_candidates(s, h, scratch, r0, r1, t, 0.0, false);
            g.shuffle(scratch + r0, k);
            if (k > D) k = D;
            set_fanout_bits(h, scratch, r0, k, t);  // (the new mesh, staged in the fanout bits)
        }
        for (int64_t r = r0; r < r1; ++r) {
            if (!((h.fanout[r] >> t) & 1)) continue;
            h.fanout[r] &= ~(1ull << t);
            ev_graft(s, (uint64_t)r, t, h.now);
            atomicOr((unsigned long long*)&h.ctl[2 * (size_t)r], 1ull << t);
            const uint32_t q = h.rev[r];
            if (q != NO_PAIR && !(q & HALO)) h.inbox[q] = 1;
            h.dirty[r] = 1;
            ++grafts;
        }
        h.fan_has[v] &= ~(1ull << t);
        h.lastpub[(size_t)v * s.n_topics + t] = 0;
    }
    unsigned long long c[2] = {grafts, prunes};
#pragma unroll
    for (int k = 0; k < 2; ++k)
        for (int off = 32; off > 0; off >>= 1) c[k] += __shfl_xor(c[k], off, 64);
    if (threadIdx.x == 0) {
        if (c[0]) atomicAdd(&h.stats[HB_GRAFTS], c[0]);
        if (c[1]) atomicAdd(&h.stats[HB_PRUNES], c[1]);
    }
}

static inline unsigned mb_blocks(uint64_t n, unsigned bs, unsigned cap) {
    const uint64_t b = (n + bs - 1) / bs;
    return (unsigned)(b < cap ? (b ? b : 1) : cap);
}

hipError_t launch_psub(const int32_t* col, const uint64_t* sub, uint64_t* psub, uint64_t n_pairs, hipStream_t st) {
    if (n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_psub, dim3(mb_blocks(n_pairs, 256, 4096)), dim3(256), 0, st, col, sub, psub, n_pairs);
    return hipGetLastError();
}

hipError_t launch_fanout_pick(const DevState& s, const HbState& h, const uint32_t* sources, uint32_t n_src,
                              uint32_t topic, int64_t now, uint64_t seed, double thr, hipStream_t st) {
    if (n_src == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fanout_pick, dim3(mb_blocks(n_src, 64, 4096)), dim3(64), 0, st, s, h, sources, n_src, topic,
                       now, seed, thr, h.mscratch);
    return hipGetLastError();
}

hipError_t launch_hb_fanout(const DevState& s, const HbState& h, uint32_t t, hipStream_t st) {
    if (h.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_fanout, dim3(mb_blocks(h.n_nodes, 64, 8192)), dim3(64), 0, st, s, h, t, h.gp.fanout_ttl,
                       h.mscratch);
    return hipGetLastError();
}

hipError_t launch_join(const DevState& s, const HbState& h, const uint32_t* nodes, const uint32_t* topics,
                       uint32_t n, uint32_t leave, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_join, dim3(mb_blocks(n, 64, 4096)), dim3(64), 0, st, s, h, nodes, topics, n, leave, h.mscratch);
    return hipGetLastError();
}

}  // namespace gsx
