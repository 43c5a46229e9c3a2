// gsx_propagate.hip — message propagation over the overlay (A13-A14).
//
// Bit-sliced, pull-based frontier expansion: messages travel in 64-message
// words; per node and word the engine keeps `seen` and the current frontier
// as u64 masks.  One launch per hop: thread u walks its own pairs (u -> v) in
// ascending neighbour order and pulls v's frontier word through the reverse
// pair (v -> u) — its eligibility byte, v's "first got it from u" mask and
// the origin mask — so the first deliverer of every new message is the
// lowest-indexed sender of that hop without atomics, and every per-receiver
// word is written by exactly one thread.  Router semantics: floodsub.go:76-100,
// gossipsub.go:943-1013, randomsub.go:99-160; dedup: pubsub.go:919-936,
// 1046-1090.  Integer/bit work only: HBM/L2 bound, no MFMA, no LDS.
#include "gsx_ops.h"

namespace gsx {

// Eligibility of every pair (v -> u) for this call (topic, router, scores).
__global__ __launch_bounds__(256) void k_prop_fwd(PropState ps, DevState s) {
    const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (r >= s.n_pairs) return;
    const uint8_t pf = s.pflags[r];
    uint8_t out = 0;
    if ((pf & (PAIR_PRESENT | PAIR_CONNECTED)) == (PAIR_PRESENT | PAIR_CONNECTED)) {  // in ps.topics[topic]
        const uint8_t ef = ps.eflags[r];
        if (ps.router == ROUTER_FLOODSUB) {  // every topic peer (floodsub.go:81-90)
            out = FWD_FORWARD | FWD_PUBLISH;
        } else if (ps.router == ROUTER_RANDOMSUB) {  // FloodSub peers always, the rest by draw (randomsub.go:112-143)
            out = (ef & EDGE_FLOODSUB) ? (FWD_FORWARD | FWD_PUBLISH) : FWD_RSUB_CAND;
        } else {  // gossipsub
            const bool direct = ef & EDGE_DIRECT;
            const bool above = s.score[r] >= ps.publish_threshold;
            bool fwd = direct || (!(ef & EDGE_GOSSIPSUB) && above);  // direct + floodsub peers (:962-975)
            if (!fwd && ps.topic < s.n_topics)                       // mesh peers (:977-999)
                fwd = s.rflags[flag_index(r, ps.topic, s.n_topics)] & REC_IN_MESH;
            const bool pub = ps.flood_publish ? (direct || above) : fwd;  // flood publish (:953-960)
            out = (fwd ? FWD_FORWARD : 0) | (pub ? FWD_PUBLISH : 0);
        }
    }
    ps.fwd[r] = out;
}

// Sources: seen / frontier / origin bits and hop 0 (the local publish).
__global__ __launch_bounds__(256) void k_prop_init(PropState ps, uint64_t* front) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= ps.n_msgs) return;
    const uint32_t src = ps.msgs[k].source;
    const size_t i = (size_t)(k / 64) * ps.n_nodes + src;
    const unsigned long long bit = 1ull << (k % 64);
    atomicOr((unsigned long long*)&ps.origin[i], bit);
    atomicOr((unsigned long long*)&ps.seen[i], bit);
    atomicOr((unsigned long long*)&front[i], bit);
    ps.hop[(size_t)k * ps.n_nodes + src] = 0;
}

// ---- RandomSub's draw: the canonical RNG with tag 7 (gsx_ops.h) ----------
constexpr uint64_t TAG_RANDOMSUB = 7;

// For every frontier vertex v and message m of this hop (randomsub.go:112-143):
// candidates = its non-FloodSub topic peers except `from` and the origin, in
// ascending order; above RandomSubD they are shuffled (shufflePeers,
// gossipsub.go:1890-1895) and the first max(6, ceil(sqrt(size))) kept.  The
// kept pairs get message m's bit in `sel`.
__global__ __launch_bounds__(64) void k_rsub_select(PropState ps, const uint64_t* __restrict__ front) {
    const uint32_t v = blockIdx.x * 64u + threadIdx.x;
    if (v >= ps.n_nodes) return;
    const int64_t r0 = ps.row_ptr[v], r1 = ps.row_ptr[v + 1];
    uint32_t cand[RSUB_MAX_DEG];
    for (uint32_t w = 0; w < ps.n_words; ++w) {
        uint64_t f = front[(size_t)w * ps.n_nodes + v];
        while (f) {
            const int b = __builtin_ctzll(f);
            f &= f - 1;
            const uint32_t k = w * 64 + b;
            const uint32_t origin = ps.msgs[k].source;
            int n = 0;
            for (int64_t r = r0; r < r1 && n < RSUB_MAX_DEG; ++r) {
                if (!(ps.fwd[r] & FWD_RSUB_CAND)) continue;
                if ((uint32_t)ps.col[r] == origin) continue;
                if (ps.from_mask[(size_t)w * ps.n_pairs + r] & (1ull << b)) continue;  // u == from
                cand[n++] = (uint32_t)r;
            }
            int keep = n;
            if (n > RANDOMSUB_D) {
                int target = RANDOMSUB_D;
                if ((int)ps.rsub_sqrt > target) target = (int)ps.rsub_sqrt;
                if (target > n) target = n;
                Rng g{ps.seed, TAG_RANDOMSUB, v, ps.msgs[k].msg_id << 16, 0};
                g.shuffle(cand, n);
                keep = target;
            }
            for (int i = 0; i < keep; ++i) ps.sel[(size_t)w * ps.n_pairs + cand[i]] |= 1ull << b;
        }
    }
}

// ---- one hop ----------------------------------------------------------------
// `front` holds the messages each vertex first received at hop h-1; `nxt`
// receives those first received now.
__global__ __launch_bounds__(256) void k_prop_hop(PropState ps, uint32_t h, const uint64_t* __restrict__ front,
                                                  uint64_t* __restrict__ nxt) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    if (h > 1 && ps.stats[STAT_HOP0 + h - 1] == 0) {  // nothing arrived last hop: the frontier is empty
        if (u < ps.n_nodes)
            for (uint32_t w = 0; w < ps.n_words; ++w) nxt[(size_t)w * ps.n_nodes + u] = 0;
        return;
    }
    unsigned long long n_new = 0, n_dup = 0;
    if (u < ps.n_nodes) {
        const int64_t q0 = ps.row_ptr[u], q1 = ps.row_ptr[u + 1];
        for (uint32_t w = 0; w < ps.n_words; ++w) {
            const size_t wn = (size_t)w * ps.n_nodes, wp = (size_t)w * ps.n_pairs;
            const uint64_t seen = ps.seen[wn + u];
            const uint64_t mine = ps.origin[wn + u];  // never sent back to its origin
            uint64_t acc = 0;
            for (int64_t q = q0; q < q1; ++q) {  // ascending sender index
                const uint32_t r = ps.rev[q];    // the pair (v -> u)
                if (r == NO_PAIR) continue;
                const uint32_t v = (uint32_t)ps.col[q];
                const uint64_t f = front[wn + v];
                if (!f) continue;
                const uint8_t fw = ps.fwd[r];
                uint64_t elig;
                if ((fw & (FWD_FORWARD | FWD_PUBLISH)) == (FWD_FORWARD | FWD_PUBLISH)) elig = ~0ull;
                else if (fw & (FWD_FORWARD | FWD_PUBLISH)) {
                    const uint64_t own = ps.origin[wn + v];  // messages v published itself
                    elig = (fw & FWD_FORWARD) ? ~own : own;
                } else elig = 0;
                if (ps.sel) elig |= ps.sel[wp + r];
                const uint64_t c = f & elig & ~mine & ~ps.from_mask[wp + r];  // not back to v's `from`
                if (!c) continue;
                const uint64_t newb = c & ~seen & ~acc;
                const uint64_t dup_now = c & acc;    // first received this hop from a lower sender
                const uint64_t dup_old = c & seen;   // first received at an earlier hop
                acc |= newb;
                if (newb) ps.from_mask[wp + q] |= newb;  // u first got these from v
                n_new += __popcll(newb);
                n_dup += __popcll(dup_now) + __popcll(dup_old);
                if (ps.credit && (dup_now | dup_old)) {
                    // DuplicateMessage -> markDuplicateMessageDelivery with the
                    // record validated at u's first receipt (score.go:806-809, 965)
                    uint32_t k = __popcll(dup_now);
                    if (ps.all_dups_in_window) {
                        k += __popcll(dup_old);
                    } else {
                        uint64_t d = dup_old;
                        while (d) {
                            const int b = __builtin_ctzll(d);
                            d &= d - 1;
                            const int64_t h0 = ps.hop[(size_t)(w * 64 + b) * ps.n_nodes + u];
                            if (((int64_t)h - h0) * ps.hop_latency <= ps.window) ++k;
                        }
                    }
                    ps.dupcnt[q] += k;
                }
            }
            nxt[wn + u] = acc;
            if (acc) {
                ps.seen[wn + u] = seen | acc;
                uint64_t a = acc;
                while (a) {
                    const int b = __builtin_ctzll(a);
                    a &= a - 1;
                    ps.hop[(size_t)(w * 64 + b) * ps.n_nodes + u] = (uint8_t)h;
                }
            }
        }
    }
    // counters: wave reduction, then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        n_new += __shfl_down(n_new, off, 64);
        n_dup += __shfl_down(n_dup, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (n_new) atomicAdd((unsigned long long*)&ps.stats[STAT_HOP0 + h], n_new);
        if (n_dup) atomicAdd((unsigned long long*)&ps.stats[STAT_DUPS], n_dup);
    }
}

// ---- P2/P3 credits ------------------------------------------------------------
// Receiver pair q = (u -> v): k1 first receipts from v, k2 duplicates inside
// the window.  markFirstMessageDelivery: fmd k1 steps of +1 then cap, mmd too
// when in mesh; markDuplicateMessageDelivery: mmd k2 more steps when in mesh
// (score.go:912-974).  All steps are identical, so their order does not matter;
// they are applied one by one because +1 on a fractional counter rounds.
__global__ __launch_bounds__(256) void k_prop_credit(PropState ps, DevState s) {
    const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= s.n_pairs) return;
    if (!(s.pflags[q] & PAIR_PRESENT) || ps.topic >= s.n_topics) return;
    const DevTopicParams& tp = s.tp[ps.topic];
    if (!tp.scored) return;
    uint32_t k1 = 0;
    for (uint32_t w = 0; w < ps.n_words; ++w) k1 += __popcll(ps.from_mask[(size_t)w * ps.n_pairs + q]);
    const uint32_t k2 = ps.dupcnt[q];
    if (k1 == 0 && k2 == 0) return;
    const size_t b = rec_index(q, ps.topic, s.n_topics, FMD);
    double f = s.rec[b + FMD * TILE];
    for (uint32_t i = 0; i < k1; ++i) {
        f = f + 1;
        if (f > tp.cap2) f = tp.cap2;
    }
    s.rec[b + FMD * TILE] = f;
    if (!(s.rflags[flag_index(q, ps.topic, s.n_topics)] & REC_IN_MESH)) return;
    double m = s.rec[b + MMD * TILE];
    for (uint32_t i = 0; i < k1 + k2; ++i) {
        m = m + 1;
        if (m > tp.cap3) m = tp.cap3;
    }
    s.rec[b + MMD * TILE] = m;
}

// First deliverer per (message, node) from the per-pair "first got it from" masks.
__global__ __launch_bounds__(256) void k_prop_from(PropState ps, int32_t* __restrict__ first_from) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    if (u >= ps.n_nodes) return;
    for (uint32_t w = 0; w < ps.n_words; ++w)
        for (int64_t q = ps.row_ptr[u]; q < ps.row_ptr[u + 1]; ++q) {
            uint64_t bits = ps.from_mask[(size_t)w * ps.n_pairs + q];
            while (bits) {
                const int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                const uint32_t k = w * 64 + b;
                if (k < ps.n_msgs) first_from[(size_t)k * ps.n_nodes + u] = ps.col[q];
            }
        }
}

// ---- launchers ----------------------------------------------------------------
static inline unsigned nblk(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_prop_from(const PropState& ps, int32_t* first_from, hipStream_t st) {
    if (ps.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_from, dim3(nblk(ps.n_nodes, 256)), dim3(256), 0, st, ps, first_from);
    return hipGetLastError();
}

hipError_t launch_prop_fwd(const PropState& ps, const DevState& s, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_fwd, dim3(nblk(s.n_pairs, 256)), dim3(256), 0, st, ps, s);
    return hipGetLastError();
}
hipError_t launch_prop_init(const PropState& ps, uint64_t* front, hipStream_t st) {
    if (ps.n_msgs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_init, dim3(nblk(ps.n_msgs, 256)), dim3(256), 0, st, ps, front);
    return hipGetLastError();
}
hipError_t launch_prop_hop(const PropState& ps, uint32_t h, const uint64_t* front, uint64_t* nxt, hipStream_t st) {
    if (ps.n_nodes == 0) return hipSuccess;
    if (ps.sel) hipLaunchKernelGGL(k_rsub_select, dim3(nblk(ps.n_nodes, 64)), dim3(64), 0, st, ps, front);
    hipLaunchKernelGGL(k_prop_hop, dim3(nblk(ps.n_nodes, 256)), dim3(256), 0, st, ps, h, front, nxt);
    return hipGetLastError();
}
hipError_t launch_prop_credit(const PropState& ps, const DevState& s, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_credit, dim3(nblk(s.n_pairs, 256)), dim3(256), 0, st, ps, s);
    return hipGetLastError();
}

}  // namespace gsx
