// gsx_propagate.hip — message propagation over the overlay (A13-A14).
//
// Bit-sliced, pull-based frontier expansion: messages travel in 64-message
// words; per node the engine keeps `seen`, `origin` and the current frontier
// as node-major word rows ([node][word]), so one gather brings every word of
// a neighbour.  One launch per hop: thread u walks its own pairs (u -> v) in
// ascending neighbour order and pulls v's frontier row through the reverse
// pair (v -> u) — its eligibility byte (read through u's own pair, fwd_in),
// v's "first got it from u" row and the origin rows — so the first deliverer
// of every new message is the lowest-indexed sender of that hop without
// atomics, and every per-receiver word has exactly one writer.
//
// Range sharding (gsx.h, gsx_load_overlay_shard): a pair whose neighbour
// lives on another rank carries HALO | slot in rev[]; the neighbour's rank
// packs, per hop, exactly what v sends to u (frontier & eligibility & not
// back to its `from`) into the slot order the receiver asked for
// (k_prop_pack), the host exchanges the packed rows (RCCL all-to-all), and
// the hop kernel reads them from the halo buffer in place of the local
// gather.  Nothing else crosses shards: seen, hop, first deliverer and the
// P2/P3 credits all belong to the receiver.
//
// Router semantics: floodsub.go:76-100, gossipsub.go:943-1013,
// randomsub.go:99-160; dedup: pubsub.go:919-936, 1046-1090.  Integer/bit work
// only: HBM/L2 bound, no MFMA, no LDS.
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

// fwd_in[q] = fwd[rev[q]]: the receiver reads the sender's decision through
// its own pair index (coalesced) instead of gathering it every hop.
__global__ __launch_bounds__(256) void k_prop_fwd_in(PropState ps) {
    const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= ps.n_pairs) return;
    const uint32_t r = ps.rev[q];
    ps.fwd_in[q] = (r == NO_PAIR || (r & HALO)) ? 0 : ps.fwd[r];
}

// Sources on this shard: seen / frontier / origin bits and hop 0 (the local publish).
__global__ __launch_bounds__(256) void k_prop_init(PropState ps, uint64_t* front) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= ps.n_msgs) return;
    const uint32_t src = ps.msgs[k].source;
    if (src < ps.node_lo || src - ps.node_lo >= ps.n_nodes) return;
    const uint32_t u = src - ps.node_lo;
    const size_t i = (size_t)u * ps.n_words + k / 64;
    const unsigned long long bit = 1ull << (k % 64);
    atomicOr((unsigned long long*)&ps.origin[i], bit);
    atomicOr((unsigned long long*)&ps.seen[i], bit);
    atomicOr((unsigned long long*)&front[i], bit);
    ps.hop[(size_t)u * ps.n_words * 64 + k] = 0;
}

// What pair (v -> u) lets through for a sender frontier word f:
// FORWARD covers messages v received, PUBLISH the ones v published (own).
__device__ __forceinline__ uint64_t elig_word(uint8_t fw, uint64_t own) {
    const uint8_t m = fw & (FWD_FORWARD | FWD_PUBLISH);
    if (m == (FWD_FORWARD | FWD_PUBLISH)) return ~0ull;
    if (m == FWD_FORWARD) return ~own;
    if (m == FWD_PUBLISH) return own;
    return 0;
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
    const uint32_t W = ps.n_words;
    uint32_t cand[RSUB_MAX_DEG];
    for (uint32_t w = 0; w < W; ++w) {
        uint64_t f = front[(size_t)v * W + w];
        while (f) {
            const int b = __builtin_ctzll(f);
            f &= f - 1;
            const uint32_t k = w * 64 + b;
            const uint32_t origin = ps.msgs[k].source;
            int n = 0;
            for (int64_t r = r0; r < r1 && n < RSUB_MAX_DEG; ++r) {
                if (!(ps.fwd[r] & FWD_RSUB_CAND)) continue;
                if ((uint32_t)ps.col[r] == origin) continue;
                if (ps.from_mask[(size_t)r * W + w] & (1ull << b)) continue;  // u == from
                cand[n++] = (uint32_t)r;
            }
            int keep = n;
            if (n > RANDOMSUB_D) {
                int target = RANDOMSUB_D;
                if ((int)ps.rsub_sqrt > target) target = (int)ps.rsub_sqrt;
                if (target > n) target = n;
                Rng g{ps.seed, TAG_RANDOMSUB, (uint64_t)ps.node_lo + v, ps.msgs[k].msg_id << 16, 0};
                g.shuffle(cand, n);
                keep = target;
            }
            for (int i = 0; i < keep; ++i) ps.sel[(size_t)cand[i] * W + w] |= 1ull << b;
        }
    }
}

// ---- shard exchange: pack what each cross-shard pair (v -> u) sends ---------------
// One thread per send slot (the order the receiving rank asked for).  The
// receiver applies only its own origin mask; eligibility, RandomSub draws
// and the `from` exclusion are the sender's and are applied here.
__global__ __launch_bounds__(256) void k_prop_pack(PropState ps, const uint64_t* __restrict__ front,
                                                   uint64_t* __restrict__ send) {
    const uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint32_t W = ps.n_words;
    unsigned long long n_send = 0;
    if (j < ps.n_send) {
        uint64_t* out = send + j * W;
        const uint32_t r = ps.send_pair[j];
        if (r == NO_PAIR) {
            for (uint32_t w = 0; w < W; ++w) out[w] = 0;
        } else {
            const uint32_t v = ps.pair_obs[r];
            const uint8_t fw = ps.fwd[r];
            for (uint32_t w = 0; w < W; ++w) {
                const uint64_t f = front[(size_t)v * W + w];
                uint64_t c = 0;
                if (f) {
                    const uint64_t own = ps.origin[(size_t)v * W + w];
                    uint64_t el = elig_word(fw, own);
                    if (ps.sel) el |= ps.sel[(size_t)r * W + w];
                    c = f & el;
                    n_send += c != 0;
                    if (c) c &= ~ps.from_mask[(size_t)r * W + w];
                }
                out[w] = c;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) n_send += __shfl_down(n_send, off, 64);
    if ((threadIdx.x & 63) == 0 && n_send) atomicAdd((unsigned long long*)&ps.stats[STAT_EDGE_SENDS], n_send);
}

// ---- one hop ----------------------------------------------------------------
// `front` holds the messages each vertex first received at hop h-1; `nxt`
// receives those first received now.  CW words are processed per walk of
// u's pairs (a 64·CW-message chunk lives in registers).
template <int CW>
__device__ __forceinline__ void load_words(uint64_t (&d)[CW], const uint64_t* p) {
#pragma unroll
    for (int i = 0; i < CW; ++i) d[i] = p[i];
}

template <int CW>
__global__ __launch_bounds__(256) void k_prop_hop(PropState ps, uint32_t h, const uint64_t* __restrict__ front,
                                                  uint64_t* __restrict__ nxt) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    const uint32_t W = ps.n_words;
    if (!ps.sharded && h > 1 && ps.stats[STAT_HOP0 + h - 1] == 0) {  // nothing arrived last hop: empty frontier
        if (u < ps.n_nodes)
            for (uint32_t w = 0; w < W; ++w) nxt[(size_t)u * W + w] = 0;
        return;
    }
    unsigned long long n_new = 0, n_dup = 0, n_send = 0, n_vnew = 0;
    if (u < ps.n_nodes) {
        const int64_t q0 = ps.row_ptr[u], q1 = ps.row_ptr[u + 1];
        const size_t un = (size_t)u * W;
        const size_t hrow = un * 64;
        for (uint32_t w0 = 0; w0 < W; w0 += CW) {
            uint64_t seen[CW], mine[CW], acc[CW];
            load_words<CW>(seen, ps.seen + un + w0);
            load_words<CW>(mine, ps.origin + un + w0);  // never sent back to its origin
#pragma unroll
            for (int i = 0; i < CW; ++i) acc[i] = 0;
            for (int64_t q = q0; q < q1; ++q) {  // ascending sender index
                const uint32_t r = ps.rev[q];    // the pair (v -> u)
                if (r == NO_PAIR) continue;
                uint64_t c[CW];
                if (r & HALO) {  // remote sender: its rank packed exactly what it sends
                    load_words<CW>(c, ps.halo + (size_t)(r & ~HALO) * W + w0);
                } else {
                    const uint32_t v = (uint32_t)ps.col[q] - ps.node_lo;
                    uint64_t f[CW];
                    load_words<CW>(f, front + (size_t)v * W + w0);
                    uint64_t any = 0;
#pragma unroll
                    for (int i = 0; i < CW; ++i) any |= f[i];
                    if (!any) continue;
                    const uint8_t fw = ps.fwd_in[q];
                    uint64_t own[CW], sl[CW];
                    const uint8_t m = fw & (FWD_FORWARD | FWD_PUBLISH);
                    if (m == FWD_FORWARD || m == FWD_PUBLISH) load_words<CW>(own, ps.origin + (size_t)v * W + w0);
                    else
#pragma unroll
                        for (int i = 0; i < CW; ++i) own[i] = 0;
                    if (ps.sel) load_words<CW>(sl, ps.sel + (size_t)r * W + w0);
                    else
#pragma unroll
                        for (int i = 0; i < CW; ++i) sl[i] = 0;
                    uint64_t hit = 0;
#pragma unroll
                    for (int i = 0; i < CW; ++i) {
                        c[i] = f[i] & (elig_word(fw, own[i]) | sl[i]);
                        n_send += c[i] != 0;
                        hit |= c[i] & seen[i];
                    }
                    // Not back to v's `from` (floodsub.go:82, gossipsub.go:1007,
                    // randomsub.go:113).  Those messages reached v from u, so u
                    // has already seen them: the row is only needed when a
                    // duplicate is possible.
                    if (hit) {
                        uint64_t fm[CW];
                        load_words<CW>(fm, ps.from_mask + (size_t)r * W + w0);
#pragma unroll
                        for (int i = 0; i < CW; ++i) c[i] &= ~fm[i];
                    }
                }
                uint64_t any = 0;
#pragma unroll
                for (int i = 0; i < CW; ++i) {
                    c[i] &= ~mine[i];
                    any |= c[i];
                }
                if (!any) continue;
                uint32_t k = 0;
#pragma unroll
                for (int i = 0; i < CW; ++i) {
                    const uint64_t newb = c[i] & ~seen[i] & ~acc[i];
                    const uint64_t dup_now = c[i] & acc[i];  // first received this hop from a lower sender
                    const uint64_t dup_old = c[i] & seen[i];  // first received at an earlier hop
                    acc[i] |= newb;
                    if (newb) ps.from_mask[(size_t)q * W + w0 + i] |= newb;  // u first got these from v
                    n_new += __popcll(newb);
                    n_dup += __popcll(dup_now) + __popcll(dup_old);
                    if (ps.credit && (dup_now | dup_old)) {
                        // DuplicateMessage -> markDuplicateMessageDelivery with the
                        // record validated at u's first receipt (score.go:806-809, 965)
                        k += __popcll(dup_now);
                        if (ps.all_dups_in_window) {
                            k += __popcll(dup_old);
                        } else {
                            uint64_t d = dup_old;
                            while (d) {
                                const int b = __builtin_ctzll(d);
                                d &= d - 1;
                                const int64_t h0 = ps.hop[hrow + (size_t)(w0 + i) * 64 + b];
                                if (((int64_t)h - h0) * ps.hop_latency <= ps.window) ++k;
                            }
                        }
                    }
                }
                if (k) ps.dupcnt[q] += k;
            }
#pragma unroll
            for (int i = 0; i < CW; ++i) {
                nxt[un + w0 + i] = acc[i];
                if (acc[i]) {
                    ps.seen[un + w0 + i] = seen[i] | acc[i];
                    ++n_vnew;
                    uint64_t a = acc[i];
                    while (a) {
                        const int b = __builtin_ctzll(a);
                        a &= a - 1;
                        ps.hop[hrow + (size_t)(w0 + i) * 64 + b] = (uint8_t)h;
                    }
                }
            }
        }
    }
    // counters: wave reduction, then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        n_new += __shfl_down(n_new, off, 64);
        n_dup += __shfl_down(n_dup, off, 64);
        n_send += __shfl_down(n_send, off, 64);
        n_vnew += __shfl_down(n_vnew, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (n_new) atomicAdd((unsigned long long*)&ps.stats[STAT_HOP0 + h], n_new);
        if (n_dup) atomicAdd((unsigned long long*)&ps.stats[STAT_DUPS], n_dup);
        if (n_send) atomicAdd((unsigned long long*)&ps.stats[STAT_EDGE_SENDS], n_send);
        if (n_vnew) atomicAdd((unsigned long long*)&ps.stats[STAT_NEW_WORDS], n_vnew);
    }
}

// ---- P2/P3 credits ------------------------------------------------------------
// Per receiver pair q = (u -> v), add this call's first receipts from v (the
// popcount of its from row) and in-window duplicates to the pending counts.
__global__ __launch_bounds__(256) void k_prop_count(PropState ps) {
    const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= ps.n_pairs) return;
    uint32_t k1 = 0;
    for (uint32_t w = 0; w < ps.n_words; ++w) k1 += __popcll(ps.from_mask[(size_t)q * ps.n_words + w]);
    if (k1) ps.firstcnt[q] += k1;
}

// Fold pending counts: k1 first receipts, k2 duplicates inside the window.
// markFirstMessageDelivery: fmd k1 steps of +1 then cap, mmd too when in
// mesh; markDuplicateMessageDelivery: mmd k2 more steps when in mesh
// (score.go:912-974).  All steps are identical, so their order does not
// matter; they are applied one by one because +1 on a fractional counter rounds.
__global__ __launch_bounds__(256) void k_prop_fold(PropState ps, DevState s, const uint32_t* __restrict__ first,
                                                   const uint32_t* __restrict__ dup) {
    const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= s.n_pairs) return;
    if (!(s.pflags[q] & PAIR_PRESENT) || ps.topic >= s.n_topics) return;
    const DevTopicParams& tp = s.tp[ps.topic];
    if (!tp.scored) return;
    const uint32_t k1 = first[q];
    const uint32_t k2 = dup[q];
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

// First deliverer per (message, node) from the per-pair "first got it from" rows.
__global__ __launch_bounds__(256) void k_prop_from(PropState ps, int32_t* __restrict__ first_from) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    if (u >= ps.n_nodes) return;
    const uint32_t W = ps.n_words;
    for (int64_t q = ps.row_ptr[u]; q < ps.row_ptr[u + 1]; ++q)
        for (uint32_t w = 0; w < W; ++w) {
            uint64_t bits = ps.from_mask[(size_t)q * W + w];
            while (bits) {
                const int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                const uint32_t k = w * 64 + b;
                if (k < ps.n_msgs) first_from[(size_t)k * ps.n_nodes + u] = ps.col[q];
            }
        }
}

// [node][word*64] arrival hops -> the ABI's [message][node].
__global__ __launch_bounds__(256) void k_prop_hops_export(PropState ps, uint8_t* __restrict__ out) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    const uint32_t k = blockIdx.y;
    if (u >= ps.n_nodes) return;
    out[(size_t)k * ps.n_nodes + u] = ps.hop[(size_t)u * ps.n_words * 64 + k];
}

// ---- launchers ----------------------------------------------------------------
static inline unsigned nblk(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_prop_from(const PropState& ps, int32_t* first_from, hipStream_t st) {
    if (ps.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_from, dim3(nblk(ps.n_nodes, 256)), dim3(256), 0, st, ps, first_from);
    return hipGetLastError();
}
hipError_t launch_prop_hops_export(const PropState& ps, uint8_t* hop_mn, hipStream_t st) {
    if (ps.n_nodes == 0 || ps.n_msgs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_hops_export, dim3(nblk(ps.n_nodes, 256), ps.n_msgs), dim3(256), 0, st, ps, hop_mn);
    return hipGetLastError();
}
hipError_t launch_prop_fwd(const PropState& ps, const DevState& s, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_fwd, dim3(nblk(s.n_pairs, 256)), dim3(256), 0, st, ps, s);
    hipLaunchKernelGGL(k_prop_fwd_in, dim3(nblk(s.n_pairs, 256)), dim3(256), 0, st, ps);
    return hipGetLastError();
}
hipError_t launch_prop_init(const PropState& ps, uint64_t* front, hipStream_t st) {
    if (ps.n_msgs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_init, dim3(nblk(ps.n_msgs, 256)), dim3(256), 0, st, ps, front);
    return hipGetLastError();
}
hipError_t launch_rsub_select(const PropState& ps, const uint64_t* front, hipStream_t st) {
    if (ps.n_nodes == 0 || !ps.sel) return hipSuccess;
    hipLaunchKernelGGL(k_rsub_select, dim3(nblk(ps.n_nodes, 64)), dim3(64), 0, st, ps, front);
    return hipGetLastError();
}
hipError_t launch_prop_pack(const PropState& ps, const uint64_t* front, uint64_t* send, hipStream_t st) {
    if (ps.n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_pack, dim3(nblk(ps.n_send, 256)), dim3(256), 0, st, ps, front, send);
    return hipGetLastError();
}
hipError_t launch_prop_hop(const PropState& ps, uint32_t h, const uint64_t* front, uint64_t* nxt, hipStream_t st) {
    if (ps.n_nodes == 0) return hipSuccess;
    const dim3 g(nblk(ps.n_nodes, 256)), b(256);
    // n_words is 1, 2 or a multiple of 4 (the engine pads)
    if (ps.n_words == 1) hipLaunchKernelGGL(k_prop_hop<1>, g, b, 0, st, ps, h, front, nxt);
    else if (ps.n_words == 2) hipLaunchKernelGGL(k_prop_hop<2>, g, b, 0, st, ps, h, front, nxt);
    else hipLaunchKernelGGL(k_prop_hop<4>, g, b, 0, st, ps, h, front, nxt);
    return hipGetLastError();
}
hipError_t launch_prop_count(const PropState& ps, hipStream_t st) {
    if (ps.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_count, dim3(nblk(ps.n_pairs, 256)), dim3(256), 0, st, ps);
    return hipGetLastError();
}
hipError_t launch_prop_fold(const PropState& ps, const DevState& s, const uint32_t* first, const uint32_t* dup,
                            hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_fold, dim3(nblk(s.n_pairs, 256)), dim3(256), 0, st, ps, s, first, dup);
    return hipGetLastError();
}

}  // namespace gsx
