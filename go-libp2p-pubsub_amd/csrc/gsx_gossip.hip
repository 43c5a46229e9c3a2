// The gossip exchange of a heartbeat (include/gsx.h step (D)): IHAVE handling,
// IWANT answers and their receipt (gossipsub.go:615-716), and the promise
// tracking behind the P7 penalty (gossip_tracer.go:48-153, gossipsub.go:1578-1583).
//
// One lane per receiving node u walks its pairs q = (u -> v) twice:
//  pass 1: handleIHave for the one IHAVE RPC v sent (every topic): the score
//          / MaxIHaveMessages / iasked gates, the ids v advertised that u has
//          not seen (u's seen rows as the exchange started), the asked subset
//          and the one promise (serial << 32 | message index of the element at
//          Int31n(asked) in canonical order);
//  pass 2: v answers (its score of u, its cache after the Shift) and u
//          receives the answer: a first receipt (not in u's receipts of this
//          exchange) is delivered or rejected, fulfils u's promises for it and
//          is recorded in the set's receipt rows; a further copy is a duplicate.
// Canonical order: topics ascending, then the advertised batches in cache
// order (windows newest first, Put order), then message index.  Every
// per-pair state (promises, records of q) belongs to u's lane.
#include "gsx_device.h"
#include "gsx_ops.h"

#include <algorithm>

namespace gsx {

constexpr uint32_t VAL_ACCEPT = 0, VAL_REJECT = 1;  // GSX_VALIDATION_ACCEPT / _REJECT (gsx.h)

namespace {

__device__ __forceinline__ void gx_flush(unsigned long long* stats, int k, uint64_t c) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x % 64) == 0 && c) atomicAdd(&stats[k], (unsigned long long)c);
}

// Words per gxs_rows entry: the receive slot, the rows, the inside rows (gxs_vin).
__device__ __forceinline__ size_t gxs_ew(const HbState& h) { return 1 + (size_t)h.gxs_fw * (h.gxs_vin ? 2 : 1); }
// Word w of the sender's cache row of batch b, the sender being v, the peer
// of the receiver's pair q: a local sender's row; on a range shard a remote
// one's from the rows its rank sent (gxs_rows), none when it sent none (every
// message v holds is common: nothing to ask).  v is a global node id.
__device__ __forceinline__ uint64_t gx_mem(const HbState& h, const GxBatch& b, uint64_t q, uint32_t v, uint32_t w) {
    if (h.gxs_hidx && (h.rev[q] & HALO)) {
        const uint32_t k = h.gxs_hidx[q];
        return k == NO_PAIR ? 0ull : h.gxs_rows[(size_t)k * gxs_ew(h) + 1 + b.woff + w];
    }
    return b.mem[(size_t)(v - h.node_lo) * b.n_words + w];
}
// The bits of `bits` (messages v served u from its cache, word w of batch b)
// whose copy at v is inside the P3 window: v's copies are old (validated
// before the round: gsx.h (D)); a remote v's from the inside rows its rank sent.
// (MIX: some set of the round is mixed; the instance without it keeps its registers)
template <bool MIX>
__device__ __forceinline__ uint64_t gx_in_at_sender(const HbState& h, const GxBatch& b, uint64_t q, uint32_t v,
                                                    uint32_t w, uint64_t bits) {
    if (!MIX || b.old_in != 2 || !bits) return b.old_in ? bits : 0ull;
    if (h.gxs_hidx && (h.rev[q] & HALO)) {
        const uint32_t k = h.gxs_hidx[q];
        return k == NO_PAIR ? 0ull : bits & h.gxs_rows[(size_t)k * gxs_ew(h) + b.vin_off + w];
    }
    return vc_inside(b.vc, (size_t)(v - h.node_lo) * b.n_words + w, bits);
}
// The advertised batches whose row at the sender holds an uncommon message (gx_rhm).
__device__ __forceinline__ uint64_t gx_rhm_of(const HbState& h, uint64_t q, uint32_t v) {
    if (h.gxs_hidx && (h.rev[q] & HALO)) return h.gxs_hidx[q] == NO_PAIR ? 0ull : ~0ull;
    return h.gx_rhm[v - h.node_lo];
}
// handleIWant's gate at the peer v of q (r its pair to u): v's score of u.
__device__ __forceinline__ bool gx_answers(const DevState& s, const HbState& h, uint64_t q, uint32_t r) {
    if (r & HALO) return h.gxs_rans && h.gxs_rans[q];
    return !(s.score[r] < h.gossip_threshold);
}

// Streams the ids v advertised to u (pair q = (u -> v), r its reverse) on
// the topics of `tb` that u had not seen: f(batch index, message index) for
// each, in canonical order; returns false when f asks to stop.  A truncated
// list (ihave_tr) is the subset row the sender kept (GxSub); a batch whose
// every message u has seen is skipped without reading its rows.
template <typename F>
__device__ __forceinline__ bool gx_walk(const HbState& h, uint64_t tb, uint32_t u, uint32_t v, uint64_t q, uint32_t r,
                                        F&& f) {
    const uint64_t tr = h.ihave_tr[q];
    for (; tb; tb &= tb - 1) {
        const uint32_t t = (uint32_t)__builtin_ctzll(tb);
        const uint64_t* sub = nullptr;
        if ((tr >> t) & 1) {
            const GxSub& G = h.gsubs[t];
            sub = G.pool + (size_t)G.idx[r] * G.tw;
        }
        for (uint32_t g = h.gx_off[t]; g < h.gx_off[t + 1]; ++g) {
            const GxBatch& b = h.gx[g];
            if (b.full[u]) continue;
            const uint32_t W = b.n_words;
            for (uint32_t w = 0; w < W; ++w) {
                uint64_t m = gx_mem(h, b, q, v, w) & ~b.all[(size_t)u * W + w];
                if (sub) m &= sub[b.row_off + w];
                for (; m; m &= m - 1)
                    if (!f(g, w * 64 + (uint32_t)__builtin_ctzll(m))) return false;
            }
        }
    }
    return true;
}

}  // namespace

// applyIwantPenalties at the heartbeat start: a promise whose expiry is
// before now is broken, AddPenalty(peer, count) (GetBrokenPromises :79-115).
__global__ __launch_bounds__(256) void k_gx_promises(DevState s, HbState h) {
    uint64_t broken = 0;
    const uint32_t S = h.prom_slots;
    for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < h.n_pairs; q += (uint64_t)gridDim.x * 256u) {
        if (!h.prom_any[q]) continue;
        int c = 0;
        bool left = false;
        for (uint32_t k = 0; k < S; ++k) {
            const int64_t e = h.prom_e[q * S + k];
            if (e != 0 && e < h.now) {
                h.prom_e[q * S + k] = 0;
                ++c;
            } else {
                left |= e != 0;
            }
        }
        if (!left) h.prom_any[q] = 0;
        if (c) {
            ev_penalty(s, q, c);
            broken += (uint64_t)c;
            h.dirty[q] = 1;  // re-scored before the heartbeat reads it
        }
    }
    unsigned long long v[1] = {broken};
    const uint32_t slot[1] = {HB_BROKEN_PROMISES};
    block_count<1>(v, h.stats, slot);
}

// GetBrokenPromises alone (gsx_promise_broken): per-pair counts, freed.
__global__ __launch_bounds__(256) void k_gx_broken(HbState h, uint32_t* __restrict__ counts) {
    uint64_t broken = 0;
    const uint32_t S = h.prom_slots;
    for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < h.n_pairs; q += (uint64_t)gridDim.x * 256u) {
        uint32_t c = 0;
        bool left = false;
        for (uint32_t k = 0; k < S; ++k) {
            const int64_t e = h.prom_e[q * S + k];
            if (e != 0 && e < h.now) {
                h.prom_e[q * S + k] = 0;
                ++c;
            } else {
                left |= e != 0;
            }
        }
        if (!left) h.prom_any[q] = 0;
        counts[q] = c;
        broken += c;
    }
    unsigned long long v[1] = {broken};
    const uint32_t slot[1] = {HB_BROKEN_PROMISES};
    block_count<1>(v, h.stats, slot);
}

__global__ __launch_bounds__(256) void k_gx_count(HbState h, unsigned long long* n) {
    unsigned long long c[1] = {0};
    const uint64_t tot = h.n_pairs * h.prom_slots;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < tot; i += (uint64_t)gridDim.x * 256u)
        c[0] += h.prom_e[i] != 0;
    const uint32_t slot[1] = {0};
    block_count<1>(c, n, slot);
}

__global__ __launch_bounds__(256) void k_gx_prom_grow(const uint64_t* __restrict__ h_in, const int64_t* __restrict__ e_in,
                                                      uint32_t from, uint64_t* __restrict__ h_out,
                                                      int64_t* __restrict__ e_out, uint32_t to, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n * to; i += (uint64_t)gridDim.x * 256u) {
        const uint64_t q = i / to, k = i % to;
        h_out[i] = k < from ? h_in[q * from + k] : 0;
        e_out[i] = k < from ? e_in[q * from + k] : 0;
    }
}

// The candidate word (batch b, word w) of the ids v advertised to u that u
// had not seen, within the subset row of a truncated list.
// u's own row first: v's cache word is read only where u lacks a message
// (mem has no bit past n_msgs, so this is mem & ~all exactly).
__device__ __forceinline__ uint64_t gx_word(const HbState& h, const GxBatch& b, uint32_t u, uint64_t q, uint32_t v,
                                            uint32_t w, const uint64_t* sub) {
    const uint32_t W = b.n_words;
    const uint32_t left = b.n_msgs > w * 64 ? b.n_msgs - w * 64 : 0;
    const uint64_t valid = left >= 64 ? ~0ull : ((1ull << left) - 1);
    const uint64_t miss = ~b.all[(size_t)u * W + w] & valid;
    if (!miss) return 0;
    uint64_t m = gx_mem(h, b, q, v, w) & miss;
    if (sub) m &= sub[b.row_off + w];
    return m;
}

__device__ __forceinline__ const uint64_t* gx_subrow(const HbState& h, uint64_t tr, uint32_t t, uint32_t r) {
    if (!((tr >> t) & 1)) return nullptr;
    const GxSub& G = h.gsubs[t];
    return G.pool + (size_t)G.idx[r] * G.tw;
}

// The advertised batches a receiver has not seen whole: bit g of the mask
// (batches past 64 always walked); every other batch holds no candidate.
__device__ __forceinline__ uint64_t gx_unseen(const HbState& h, uint32_t n_gx, uint32_t u) {
    uint64_t nf = n_gx > 64 ? ~0ull : 0ull;
    const uint32_t lim = n_gx < 64 ? n_gx : 64;
    for (uint32_t g0 = 0; g0 < lim; g0 += 8) {  // eight batches' bytes in flight per round trip
        uint8_t fb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) fb[j] = g0 + j < lim ? h.gx[g0 + j].full[u] : 1;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (!fb[j]) nf |= 1ull << (g0 + j);
    }
    return nf;
}
__device__ __forceinline__ bool gx_skip(uint64_t nf, uint32_t g) { return g < 64 && !((nf >> g) & 1); }

// |iwant| before the budget: popcounts of the candidate words (no bit walk).
__device__ __forceinline__ uint32_t gx_count(const HbState& h, uint64_t tb, uint32_t u, uint32_t v, uint64_t q,
                                             uint32_t r, uint64_t nf) {
    const uint64_t tr = h.ihave_tr[q];
    uint32_t n = 0;
    for (; tb; tb &= tb - 1) {
        const uint32_t t = (uint32_t)__builtin_ctzll(tb);
        const uint64_t* sub = gx_subrow(h, tr, t, r);
        for (uint32_t g = h.gx_off[t]; g < h.gx_off[t + 1]; ++g) {
            if (gx_skip(nf, g)) continue;
            const GxBatch& b = h.gx[g];
            for (uint32_t w = 0; w < b.n_words; ++w) n += (uint32_t)__popcll(gx_word(h, b, u, q, v, w, sub));
        }
    }
    return n;
}

// The j-th candidate in canonical order (word popcounts, then a bit walk in one word).
__device__ __forceinline__ void gx_nth(const HbState& h, uint64_t tb, uint32_t u, uint32_t v, uint64_t q, uint32_t r,
                                       uint64_t nf, uint32_t j, uint32_t& pick_g, uint32_t& pick_k) {
    const uint64_t tr = h.ihave_tr[q];
    for (; tb; tb &= tb - 1) {
        const uint32_t t = (uint32_t)__builtin_ctzll(tb);
        const uint64_t* sub = gx_subrow(h, tr, t, r);
        for (uint32_t g = h.gx_off[t]; g < h.gx_off[t + 1]; ++g) {
            if (gx_skip(nf, g)) continue;
            const GxBatch& b = h.gx[g];
            for (uint32_t w = 0; w < b.n_words; ++w) {
                uint64_t m = gx_word(h, b, u, q, v, w, sub);
                const uint32_t c = (uint32_t)__popcll(m);
                if (j >= c) {
                    j -= c;
                    continue;
                }
                for (; j; --j) m &= m - 1;
                pick_g = g;
                pick_k = w * 64 + (uint32_t)__builtin_ctzll(m);
                return;
            }
        }
    }
}

// Per-(pair, topic) credits of the received ids, as the one-at-a-time tracer
// calls would leave them (score.go:894-974): k1 first deliveries (FMD, and MMD
// in the mesh), k2 accepted duplicates (MMD in the mesh), k4 invalid ones (IMD)
// — every step of a counter is the same capped +1, so their order is free.
__device__ __forceinline__ void gx_credit(const DevState& s, uint64_t q, uint32_t t, uint32_t k1, uint32_t k2,
                                          uint32_t k4) {
    if (!(k1 | k2 | k4) || !scored_topic(s, q, t)) return;
    const DevTopicParams& tp = s.tp[t];
    const size_t b = rec_index(q, t, s.n_topics, FMD);
    if (k4) s.rec[b + IMD * TILE] = add_ones_capped(s.rec[b + IMD * TILE], k4, __builtin_inf());
    if (k1) s.rec[b + FMD * TILE] = add_ones_capped(s.rec[b + FMD * TILE], k1, tp.cap2);
    if ((k1 | k2) && (s.rflags[flag_index(q, t, s.n_topics)] & REC_IN_MESH))
        s.rec[b + MMD * TILE] = add_ones_capped(s.rec[b + MMD * TILE], k1 + k2, tp.cap3);
}

// The words w of a set whose message node x published (src: node << 32 |
// index, ascending, n entries).
__device__ __forceinline__ uint64_t origin_word(const uint64_t* src, uint32_t n, uint32_t x, uint32_t w) {
    uint32_t lo = 0, hi = n;
    const uint64_t key = (uint64_t)x << 32;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        if (src[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    uint64_t m = 0;
    for (uint32_t i = lo; i < n && (src[i] >> 32) == x; ++i) {
        const uint32_t k = (uint32_t)src[i];
        if (k / 64 == w) m |= 1ull << (k % 64);
    }
    return m;
}

// The IWANT first receipts of pair q = (u -> v) per topic this round that u
// would forward back to v but for the `from` exclusion (those v published are
// excluded as the origin already): the forwarding's hop-1 back-sends (GxFwd).
// At v those copies are old (v served them from its cache): counted apart by
// the old_in of their set (inside the P3 window or not).
// Counted per set group (GxBatch::grp: up to 64 sets of one topic).
__device__ __forceinline__ void gx_back0_clear(const HbState& h, uint64_t q) {  // (once per answered pair)
    if (!h.gxb_st0 || h.gxb_st0[q] == h.gxb_stamp) return;
    h.gxb_st0[q] = h.gxb_stamp;
    for (uint32_t i = 0; i < h.gxb_ngrp; ++i) h.gxb_cnt0[(size_t)i * h.n_pairs + q] = 0;
}
__device__ __forceinline__ void gx_back0(const HbState& h, uint64_t q, uint32_t grp, uint32_t k_in, uint32_t k_out) {
    if (!h.gxb_st0 || !(k_in | k_out)) return;
    gx_back0_clear(h, q);
    h.gxb_cnt0[(size_t)grp * h.n_pairs + q] += k_in | k_out << 16;
}

// The IWANT draws of pair q = (u -> v) (the asked subset, AddPromise's pick):
// keyed by the global node ids, so a range shard draws what one engine draws.
__device__ __forceinline__ Rng gx_iwant_rng(const HbState& h, uint32_t u, uint32_t v) {
    return Rng{h.seed, TAG_IWANT, ((uint64_t)(h.node_lo + u) << 32) | v, h.tick << 32, 0};
}

// handleIWant at v and the receipt at u, one id at a time (pass 2 for a pair
// whose asked subset was sampled, kk < n: the same draws select it again),
// each receipt credited by its own tracer call.
template <bool MIX>
__device__ __forceinline__ void gx_receive_sampled(const DevState& s, const HbState& h, uint32_t u, uint64_t q,
                                                   uint32_t r, uint64_t tb, uint32_t kk, uint32_t n, uint64_t& served,
                                                   uint64_t& delivered, uint64_t& rejected, uint64_t& dups) {
    const uint32_t v = (uint32_t)h.col[q];
    const DevGossipParams& gp = h.gp;
    Rng g = gx_iwant_rng(h, u, v);
    uint32_t i = 0, sel = 0;
    gx_walk(h, tb, u, v, q, r, [&](uint32_t gi, uint32_t k) {
        const bool take = (uint32_t)g.int31n((int32_t)(n - i)) < kk - sel;
        ++i;
        if (!take) return true;
        ++sel;
        const GxBatch& b = h.gx[gi];
        // no longer in v's cache; or GetForPeer's count above GossipRetransmission
        if (!b.avail || gp.retransmission < 1) return sel < kk;
        ++served;
        const uint32_t W = b.n_words, t = b.topic, val = b.val[k];
        uint64_t* xw = b.x + (size_t)u * W + k / 64;
        const uint64_t bit = 1ull << (k % 64);
        if (*xw & bit) {  // DuplicateMessage
            ++dups;
            if (val == VAL_ACCEPT) ev_mesh(s, q, t);
            else if (val == VAL_REJECT) ev_invalid(s, q, t);
        } else {
            *xw |= bit;
            if (val == VAL_ACCEPT) {
                ++delivered;
                ev_first(s, q, t);
                if (h.gxb_st0 && !((origin_word(b.src, b.n_msgs, v, k / 64) >> (k % 64)) & 1)) {
                    const uint32_t in = gx_in_at_sender<MIX>(h, b, q, v, k / 64, bit) ? 1u : 0u;
                    gx_back0(h, q, b.grp, in, 1u - in);
                }
                *b.got = 1;
            } else {
                ++rejected;
                if (val == VAL_REJECT) ev_invalid(s, q, t);
            }
        }
        return sel < kk;
    });
}

// handleIHave's gates (:615-633) for the IHAVE RPC on pair q = (u -> v):
// 0 = nobody to answer (v untracked or on another shard), 1 = ignored (v's
// score below GossipThreshold, MaxIHaveMessages, MaxIHaveLength asked), 2 = handled.
__device__ __forceinline__ int gx_gate(const DevState& s, const HbState& h, uint64_t q, uint32_t r) {
    if (r == NO_PAIR || ((r & HALO) && !h.gxs_hidx)) return 0;
    if (s.score[q] < h.gossip_threshold) return 1;  // :617-621
    // peerhave / iasked (:624-633) are cleared at every heartbeat start (:1566-1576)
    // and each pair handles one IHAVE RPC per heartbeat (every topic in it), so at
    // this check they are 1 and 0: the limits only test the parameters
    if ((int64_t)h.gp.max_ihave_msgs < 1) return 1;  // :624-628
    if ((int64_t)h.gp.max_ihave <= 0) return 1;       // :630-633
    return 2;
}

__device__ __forceinline__ uint32_t gx_wsum(uint32_t x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += (uint32_t)__shfl_xor((int)x, off, 64);
    return x;
}
__device__ __forceinline__ uint32_t gx_excl(uint32_t x, uint32_t lane) {  // exclusive prefix sum over the wave
    uint32_t incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, off, 64);
        if (lane >= (uint32_t)off) incl += y;
    }
    return incl - x;
}

// The flat word list of the advertised batches (GxBatch::woff; canonical
// order: topics ascending, then cache order) is walked in rounds of 64 words,
// every topic at once: in round i lane L holds word 64 i + L (its batch from
// gx_wb), so a batch word always belongs to the same lane and a round's words
// are in canonical order by lane.  The lane's candidate word: its batch on a
// topic of tb that u had not seen whole, within the subset row of a truncated
// list; g: the word's batch.
__device__ __forceinline__ uint64_t gx_fword(const HbState& h, uint64_t tb, uint32_t u, uint64_t q, uint32_t v,
                                             uint64_t tr, uint32_t r, uint64_t nf, uint32_t f, uint32_t& g,
                                             uint32_t& w) {
    g = 0;
    w = 0;
    if (f >= h.gx_fw) return 0;
    g = h.gx_wb[f];
    if (gx_skip(nf, g)) return 0;
    const GxBatch& b = h.gx[g];
    if (!((tb >> b.topic) & 1)) return 0;
    w = f - b.woff;
    return gx_word(h, b, u, q, v, w, gx_subrow(h, tr, b.topic, r));
}

// |iwant| of pair q (every lane gets it): popcounts of the candidate words.
__device__ __forceinline__ uint32_t gx_wcount(const HbState& h, uint64_t tb, uint32_t u, uint64_t q, uint32_t v,
                                              uint64_t tr, uint32_t r, uint64_t nf, uint32_t lane) {
    uint32_t c = 0, g, w;
    for (uint32_t f = lane; f < h.gx_fw; f += 64) c += (uint32_t)__popcll(gx_fword(h, tb, u, q, v, tr, r, nf, f, g, w));
    return gx_wsum(c);
}

// The j-th candidate of pair q in canonical order (every lane gets it).
__device__ __forceinline__ void gx_wnth(const HbState& h, uint64_t tb, uint32_t u, uint64_t q, uint32_t v,
                                        uint64_t tr, uint32_t r, uint64_t nf, uint32_t lane, uint32_t j,
                                        uint32_t& pick_g, uint32_t& pick_k) {
    for (uint32_t f0 = 0; f0 < h.gx_fw; f0 += 64) {  // (uniform rounds)
        uint32_t g, w;
        uint64_t m = gx_fword(h, tb, u, q, v, tr, r, nf, f0 + lane, g, w);
        const uint32_t c = (uint32_t)__popcll(m);
        const uint32_t e = gx_excl(c, lane);
        const uint32_t tot = (uint32_t)__shfl((int)(e + c), 63, 64);
        if (j >= tot) {
            j -= tot;
            continue;
        }
        const bool mine = e <= j && j < e + c;
        uint32_t k = 0;
        if (mine) {
            for (uint32_t i = j - e; i; --i) m &= m - 1;
            k = w * 64 + (uint32_t)__builtin_ctzll(m);
        }
        const int src = __ffsll((long long)__ballot(mine)) - 1;
        pick_g = (uint32_t)__shfl((int)g, src, 64);
        pick_k = (uint32_t)__shfl((int)k, src, 64);
        return;
    }
}

// AddPromise (gossip_tracer.go:59-74): once per (message, peer); the host
// keeps a free slot on every pair before each exchange (one promise per pair).
__device__ __forceinline__ void gx_promise(const HbState& h, uint64_t q, uint64_t handle, uint32_t& occ) {
    const uint32_t S = h.prom_slots;
    uint64_t* ph_ = h.prom_h + (size_t)q * S;
    int64_t* pe_ = h.prom_e + (size_t)q * S;
    int free_slot = -1;
    bool have = false;
    uint32_t used = 0;
    for (uint32_t k = 0; k < S; ++k) {
        if (pe_[k] == 0) {
            if (free_slot < 0) free_slot = (int)k;
        } else {
            ++used;
            if (ph_[k] == handle) have = true;
        }
    }
    if (!have && free_slot >= 0) {
        ph_[free_slot] = handle;
        pe_[free_slot] = h.now + h.gp.followup_ns;
        h.prom_any[q] = 1;
        ++used;
    } else if (!have) {
        h.gx_err[1] = 1;  // (the host's invariant broken: never)
    }
    occ = used > occ ? used : occ;
}

// The asked subset of a sampled pair (kk < n, selection sampling over the
// canonical walk) and AddPromise's pick in it (the element at Int31n(kk)).
__device__ __forceinline__ void gx_pick_sampled(const HbState& h, uint64_t tb, uint32_t u, uint32_t v, uint64_t q,
                                                uint32_t r, uint32_t n, uint32_t kk, uint32_t& pick_g,
                                                uint32_t& pick_k) {
    Rng g = gx_iwant_rng(h, u, v);
    uint32_t i = 0, sel = 0;
    gx_walk(h, tb, u, v, q, r, [&](uint32_t, uint32_t) {
        if ((uint32_t)g.int31n((int32_t)(n - i)) < kk - sel) ++sel;
        ++i;
        return sel < kk;
    });
    const uint32_t j = (uint32_t)g.int31n((int32_t)kk);
    Rng g2 = gx_iwant_rng(h, u, v);  // the same selection again
    i = 0;
    sel = 0;
    gx_walk(h, tb, u, v, q, r, [&](uint32_t gi, uint32_t k) {
        const bool take = (uint32_t)g2.int31n((int32_t)(n - i)) < kk - sel;
        ++i;
        if (!take) return true;
        if (sel++ < j) return true;
        pick_g = gi;
        pick_k = k;
        return false;
    });
}

#ifdef GSX_GX_PROF  // (diagnostic build only: k_gx_ask's work counts, printed per round)
__device__ unsigned long long gx_prof[16];
#define GXP(i, v) atomicAdd(&gx_prof[i], (unsigned long long)(v))
extern "C" void gx_prof_dump() {
    unsigned long long c[16];
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(gx_prof), sizeof(c));
    fprintf(stderr, "gx_prof tall=%llu gate2=%llu gate2_nf=%llu heavy=%llu cb=%llu batches=%llu words=%llu n_pos=%llu "
                    "nodes_nf=%llu nf_bits=%llu tr=%llu poor_bits=%llu cb_rhm=%llu miss_sum=%llu\n",
            c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9], c[10], c[13], c[14], c[15]);
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(gx_prof), z, sizeof(z));
}
#else
#define GXP(i, v) ((void)0)
#endif
constexpr uint32_t GX_END = 0xFFFFFFFFu;  // GxBatch::nxt: the set's last batch
constexpr uint32_t GX_MW = 128;  // words of unseen batches a receiver's lane walks itself (else: a wave, GX_HEAVY)
constexpr uint32_t GX_HEAVY = 1u << 31;  // gx_nodes entry: pass 1 runs in k_gx_node
constexpr uint32_t GX_REQ_ALL = 1u << 31;  // gx_req: the pair asked for every candidate (kk = |iwant|)

// v's cache row of batch b (pair q = (u -> v)): a local sender's; on a range
// shard a remote one's from the rows its rank sent; null when it sent none.
__device__ __forceinline__ const uint64_t* gx_memrow(const HbState& h, const GxBatch& b, uint64_t q, uint32_t v) {
    if (h.gxs_hidx && (h.rev[q] & HALO)) {
        const uint32_t k = h.gxs_hidx[q];
        return k == NO_PAIR ? nullptr : h.gxs_rows + (size_t)k * gxs_ew(h) + 1 + b.woff;
    }
    return b.mem + (size_t)(v - h.node_lo) * b.n_words;
}
// The candidate words of pair q in canonical order (the batches of cb on the
// topics of tb, words ascending): f(batch, word, v's cache word & ~u's, within
// the subset row of a truncated list) for each nonzero one; stops when f
// returns false.  (mem has no bit past n_msgs: no validity mask.)
// wm: u's miss masks from k_gx_ask's LDS (batch g's byte at wm[64 g]: bit w
// = u lacks a message of word w; batches of at most 8 words), so v's words
// are gathered only where u lacks something.
template <typename F>
__device__ __forceinline__ void gx_cwalk(const HbState& h, uint64_t cb, uint64_t tb, uint32_t uu, uint64_t q,
                                         uint32_t v, uint64_t tr, uint32_t r, const uint8_t* wm, F&& f) {
    for (; cb; cb &= cb - 1) {
        const uint32_t g = (uint32_t)__builtin_ctzll(cb);
        const GxBatch& b = h.gx[g];
        if (!((tb >> b.topic) & 1)) continue;
        GXP(5, 1);
        const uint64_t* mrow = gx_memrow(h, b, q, v);
        if (!mrow) return;  // (a remote sender with no uncommon rows: none in any batch)
        const uint32_t W = b.n_words;
        const uint64_t* arow = b.all + (size_t)uu * W;
        const uint64_t* sub = gx_subrow(h, tr, b.topic, r);
        const uint32_t wmask = W <= 8 ? wm[64 * g] : 0xFFFFFFFFu;
        for (uint32_t w = 0; w < W; ++w) {
            if (!((wmask >> (w < 32 ? w : 31)) & 1)) continue;
            GXP(6, 1);
            uint64_t c = mrow[w] & ~arow[w];
            if (sub) c &= sub[b.row_off + w];
            if (c && !f(g, w, c)) return;
        }
    }
}

// Pass 1: handleIHave (:615-679) for the one IHAVE RPC each sender v sent
// (every topic): the score / MaxIHaveMessages / iasked gates, |iwant| from
// word popcounts, the asked subset (all; or a uniform kk-subset by selection
// sampling) and AddPromise's pick (gossip_tracer.go:53).  Everything it
// touches is per pair (the IHAVE counters, the request, the promise of q), so
// the pairs of a node are independent.  A wave takes 64 consecutive nodes:
//  - a lane per node finds the advertised batches its node has not seen whole
//    (only they can hold a candidate); a node with none asks for nothing; one
//    whose unseen batches hold more than GX_MW words is heavy (k_gx_node's
//    wave runs its pass 1: GX_HEAVY);
//  - the lanes then take the tile's pairs in order, a lane per pair (the
//    per-pair arrays are read coalesced), each walking the words of its node's
//    unseen batches (u's row and v's cache row side by side, no LDS list: the
//    kernel keeps 6 waves per SIMD);
//  - a node with a heavy walk or an asked pair is listed for k_gx_node (pass 2).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void k_gx_ask(DevState s, HbState h) {
    __shared__ uint8_t wms[64][64];  // [batch][node of the tile]: words (<= 8 per batch) where the node lacks a message
    __shared__ int64_t rp[65];      // row_ptr of the tile's nodes
    __shared__ uint64_t nfs[64];    // per node: the unseen-batch mask
    __shared__ uint64_t pms[64];    // per node (gx_poor): the batches it misses more than GX_POOR messages of
    __shared__ uint32_t nmls[64];   // per node: GX_HEAVY
    __shared__ uint32_t lst[64];    // per node: listed for k_gx_node
    const uint32_t lane = threadIdx.x;
    uint64_t ignored = 0, iw_msgs = 0, iw_ids = 0;
    uint32_t occ = 0;
    const uint32_t n_gx = h.gx_off[s.n_topics];
    for (uint32_t tile = blockIdx.x * 64u; tile < h.n_nodes; tile += gridDim.x * 64u) {
        const uint32_t u = tile + lane;
        {  // ---- lane per node: unseen batches, their words
            uint64_t nf = 0, pm = 0;
            uint32_t nw = 0;
            bool heavy = n_gx > 64;
            if (u < h.n_nodes) {
                nf = gx_unseen(h, n_gx, u);
                for (uint64_t m = heavy ? 0 : nf; m; m &= m - 1) {
                    const uint32_t g = (uint32_t)__builtin_ctzll(m);
                    const GxBatch& b = h.gx[g];
                    const uint32_t W = b.n_words;
                    nw += W;
                    if (nw > GX_MW) {
                        heavy = true;
                        break;
                    }
                    if (W <= 8) {
                        uint32_t mk = 0, miss = 0;
                        for (uint32_t w = 0; w < W; ++w) {
                            const uint32_t left = b.n_msgs > w * 64 ? b.n_msgs - w * 64 : 0;
                            const uint64_t valid = left >= 64 ? ~0ull : ((1ull << left) - 1);
                            const uint64_t lack = ~b.all[(size_t)u * W + w] & valid;
                            if (lack) mk |= 1u << w;
                            miss += (uint32_t)__popcll(lack);
                        }
                        wms[g][lane] = (uint8_t)mk;
                        if (miss > GX_POOR) pm |= 1ull << g;  // (k_gx_setprep's test: n_msgs - seen > GX_POOR)
                        GXP(15, miss);
                    } else {
                        pm |= 1ull << g;  // (no word masks: unfiltered)
                    }
                }
            }
            nfs[lane] = nf;
            pms[lane] = h.gx_poor ? pm : 0ull;
            GXP(13, __popcll(pm));
            GXP(8, nf != 0);
            GXP(9, __popcll(nf));
            nmls[lane] = heavy ? GX_HEAVY : 0u;
            lst[lane] = 0;
            rp[lane] = h.row_ptr[u < h.n_nodes ? u : h.n_nodes];
            if (lane == 0) rp[64] = h.row_ptr[tile + 64 < h.n_nodes ? tile + 64 : h.n_nodes];
        }
        __syncthreads();
        // ---- lane per pair, the tile's pairs in order
        uint32_t k = 0;  // the node of pair q (monotonic: q only grows)
        const int64_t qe = rp[64];
        // the next pair's IHAVE bits and reverse pair are loaded before this one's
        // chain (gate, peer, rhm, rows) runs: one round trip fewer per pair
        uint64_t tall_n = rp[0] + lane < qe ? h.ihave_bits[rp[0] + lane] : 0ull;
        uint32_t rev_n = rp[0] + lane < qe ? h.rev[rp[0] + lane] : NO_PAIR;
        for (int64_t q = rp[0] + lane; q < qe; q += 64) {
            while (rp[k + 1] <= q) ++k;
            const uint64_t tall = tall_n;  // topics v sent u an IHAVE for (receiver-side)
            const uint32_t r = rev_n;
            if (q + 64 < qe) {
                tall_n = h.ihave_bits[q + 64];
                rev_n = h.rev[q + 64];
            }
            if (!tall) continue;
            GXP(0, 1);
            const int gt = gx_gate(s, h, (uint64_t)q, r);
            ignored += gt == 1;
            const uint64_t nf = nfs[k];
            GXP(1, gt == 2);
            if (gt != 2 || !nf) continue;
            GXP(2, 1);
            const uint32_t nm = nmls[k];
            if (nm & GX_HEAVY) {
                GXP(3, 1);
                lst[k] = 1;
                continue;
            }
            const uint32_t uu = tile + k;
            const uint64_t tb = tall & (h.sub ? h.sub[uu] : ~0ull);  // joined topics only (:638-641)
            const uint32_t v = (uint32_t)h.col[q];
            // the unseen batches whose row at v holds a message not every node had:
            // only there can v hold one u lacks
            const uint64_t cb = nf & (gx_rhm_of(h, (uint64_t)q, v) | pms[k]);
            GXP(14, (nf & gx_rhm_of(h, (uint64_t)q, v)) != 0);
            if (!cb) continue;  // |iwant| = 0 (:652-654)
            GXP(4, 1);
            const uint64_t tr = h.ihave_tr[q];
            GXP(10, tr != 0);
            // |iwant|: v's cache words where u lacks something (topics of the RPC,
            // the subset row of a truncated list)
            uint32_t n = 0;
            gx_cwalk(h, cb, tb, uu, (uint64_t)q, v, tr, r, &wms[0][k], [&](uint32_t, uint32_t, uint64_t c) {
                n += (uint32_t)__popcll(c);
                return true;
            });
            if (n == 0) continue;  // :652-654
            GXP(7, 1);
            const uint32_t budget = (uint32_t)h.gp.max_ihave;  // MaxIHaveLength - iasked (0: above)
            const uint32_t kk = n < budget ? n : budget;
            uint32_t pick_g = 0, pick_k = 0;
            if (kk == n) {  // the element at Int31n(kk) of all of them, canonical order
                Rng g = gx_iwant_rng(h, uu, v);
                uint32_t j = (uint32_t)g.int31n((int32_t)kk);
                gx_cwalk(h, cb, tb, uu, (uint64_t)q, v, tr, r, &wms[0][k], [&](uint32_t gi, uint32_t w, uint64_t c) {
                    const uint32_t pc = (uint32_t)__popcll(c);
                    if (j >= pc) {
                        j -= pc;
                        return true;
                    }
                    for (; j; --j) c &= c - 1;
                    pick_g = gi;
                    pick_k = w * 64 + (uint32_t)__builtin_ctzll(c);
                    return false;
                });
            } else {
                gx_pick_sampled(h, tb, uu, v, q, r, n, kk, pick_g, pick_k);
            }
            ++iw_msgs;
            iw_ids += kk;
            h.gx_req[q] = kk | (kk == n ? GX_REQ_ALL : 0u);
            gx_promise(h, (uint64_t)q, ((uint64_t)h.gx[pick_g].serial << 32) | pick_k, occ);
            lst[k] = 1;
        }
        __syncthreads();
        {  // ---- lane per node: the listed ones
            const bool take = u < h.n_nodes && lst[lane];
            const uint32_t k = wave_append(&h.gx_err[6], take);
            if (take) h.gx_nodes[k] = u | (nmls[lane] & GX_HEAVY);
            const uint64_t tm = __ballot(take);  // (a tile is one word of the touch bits)
            if (lane == 0 && tm && h.gx_touch) atomicOr(reinterpret_cast<unsigned long long*>(&h.gx_touch[tile >> 6]), tm);
        }
        __syncthreads();  // (the tile's LDS is rewritten next)
    }
    gx_flush(h.stats, HB_IHAVE_IGNORED, ignored);
    gx_flush(h.stats, HB_IWANT_MSGS, iw_msgs);
    gx_flush(h.stats, HB_IWANT_IDS, iw_ids);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)occ, off, 64);
        occ = o > occ ? o : occ;
    }
    if (lane == 0 && occ) atomicMax(h.prom_occ, occ);
}

// One wave per listed node u, senders ascending throughout (every per-pair
// state — IHAVE counters, promises, records of q — is u's alone):
//  pass 1 (GX_HEAVY nodes): k_gx_ask's handleIHave with the counts and the
//          pick in rounds of 64 candidate words (gx_wcount, gx_wnth);
//  pass 2: v answers (handleIWant :681-716: its score of u, its cache after
//          the Shift) and u receives, word-parallel when u asked for every
//          candidate (kk = n): lane i takes the words i, i + 64, ... of each
//          advertised batch in cache order (a batch word always goes to the
//          same lane, and the batches of one message set share their receipt
//          rows word for word, so a later copy — another batch, a later pair —
//          meets the receipt its lane wrote); per topic the first deliveries,
//          accepted duplicates and invalid ones are summed and credited once
//          (gx_credit); a sampled pair (kk < n) is received by lane 0 one id
//          at a time;
//  then fulfillPromise (:119-126): u's promises whose message is now in its
//  receipt rows (promises are only added in pass 1).
template <bool MIX>
__global__ __launch_bounds__(64) void k_gx_node(DevState s, HbState h) {
    __shared__ uint32_t kc[3][64];  // per topic (GSX_MAX_TOPICS): k1, k2, k4 of the pair being received
    __shared__ uint32_t gser[64];   // the first 64 advertised batches' set serials (fulfillPromise)
    const uint32_t lane = threadIdx.x;
    gser[lane] = lane < h.gx_off[s.n_topics] ? h.gx[lane].serial : ~0u;
    __syncthreads();
    const uint32_t S = h.prom_slots;
    const DevGossipParams& gp = h.gp;
    uint64_t iw_msgs = 0, iw_ids = 0, served = 0, delivered = 0, rejected = 0, dups = 0;
    uint32_t occ = 0;
    const uint32_t n_list = h.gx_err[6];
    const uint32_t n_gx = h.gx_off[s.n_topics];
    for (uint32_t li = blockIdx.x; li < n_list; li += gridDim.x) {
        const uint32_t entry = h.gx_nodes[li];
        const uint32_t u = entry & ~GX_HEAVY;
        const int64_t r0 = h.row_ptr[u], r1 = h.row_ptr[u + 1];
        uint64_t nf = n_gx > 64 ? ~0ull : __ballot(lane < n_gx && !h.gx[lane].full[u]);
        if (entry & GX_HEAVY) {  // ---- pass 1 for a node with many unseen batches
            for (int64_t q = r0; q < r1; ++q) {
                const uint64_t tall = h.ihave_bits[q];
                if (!tall) continue;
                const uint32_t r = h.rev[q];
                if (gx_gate(s, h, (uint64_t)q, r) != 2) continue;
                const uint64_t tb = tall & (h.sub ? h.sub[u] : ~0ull);
                const uint32_t v = (uint32_t)h.col[q];
                const uint64_t tr = h.ihave_tr[q];
                const uint32_t n = gx_wcount(h, tb, u, (uint64_t)q, v, tr, r, nf, lane);
                if (n == 0) continue;
                const uint32_t budget = (uint32_t)gp.max_ihave;  // MaxIHaveLength - iasked (0: gx_gate)
                const uint32_t kk = n < budget ? n : budget;
                uint32_t pick_g = 0, pick_k = 0;
                if (kk == n) {
                    Rng g = gx_iwant_rng(h, u, v);
                    gx_wnth(h, tb, u, (uint64_t)q, v, tr, r, nf, lane, (uint32_t)g.int31n((int32_t)kk), pick_g, pick_k);
                } else if (lane == 0) {
                    gx_pick_sampled(h, tb, u, v, q, r, n, kk, pick_g, pick_k);
                }
                if (lane == 0) {
                    ++iw_msgs;
                    iw_ids += kk;
                    h.gx_req[q] = kk | (kk == n ? GX_REQ_ALL : 0u);
                    gx_promise(h, (uint64_t)q, ((uint64_t)h.gx[pick_g].serial << 32) | pick_k, occ);
                }
            }
            __threadfence_block();  // gx_req of every pair before pass 2 reads it
        }
        // ---- pass 2: v answers, u receives (the asked pairs found 64 at a time)
        for (int64_t c0 = r0; c0 < r1; c0 += 64) {
          const uint32_t kq = c0 + lane < r1 ? h.gx_req[c0 + lane] : 0u;
          for (uint64_t am = __ballot(kq != 0); am; am &= am - 1) {  // (wave-uniform)
            const int jb = __builtin_ctzll(am);
            const int64_t q = c0 + jb;
            const uint32_t kq_j = (uint32_t)__shfl((int)kq, jb, 64);
            const uint32_t kk = kq_j & ~GX_REQ_ALL;
            // (every candidate asked: |iwant| as k_gx_ask counted it, the rows it read
            // unchanged since; else the sampled path needs the count again)
            const bool ask_all = (kq_j & GX_REQ_ALL) != 0;
            const uint64_t tall = h.ihave_bits[q];
            const uint32_t r = h.rev[q];
            const bool answered = gx_answers(s, h, (uint64_t)q, r) &&  // v ignores u's IWANT
                                  ((h.eflags[q] & EDGE_DIRECT) || !(s.score[q] < h.graylist));  // AcceptFrom at u
            const uint64_t tb = tall & (h.sub ? h.sub[u] : ~0ull);
            if (answered && lane == 0) gx_back0_clear(h, (uint64_t)q);  // (the lanes below add to the counts)
            __threadfence_block();
            if (answered) {
                const uint32_t v = (uint32_t)h.col[q];
                const uint64_t tr = h.ihave_tr[q];
                const uint32_t n = ask_all ? kk : gx_wcount(h, tb, u, (uint64_t)q, v, tr, r, nf, lane);
                if (kk == n) {
                    // a lane per (message set, word) of every set on the topics of tb
                    // (h.gx_sw, canonical order): it walks the set's batches in cache
                    // order (the one order its receipt word sees); different sets touch
                    // different receipt rows, so the topics run together; the per-topic
                    // counts meet in LDS, credited once per topic by the topic's lane
                    kc[0][lane] = kc[1][lane] = kc[2][lane] = 0;
                    __syncthreads();
                    for (uint32_t f = lane; f < h.gx_nsw; f += 64) {
                        const uint4 sw = h.gx_sw[f];  // (first batch, word, topic)
                        const uint32_t t = sw.z, w = sw.y;
                        if (!((tb >> t) & 1)) continue;
                        const uint64_t* sub = gx_subrow(h, tr, t, r);
                        uint32_t k1 = 0, k2 = 0, k4 = 0;
                        for (uint32_t gi = sw.x; gi != GX_END; gi = h.gx[gi].nxt) {
                            if (gx_skip(nf, gi)) continue;
                            const GxBatch& b = h.gx[gi];
                            // no longer in v's cache; or GetForPeer's count above GossipRetransmission
                            if (!b.avail || gp.retransmission < 1) continue;
                            const uint32_t W = b.n_words;
                            const uint64_t m = gx_word(h, b, u, (uint64_t)q, v, w, sub);
                            if (!m) continue;
                            uint64_t* xw = b.x + (size_t)u * W + w;
                            const uint64_t x0 = *xw;
                            *xw = x0 | m;
                            served += (uint64_t)__popcll(m);
                            uint64_t acc1 = 0;
                            for (uint64_t z = m & ~x0; z; z &= z - 1) {
                                const uint32_t val = b.val[w * 64 + (uint32_t)__builtin_ctzll(z)];
                                if (val == VAL_ACCEPT) {
                                    ++delivered;
                                    ++k1;
                                    acc1 |= z & (~z + 1);
                                } else {
                                    ++rejected;
                                    if (val == VAL_REJECT) ++k4;
                                }
                            }
                            for (uint64_t z = m & x0; z; z &= z - 1) {  // DuplicateMessage
                                const uint32_t val = b.val[w * 64 + (uint32_t)__builtin_ctzll(z)];
                                ++dups;
                                if (val == VAL_ACCEPT) ++k2;
                                else if (val == VAL_REJECT) ++k4;
                            }
                            if (acc1 && h.gxb_st0) {  // the back-sends of these first receipts (GxFwd)
                                const uint64_t bk = acc1 & ~origin_word(b.src, b.n_msgs, v, w);
                                if (bk) {
                                    const uint64_t bin = gx_in_at_sender<MIX>(h, b, (uint64_t)q, v, w, bk);
                                    atomicAdd(&h.gxb_cnt0[(size_t)b.grp * h.n_pairs + q],
                                              (uint32_t)__popcll(bin) | (uint32_t)__popcll(bk & ~bin) << 16);
                                }  // (cleared before the walk)
                            }
                            if (acc1) *b.got = 1;
                        }
                        if (k1) atomicAdd(&kc[0][t], k1);
                        if (k2) atomicAdd(&kc[1][t], k2);
                        if (k4) atomicAdd(&kc[2][t], k4);
                    }
                    __syncthreads();
                    if ((tb >> lane) & 1) gx_credit(s, q, lane, kc[0][lane], kc[1][lane], kc[2][lane]);
                } else if (lane == 0) {
                    gx_receive_sampled<MIX>(s, h, u, q, r, tb, kk, n, served, delivered, rejected, dups);
                }
                __threadfence_block();  // this pair's receipts before the next pair's duplicate tests
            }
            if (lane == 0) {
                if (answered && h.gx_mark) h.gx_mark[q] = 1;
                h.gx_req[q] = 0;
            }
          }
        }
        __threadfence_block();
        // fulfillPromise: u's promises whose message u received in this exchange
        const uint64_t slots = (uint64_t)(r1 - r0) * S;
        for (uint64_t i = lane; i < slots; i += 64) {
            const size_t z = (size_t)r0 * S + i;
            if (!h.prom_any[z / S] || h.prom_e[z] == 0) continue;
            const uint64_t hd = h.prom_h[z];
            const uint32_t ser = (uint32_t)(hd >> 32), k = (uint32_t)hd;
            for (uint32_t gi = 0; gi < n_gx; ++gi) {  // (the serials from LDS: no chain of descriptor loads)
                if ((gi < 64 ? gser[gi] : h.gx[gi].serial) != ser) continue;
                const GxBatch& b = h.gx[gi];
                if ((b.x[(size_t)u * b.n_words + k / 64] >> (k % 64)) & 1) h.prom_e[z] = 0;
                break;
            }
        }
    }
    gx_flush(h.stats, HB_IWANT_MSGS, iw_msgs);
    gx_flush(h.stats, HB_IWANT_IDS, iw_ids);
    gx_flush(h.stats, HB_IWANT_SERVED, served);
    gx_flush(h.stats, HB_GOSSIP_DELIVERED, delivered);
    gx_flush(h.stats, HB_GOSSIP_REJECTED, rejected);
    gx_flush(h.stats, HB_GOSSIP_DUPLICATES, dups);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)occ, off, 64);
        occ = o > occ ? o : occ;
    }
    if (lane == 0 && occ) atomicMax(h.prom_occ, occ);
}

// Per node v, bit g: v's row of advertised batch g holds a message outside
// its set's common words (batches past 64, first-hand batches: always set;
// recovered batches: set when the node's row is non-empty, from the batch's
// per-node counts).  Thread v reads its W words of any other batch row
// (adjacent nodes, adjacent rows: coalesced).
__global__ __launch_bounds__(256) void k_gx_rhm(const GxBatch* __restrict__ gx, uint32_t n_gx, uint32_t n,
                                                uint64_t* __restrict__ rhm) {
    for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < n; v += gridDim.x * 256u) {
        uint64_t m = n_gx > 64 ? ~0ull : 0ull;
        for (uint32_t g = 0; g < n_gx && g < 64; ++g) {
            const GxBatch& b = gx[g];
            // (one engine: the rows against common2, first-hand batches too — an
            // isolated node empties `common`, not common2; k_gx_ask adds the
            // batches its node is poor in)
            const uint64_t* cw = b.common2 ? b.common2 : b.common;
            if (b.dense && !b.common2) {  // (a set bit only lets the ask read the row: always safe)
                m |= 1ull << g;
                continue;
            }
            if (b.cnt && !b.dense) {  // a recovered batch: the node's count of it (its rows are sparse: most counts 0);
                if (!b.cnt[v]) continue;
                if (!b.common2) {  // a non-empty row is taken as uncommon (safe, as above)
                    m |= 1ull << g;
                    continue;
                }  // (one engine: the non-empty rows against common2 — a round recovers copies at most nodes)
            }
            const uint32_t W = b.n_words;
            const uint64_t* row = b.mem + (size_t)v * W;
            uint64_t any = 0;
            uint32_t w = 0;
            if (!(reinterpret_cast<uintptr_t>(row) & 15u))  // (16-B loads: two words each)
                for (; w + 2 <= W; w += 2) {
                    const ulonglong2 p = *reinterpret_cast<const ulonglong2*>(row + w);
                    any |= (p.x & ~(cw ? cw[w] : 0ull)) | (p.y & ~(cw ? cw[w + 1] : 0ull));
                }
            for (; w < W; ++w) any |= row[w] & ~(cw ? cw[w] : 0ull);
            if (any) m |= 1ull << g;
        }
        rhm[v] = m;
    }
}

// Thread per node v of set blockIdx.y: its W seen words read once (popcount
// for `full`, zeros to the receipt row, an AND per word reduced over the wave
// and the block, one atomic per (block, word)).
__global__ __launch_bounds__(256) void k_gx_setprep(const GxSetPrep* __restrict__ sets, uint32_t n) {
    __shared__ unsigned long long sw[64], sw2[64];
    const GxSetPrep S = sets[blockIdx.y];
    const uint32_t W = S.n_words;
    const bool and_words = S.common != nullptr && W <= 64;
    const bool and2 = and_words && S.common2 != nullptr;
    const bool read = and_words || S.full;
    if (threadIdx.x < 64) sw[threadIdx.x] = sw2[threadIdx.x] = ~0ull;
    __syncthreads();
    const uint32_t stride = gridDim.x * 256u;
    if (W <= 8) {
        // (sets of up to eight words: the lane's words held in registers, ANDed into
        // per-lane accumulators; one wave reduction per word at the end)
        uint64_t a1[8], a2[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) a1[w] = a2[w] = ~0ull;
        for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < n; v += stride) {
            uint64_t x[8];
            uint32_t c = 0;
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                const bool on = (uint32_t)w < W;
                x[w] = on && read ? S.all[(size_t)v * W + w] : ~0ull;
                if (on && read) c += (uint32_t)__popcll(x[w]);
                if (on && S.x) S.x[(size_t)v * W + w] = 0;
            }
            if (S.full) S.full[v] = c == S.n_msgs;
            const bool rich = c + GX_POOR >= S.n_msgs;  // (k_gx_ask's poor test)
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                a1[w] &= x[w];
                if (rich) a2[w] &= x[w];
            }
            if (S.x) {  // the recovered rows' summary beside them (k_gx_merge_sets writes touched nodes only)
                S.x[(size_t)W * n + v] = 0;
                reinterpret_cast<uint32_t*>(S.x + (size_t)W * n + n)[v] = 0;
            }
        }
        if (and_words) {
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                if ((uint32_t)w >= W) break;
                uint64_t b1 = a1[w], b2 = a2[w];
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) {
                    b1 &= (uint64_t)__shfl_xor((long long)b1, off, 64);
                    b2 &= (uint64_t)__shfl_xor((long long)b2, off, 64);
                }
                if ((threadIdx.x % 64) == 0) {
                    atomicAnd(&sw[w], (unsigned long long)b1);
                    if (and2) atomicAnd(&sw2[w], (unsigned long long)b2);
                }
            }
        }
    } else {
        // (a uniform trip count: every lane takes part in the wave reductions)
        for (uint32_t v0 = blockIdx.x * 256u; v0 < n; v0 += stride) {
            const uint32_t v = v0 + threadIdx.x;
            const bool in = v < n;
            uint32_t c = 0;
            for (uint32_t w = 0; w < W; ++w) {
                const uint64_t x = in && read ? S.all[(size_t)v * W + w] : ~0ull;
                if (in) {
                    c += (uint32_t)__popcll(x);
                    if (S.x) S.x[(size_t)v * W + w] = 0;
                }
                if (and_words) {
                    uint64_t a = x;
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) a &= (uint64_t)__shfl_xor((long long)a, off, 64);
                    if ((threadIdx.x % 64) == 0) atomicAnd(&sw[w], (unsigned long long)a);
                }
            }
            if (in && S.full) S.full[v] = c == S.n_msgs;
            if (and2) {  // the nodes missing at most GX_POOR messages: their words again (cached), ANDed
                const bool rich = in && c + GX_POOR >= S.n_msgs;
                for (uint32_t w = 0; w < W; ++w) {
                    uint64_t a = rich ? S.all[(size_t)v * W + w] : ~0ull;
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) a &= (uint64_t)__shfl_xor((long long)a, off, 64);
                    if ((threadIdx.x % 64) == 0) atomicAnd(&sw2[w], (unsigned long long)a);
                }
            }
            if (in && S.x) {  // the recovered rows' summary beside them (k_gx_merge_sets writes touched nodes only)
                S.x[(size_t)W * n + v] = 0;
                reinterpret_cast<uint32_t*>(S.x + (size_t)W * n + n)[v] = 0;
            }
        }
    }
    __syncthreads();
    if (and_words && threadIdx.x < W) atomicAnd(reinterpret_cast<unsigned long long*>(&S.common[threadIdx.x]), sw[threadIdx.x]);
    if (and2 && threadIdx.x < W) atomicAnd(reinterpret_cast<unsigned long long*>(&S.common2[threadIdx.x]), sw2[threadIdx.x]);
}

// Thread per node v of set blockIdx.y: merge its W receipt words and sum the
// recovered row's count and digest as k_mc_summary does (a full word adds
// its word digest, else the id digests of its bits: the same u64 sum).  Only
// the round's touched nodes (GxSetMerge::touch): every other row is zero.
__global__ __launch_bounds__(256) void k_gx_merge_sets(const GxSetMerge* __restrict__ sets, uint32_t n) {
    const GxSetMerge S = sets[blockIdx.y];
    const uint32_t W = S.n_words;
    const uint64_t* word_dig = S.msg_dig + (size_t)W * 64;
    for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < n; v += gridDim.x * 256u) {
        if (S.touch && !((S.touch[v >> 6] >> (v & 63)) & 1)) continue;  // (rows, count, digest: zero)
        uint32_t L = 0, seen = 0;
        uint64_t d = 0;
        for (uint32_t w = 0; w < W; ++w) {
            const size_t i = (size_t)v * W + w;
            uint64_t word = S.x[i];
            if (S.full) seen += (uint32_t)__popcll(S.all[i] | word);  // (the node's seen count after the merge)
            if (!word) continue;
            S.all[i] |= word;
            if (S.chg && !*S.chg) *S.chg = 1;  // (read first: one writer in many stores)
            word &= S.acc[w];
            S.x[i] = word;
            // the recovered copies were validated now: this round's code, ORed into
            // the planes of its 1-bits (a copy received now was unseen, so its
            // code bits are all 0 yet: k_prop_vcodes writes 0 for them, and only
            // accepted receipts ever take a code)
            if (S.vc && word)
                for (uint32_t c = S.code, b = 0; c; c >>= 1, ++b)
                    if (c & 1) S.vc[b * S.plane + i] |= word;
            L += (uint32_t)__popcll(word);
            const uint32_t left = S.n_msgs > w * 64 ? S.n_msgs - w * 64 : 0;
            const uint64_t full = left >= 64 ? ~0ull : ((1ull << left) - 1);
            if (word && word == full) {
                d += word_dig[w];
                continue;
            }
            for (; word; word &= word - 1) d += S.msg_dig[w * 64 + (uint32_t)__builtin_ctzll(word)];
        }
        S.dig[v] = d;
        S.cnt[v] = L;
        if (S.full) S.full[v] = seen == S.n_msgs;
    }
}

// ---- the forwarding of recovered messages (gsx.h (D), GxFwd) -------------------
//
// A delivered message is published on at once (pushMsg -> publishMessage ->
// GossipSubRouter.Publish: pubsub.go:1046-1128, gossipsub.go:943-1013), so the
// nodes that recovered messages by IWANT are the hop-0 frontier of a
// propagation inside the round.  Per hop:
//  k_gxf_mark: a lane per frontier node v pushes "you may get set s" bits to
//    the neighbours v forwards set s's topic to (one atomicOr per pair; the
//    first one lists the receiver);
//  k_gxf_pull: a lane per listed receiver x walks its pairs (x -> v) in
//    ascending v and pulls v's frontier rows (senders ascending: the first
//    deliverer is the lowest sender), with the AcceptFrom gate of x, the
//    origin exclusion and, for the `from` exclusion, the first receipts v took
//    from x at the hop before (counted per (pair, topic), subtracted from the
//    duplicates: a back-sent copy is always one); first receipts are
//    delivered (P2, P3 in the mesh), added to the round's receipt rows (the
//    recovered batch: cached) and fulfil x's promises; duplicates count for P3
//    when x got the message in this round (or, for an old copy, when the set's
//    old_in holds).  Every per-pair state touched belongs to the receiver x.

// v forwards topic t to the peer of pair r = (v -> w) (the gossipsub targets
// of Publish with ReceivedFrom != self: fwd_byte without flood publish, and
// the scores (D) started from).
__device__ __forceinline__ bool gxf_elig(const DevState& s, const HbState& h, uint64_t r, uint32_t v, uint32_t t) {
    const uint8_t pf = s.pflags[r];
    if ((pf & (PAIR_PRESENT | PAIR_CONNECTED)) != (PAIR_PRESENT | PAIR_CONNECTED) || !topic_peer(h.psub, r, t))
        return false;
    const uint8_t ef = h.eflags[r];
    if (ef & EDGE_DIRECT) return true;                                                  // :962-968
    if (!(ef & EDGE_GOSSIPSUB) && s.score[r] >= h.publish_threshold) return true;       // :970-975
    if (t >= s.n_topics) return false;
    return joined_node(h.sub, v, t) ? (s.rflags[flag_index(r, t, s.n_topics)] & REC_IN_MESH) != 0  // :977-999
                                    : ((h.fanout[r] >> t) & 1) != 0;
}

// The words of set S whose message node x published.
__device__ __forceinline__ uint64_t gxf_origin(const GxFwdSet& S, uint32_t x, uint32_t w) {
    return origin_word(S.src, S.n_msgs, x, w);
}

// Hop 0: every node's accepted receipts of the round per set (its frontier
// rows), the frontier list; and each set's origins into srcm (a thread per
// (set, message) in the grid's second half).
__device__ __forceinline__ uint32_t gxf_fout_bits(const DevState& s, const HbState& h, const GxFwd& f, uint64_t r,
                                                  uint32_t v) {
    uint32_t b = 0;
    for (uint32_t ts = 0; ts < f.n_slots; ++ts)
        if (gxf_elig(s, h, r, v, f.slot_topic[ts])) b |= 1u << ts;
    return b;
}
// The run's forwarding slots (fout) of every node's row, node-parallel; hop 0
// over the nodes k_gx_ask listed (only they received in the exchange: every
// other node's receipt rows are zero).
__global__ __launch_bounds__(256) void k_gxf_init(DevState s, HbState h, GxFwd f, uint32_t n, uint32_t n_src_total,
                                                  uint32_t node_lo) {
    if (!f.fout_lazy)
        for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < n; u += gridDim.x * 256u)
            for (int64_t r = h.row_ptr[u]; r < h.row_ptr[u + 1]; ++r)
                f.fout[r] = (uint8_t)gxf_fout_bits(s, h, f, (uint64_t)r, u);
    const uint32_t n_list = h.gx_err[6];
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n_list; i += gridDim.x * 256u) {
        const uint32_t u = h.gx_nodes[i] & ~GX_HEAVY;
        uint64_t m = 0;
        for (uint32_t si = 0; si < f.n_sets; ++si) {
            const GxFwdSet& S = f.sets[si];
            const uint32_t W = S.n_words;
            uint64_t any = 0;
            for (uint32_t w = 0; w < W; ++w) any |= S.x[(size_t)u * W + w] & S.acc[w];
            if (!any) continue;  // (a row is read only where fmask has its set)
            m |= 1ull << si;
            for (uint32_t w = 0; w < W; ++w) S.fr[0][(size_t)u * W + w] = S.x[(size_t)u * W + w] & S.acc[w];
        }
        const uint32_t k = wave_append(&f.fcnt[0], m != 0);
        if (m) {
            f.fmask[0][u] = m;
            f.flist[0][k] = u;
            atomicOr(reinterpret_cast<unsigned long long*>(&f.fbit[0][u >> 6]), 1ull << (u & 63));
        }
    }
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n_src_total; i += gridDim.x * 256u) {
        uint32_t si = 0, base = 0;
        while (base + f.sets[si].n_msgs <= i) base += f.sets[si++].n_msgs;
        const uint32_t x = (uint32_t)(f.sets[si].src[i - base] >> 32) - node_lo;  // (origins are global ids)
        if (x < n) atomicOr(reinterpret_cast<unsigned long long*>(&f.srcm[x]), 1ull << si);
    }
}

// The receiver-side view of the run's forwarding slots on a range shard (fin,
// one gather of the reverse pair's byte; the remote ones arrive after).
__global__ __launch_bounds__(256) void k_gxf_fin(DevState s, HbState h, GxFwd f) {
    for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < h.n_pairs; q += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = h.rev[q];
        uint16_t b = (r == NO_PAIR || (r & HALO)) ? 0 : f.fout[r];
        if (!(h.eflags[q] & EDGE_DIRECT) && s.score[q] < h.graylist) b |= GXF_GRAY;  // AcceptFrom at the owner
        f.fin[q] = b;
    }
}

// The run's eligible senders per receiver (GxFwd::fent), node-parallel, in
// pair order: from fin on a range shard, else fout[rev q] and x's AcceptFrom.
__device__ __forceinline__ void gxf_compact_rows(const DevState& s, const HbState& h, const GxFwd& f) {
    constexpr int CB = 8;  // pairs whose loads are in flight together (rev, then the fout gathers)
    for (uint32_t x = blockIdx.x * 256u + threadIdx.x; x < h.n_nodes; x += gridDim.x * 256u) {
        const int64_t r0 = h.row_ptr[x], r1 = h.row_ptr[x + 1];
        int64_t k = r0;
        for (int64_t q0 = r0; q0 < r1; q0 += CB) {
            uint32_t rr[CB], fi[CB];
#pragma unroll
            for (int j = 0; j < CB; ++j) rr[j] = q0 + j < r1 ? h.rev[q0 + j] : NO_PAIR;
#pragma unroll
            for (int j = 0; j < CB; ++j) {
                if (f.fin) fi[j] = q0 + j < r1 ? (uint32_t)f.fin[q0 + j] : 0u;
                else fi[j] = rr[j] == NO_PAIR ? 0u : (uint32_t)f.fout[rr[j]];
            }
#pragma unroll
            for (int j = 0; j < CB; ++j) {
                if (!(fi[j] & 0xFFu)) continue;
                const int64_t q = q0 + j;
                if (!f.fin && !(h.eflags[q] & EDGE_DIRECT) && s.score[q] < h.graylist) fi[j] |= GXF_GRAY;
                f.fent[k++] = make_uint4((uint32_t)q, rr[j], (uint32_t)h.col[q] - h.node_lo, fi[j]);
            }
        }
        f.fend[x] = (uint32_t)k;
    }
}
__global__ __launch_bounds__(256) void k_gxf_compact(DevState s, HbState h, GxFwd f) { gxf_compact_rows(s, h, f); }

// A hop whose frontier holds more than n / f.dense_div nodes (GXF_DENSE by
// default) pulls at every node (no marking): cheaper than its atomics and lists.
__device__ __forceinline__ bool gxf_dense(const GxFwd& f, uint32_t hop, uint32_t n) {
    return (uint64_t)f.fcnt[hop - 1] * f.dense_div > n;
}
// The eligible-sender lists are there for hop `hop`: on a range shard from hop
// 1 on; on one engine from the run's first dense hop on (its k_gxf_mark builds
// them: a sparse hop's few receivers walk their rows as cheaply, and a run of
// sparse hops never pays for the lists).
__device__ __forceinline__ bool gxf_fent_ready(const GxFwd& f, uint32_t hop, uint32_t n) {
    if (!f.fent) return false;
    if (f.fin) return true;
    for (uint32_t z = 1; z <= hop; ++z)
        if (gxf_dense(f, z, n)) return true;
    return false;
}

// fout of every pair at the run's first hop whose frontier holds more than
// fout_lazy nodes (min(n / GXF_FOUT_DIV, GXF_FOUT_MAX)) (so before its first dense hop, whose
// eligible-sender lists gather it): a run of small frontiers (the light
// heartbeat rounds) evaluates its few senders' slots in place and never
// pays the pass.  Every other hop returns at once.
// A dense hop always finds fout computed (its k_gxf_mark builds the lists
// from it), whatever fout_lazy is: on tiny overlays n / dense_div can fall
// below fout_lazy's floor of one node.
__device__ __forceinline__ bool gxf_fout_ready(const GxFwd& f, uint32_t hop, uint32_t n) {
    if (!f.fout_lazy) return true;
    for (uint32_t z = 1; z <= hop; ++z)
        if (f.fcnt[z - 1] > f.fout_lazy || gxf_dense(f, z, n)) return true;
    return false;
}
__global__ __launch_bounds__(256) void k_gxf_fout_pre(DevState s, HbState h, GxFwd f, uint32_t hop) {
    if (!gxf_fout_ready(f, hop, h.n_nodes) || gxf_fout_ready(f, hop - 1, h.n_nodes)) return;
    for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < h.n_nodes; u += gridDim.x * 256u)
        for (int64_t r = h.row_ptr[u]; r < h.row_ptr[u + 1]; ++r) f.fout[r] = (uint8_t)gxf_fout_bits(s, h, f, (uint64_t)r, u);
}

__device__ __forceinline__ uint64_t gxf_slot_sets(const GxFwd& f, uint32_t slots) {
    uint64_t m = 0;
    for (; slots; slots &= slots - 1) m |= f.slot_sets[__builtin_ctz(slots)];
    return m;
}
__global__ __launch_bounds__(256) void k_gxf_mark(DevState s, HbState h, GxFwd f, uint32_t hop) {
    const uint32_t p = (hop - 1) & 1;
    const uint32_t stride = gridDim.x * 256u;
    if (hop >= 2) {  // the frontier two hops back (this hop's parity): its masks and bits cleared
        const uint32_t n2 = f.fcnt[hop - 2];
        for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n2; i += stride) f.fmask[hop & 1][f.flist[hop & 1][i]] = 0;
        if (n2)
            for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < (h.n_nodes + 63) / 64; i += stride) f.fbit[hop & 1][i] = 0;
    }
    const uint32_t nf = f.fcnt[hop - 1];
    if (gxf_dense(f, hop, h.n_nodes)) {  // a dense hop: the pull visits every node
        if (f.fent && !f.fin && !gxf_fent_ready(f, hop - 1, h.n_nodes)) gxf_compact_rows(s, h, f);  // the first
        return;
    }
    const bool fo_ready = gxf_fout_ready(f, hop, h.n_nodes);
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nf; i += stride) {
        const uint32_t v = f.flist[p][i];
        const uint64_t M = f.fmask[p][v];
        for (int64_t r = h.row_ptr[v]; r < h.row_ptr[v + 1]; ++r) {
            const uint32_t fo = fo_ready ? f.fout[r] : gxf_fout_bits(s, h, f, (uint64_t)r, v);
            if (!fo) continue;
            const uint64_t ok = M & gxf_slot_sets(f, fo);
            if (!ok) continue;
            if (h.rev[r] & HALO) continue;  // a remote receiver: its rank marks it from this rank's entries
            const uint32_t w = (uint32_t)h.col[r] - h.node_lo;
            const unsigned long long old = atomicOr(reinterpret_cast<unsigned long long*>(&f.rmask[w]), ok);
            const uint32_t k = wave_append(&f.rcnt[hop], old == 0);
            if (old == 0) f.rlist[k] = w;
        }
    }
}

// The copies v would send back to x (pair r = (v -> x), topic slot ts): the
// first receipts v took from x at the hop before; hop 1: the IWANT answers x
// served v, old at x (inside the window by their set's old_in); later hops:
// copies x got in this round.  (back: all of them, back_w: those inside x's
// P3 window.)  Hop 1's counts are at r (k_gx_node's pair); a later hop's at
// gxf_bidx of the pull that took them: x's own pair q = (x -> v) when v is
// local (the reads then run along x's row), r when x is on another rank.
__device__ __forceinline__ void gxf_back(const HbState& h, const GxFwd& f, uint32_t hop, uint64_t r, uint64_t q,
                                         uint32_t ts, uint32_t& back, uint32_t& back_w) {
    back = back_w = 0;
    const uint32_t p = (hop - 1) & 1;
    if (hop == 1) {
        if (f.bst0 && f.bst0[r] == f.stamp0) {
            const uint32_t b2 = f.bcnt0[(size_t)f.slot_grp[ts] * h.n_pairs + r];
            back_w = b2 & 0xFFFFu;
            back = back_w + (b2 >> 16);
        }
    } else if (f.bst[p][q] == f.seq + hop - 1) {
        back = back_w = f.bcnt[p][(size_t)q * GXF_SLOTS + ts];
    }
}
// Where the pull of pair q (reverse r) leaves its first-receipt counts for the
// next hop's back-sends: at the reverse pair (read by its owner), or at q
// itself when the peer is on another rank (read by k_gxf_halo here).
__device__ __forceinline__ uint64_t gxf_bidx(uint64_t q, uint32_t r) { return (r & HALO) ? q : (uint64_t)r; }

__global__ __launch_bounds__(256) void k_gxf_pull(DevState s, HbState h, GxFwd f, uint32_t hop) {
    const uint32_t p = (hop - 1) & 1, pw = hop & 1;
    const uint32_t seq_cur = f.seq + hop;
    const uint32_t S_ = h.prom_slots;
    unsigned long long c_new = 0, c_dup = 0, c_gray = 0;
    const bool dense = (uint64_t)f.fcnt[hop - 1] * f.dense_div > h.n_nodes;
    const uint32_t nr = dense ? h.n_nodes : f.rcnt[hop];
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nr; i += gridDim.x * 256u) {
        const uint32_t x = dense ? i : f.rlist[i];
        uint64_t M = f.all_sets;
        if (!dense) {
            M = f.rmask[x];
            f.rmask[x] = 0;
        }
        const uint64_t srcm = f.srcm[x] & M;
        uint64_t newsets = 0;
        const int64_t r0 = h.row_ptr[x], r1 = h.row_ptr[x + 1];
        // x's pairs in blocks of GXF_PB: the filter's loads (eligibility, the
        // frontier bit and mask of the sender) of a block are issued together,
        // then the senders that send are pulled in ascending order
        constexpr int GXF_PB = 8;
        for (int64_t q0 = r0; q0 < r1; q0 += GXF_PB) {
          uint32_t fis[GXF_PB], vs[GXF_PB], rs[GXF_PB];
          uint64_t fms[GXF_PB];
#pragma unroll
          for (int j = 0; j < GXF_PB; ++j) {
              fis[j] = q0 + j < r1 ? (uint32_t)f.fin[q0 + j] : 0u;
              rs[j] = (fis[j] & 0xFFu) ? h.rev[q0 + j] : NO_PAIR;
              vs[j] = (fis[j] & 0xFFu) ? (uint32_t)h.col[q0 + j] - h.node_lo : 0u;  // (local index; unused if remote)
          }
#pragma unroll
          for (int j = 0; j < GXF_PB; ++j) {
              if (!(fis[j] & 0xFFu)) fms[j] = 0;
              else if (rs[j] & HALO) fms[j] = f.hstamp && f.hstamp[q0 + j] == seq_cur;  // a remote sender's entry this hop
              else fms[j] = (f.fbit[p][vs[j] >> 6] >> (vs[j] & 63)) & 1;
          }
#pragma unroll
          for (int j = 0; j < GXF_PB; ++j)
              if (fms[j])
                  fms[j] = ((rs[j] & HALO) ? f.hent[(size_t)f.hidx[q0 + j] * (GXF_HDR + f.rw) + 1] : f.fmask[p][vs[j]]) &
                           M & gxf_slot_sets(f, fis[j] & 0xFFu);
          for (int j = 0; j < GXF_PB; ++j) {
            const uint64_t fv = fms[j];
            if (!fv) continue;  // v forwards none of the run's topics to x, or sends nothing new this hop
            const int64_t q = q0 + j;
            const uint32_t fi = fis[j], v = vs[j];
            const uint32_t r = rs[j];
            const uint64_t* hdr = (r & HALO) ? f.hent + (size_t)f.hidx[q] * (GXF_HDR + f.rw) : nullptr;
            const bool gray = (fi & GXF_GRAY) != 0;  // AcceptFrom at x
            for (uint32_t ts = 0; ts < f.n_slots; ++ts) {
                const uint64_t sm = fv & f.slot_sets[ts];
                if (!sm) continue;
                const uint32_t t = f.slot_topic[ts];
                uint32_t n1 = 0, dt = 0, dw = 0, g = 0;
                for (uint64_t mm = sm; mm; mm &= mm - 1) {
                    const uint32_t si = (uint32_t)__builtin_ctzll(mm);
                    const GxFwdSet& S = f.sets[si];
                    const uint32_t W = S.n_words;
                    const uint64_t* F = hdr ? hdr + GXF_HDR + S.woff : S.fr[p] + (size_t)v * W;
                    uint64_t* X = S.x + (size_t)x * W;
                    const uint64_t* A = S.all + (size_t)x * W;
                    uint64_t* NF = S.fr[pw] + (size_t)x * W;
                    const bool isrc = (srcm >> si) & 1;
                    for (uint32_t w = 0; w < W; ++w) {
                        uint64_t snd = F[w];
                        if (isrc && snd) snd &= ~gxf_origin(S, x + h.node_lo, w);  // not back to the origin (:1006-1009)
                        if (!snd) continue;
                        if (gray) {
                            g += (uint32_t)__popcll(snd);
                            continue;
                        }
                        const uint64_t xw = X[w];
                        const uint64_t nw = snd & ~(A[w] | xw);
                        const uint64_t dup = snd & ~nw;
                        dt += (uint32_t)__popcll(dup);
                        // in-window duplicates: those x got this round; an old copy by its validation time
                        dw += (uint32_t)__popcll((dup & xw) | old_inside(S.old_in, S.vc, (size_t)x * W + w, dup & ~xw));
                        if (nw) {
                            n1 += (uint32_t)__popcll(nw);
                            X[w] = xw | nw;
                            if (!((newsets >> si) & 1)) {
                                newsets |= 1ull << si;
                                for (uint32_t z = 0; z < W; ++z) NF[z] = 0;
                            }
                            NF[w] |= nw;
                        }
                    }
                }
                // the copies v would send back to x: the first receipts v took from x last hop
                // (hop 1: the copies v served x from its cache, old at x: inside the
                // window by their set's old_in; later hops: x got them in this round)
                uint32_t back = 0, back_w = 0;
                if (hdr) {  // counted by the sender's rank (k_gxf_halo)
                    back = (uint32_t)(hdr[2 + ts / 4] >> (16 * (ts % 4))) & 0xFFFFu;
                    back_w = (uint32_t)(hdr[4 + ts / 4] >> (16 * (ts % 4))) & 0xFFFFu;
                } else {
                    gxf_back(h, f, hop, r, (uint64_t)q, ts, back, back_w);
                }
                if (gray) {
                    g -= back;
                } else {
                    dt -= back;
                    dw -= back_w;
                }
                c_new += n1;
                c_dup += dt;
                c_gray += g;
                if (n1 | dw) {
                    gx_credit(s, (uint64_t)q, t, n1, dw, 0);
                    if (h.gx_mark) h.gx_mark[q] = 1;
                }
                if (n1) {
                    const uint64_t bi = gxf_bidx((uint64_t)q, r);
                    if (f.bst[pw][bi] != seq_cur) {
                        f.bst[pw][bi] = seq_cur;
                        for (uint32_t z = 0; z < GXF_SLOTS; ++z) f.bcnt[pw][bi * GXF_SLOTS + z] = 0;
                    }
                    f.bcnt[pw][bi * GXF_SLOTS + ts] = (uint16_t)n1;
                }
            }
          }
        }
        const uint32_t slot_x = wave_append(&f.fcnt[hop], newsets != 0);
        if (!newsets) continue;
        for (uint64_t mm = newsets; mm; mm &= mm - 1) {  // (read first: one writer in a thousand stores)
            uint8_t* g = f.sets[__builtin_ctzll(mm)].got;
            if (!*g) *g = 1;
        }
        f.fmask[pw][x] = newsets;
        f.flist[pw][slot_x] = x;
        atomicOr(reinterpret_cast<unsigned long long*>(&f.fbit[pw][x >> 6]), 1ull << (x & 63));
        if (h.gx_touch) atomicOr(reinterpret_cast<unsigned long long*>(&h.gx_touch[x >> 6]), 1ull << (x & 63));
        // fulfillPromise (:119-126): x's promises of messages it now has
        for (uint64_t z = (uint64_t)r0 * S_; z < (uint64_t)r1 * S_; ++z) {
            if (z % S_ == 0 && !h.prom_any[z / S_]) {  // no promise on this pair
                z += S_ - 1;
                continue;
            }
            if (h.prom_e[z] == 0) continue;
            const uint64_t hd = h.prom_h[z];
            const uint32_t ser = (uint32_t)(hd >> 32), k = (uint32_t)hd;
            for (uint64_t mm = newsets; mm; mm &= mm - 1) {
                const GxFwdSet& S = f.sets[__builtin_ctzll(mm)];
                if (S.serial != ser) continue;
                if (k < S.n_msgs && ((S.x[(size_t)x * S.n_words + k / 64] >> (k % 64)) & 1)) h.prom_e[z] = 0;
                break;
            }
        }
    }
    unsigned long long v[3] = {c_new, c_dup, c_gray};
    const uint32_t slot[3] = {HB_FWD_DELIVERED, HB_FWD_DUPLICATES, HB_FWD_GRAYLISTED};
    block_count<3>(v, h.stats, slot);
}

// k_gxf_pull with G lanes per receiver x splitting its SENDERS (lane c takes
// pairs c, c + G, ... in rounds of G), as k_prop_hop_fast1 does: a round's G
// senders are gathered together and "not from a lower sender" becomes an
// exclusive prefix-OR over the group's sends, word by word.  Every per-pair
// count (first receipts, duplicates, graylisted copies, back-sends) and credit
// stays with the pair's lane; every lane writes x's receipt / frontier words
// with the same values (so each re-reads its own stores).  Same results as
// k_gxf_pull.
template <int G>
__device__ __forceinline__ uint64_t gxf_gor(uint64_t x) {  // OR over the group (aligned), every lane
#pragma unroll
    for (int o = 1; o < G; o <<= 1) x |= (uint64_t)__shfl_xor((unsigned long long)x, o, G);
    return x;
}
// B rounds of G senders have their filter loads (slot byte, reverse pair, peer;
// frontier bit; frontier mask) issued together, three latencies per B rounds.
// MIX: some set of the run has a P3 window that splits its old copies (old_in
// 2, per-copy codes: vc_inside); a separate instance, so the common one keeps
// its registers (the per-copy path costs ~23 VGPRs, a wave per SIMD).
template <int G, int B, bool MIX>
__device__ __forceinline__ void gxf_pull_run(DevState& s, HbState& h, GxFwd& f, uint32_t hop, bool dense) {
    const uint32_t p = (hop - 1) & 1, pw = hop & 1;
    const uint32_t seq_cur = f.seq + hop;
    const uint32_t S_ = h.prom_slots;
    const uint32_t lc = threadIdx.x % G;
    unsigned long long c_new = 0, c_dup = 0, c_gray = 0;
    const bool fe = gxf_fent_ready(f, hop, h.n_nodes);
    const bool fo_ready = fe || gxf_fout_ready(f, hop, h.n_nodes);
    const uint32_t nr = dense ? h.n_nodes : f.rcnt[hop];
    for (uint32_t i = (blockIdx.x * 256u + threadIdx.x) / G; i < nr; i += gridDim.x * (256u / G)) {
        const uint32_t x = dense ? i : f.rlist[i];
        uint64_t M = f.all_sets;
        if (!dense) {
            M = f.rmask[x];
            if (lc == 0) f.rmask[x] = 0;
        }
        const uint64_t srcm = f.srcm[x] & M;
        uint64_t newsets = 0;  // (the same in every lane of the group)
        const int64_t r0 = h.row_ptr[x], r1 = h.row_ptr[x + 1];
        const int64_t e1 = fe ? (int64_t)f.fend[x] : r1;  // x's eligible senders (or every pair)
        for (int64_t qb0 = r0; qb0 < e1; qb0 += G * B) {
          uint32_t fis[B], rqs[B], vqs[B], qs[B];
          uint64_t fms[B];
#pragma unroll
          for (int j = 0; j < B; ++j) {
              const int64_t ei = qb0 + j * G + lc;
              const bool in = ei < e1;
              if (fe) {  // one 16-B load per sender: (q, rev q, peer, fin)
                  const uint4 en = in ? f.fent[ei] : make_uint4(0u, NO_PAIR, 0u, 0u);
                  qs[j] = en.x;
                  rqs[j] = en.y;
                  vqs[j] = en.z;
                  fis[j] = en.w;
              } else {
                  qs[j] = (uint32_t)ei;
                  fis[j] = in && f.fin ? (uint32_t)f.fin[ei] : 0u;
                  rqs[j] = in ? h.rev[ei] : NO_PAIR;
                  vqs[j] = in ? (uint32_t)h.col[ei] - h.node_lo : 0u;  // (local index; unused if remote)
              }
          }
          if (f.fin || fe) {
#pragma unroll
            for (int j = 0; j < B; ++j) {
                fms[j] = 0;
                if (!(fis[j] & 0xFFu)) continue;
                if (rqs[j] & HALO) fms[j] = f.hstamp && f.hstamp[qs[j]] == seq_cur;  // a remote sender's entry this hop
                else fms[j] = (f.fbit[p][vqs[j] >> 6] >> (vqs[j] & 63)) & 1;  // (L2-resident: filters the mask loads)
            }
#pragma unroll
            for (int j = 0; j < B; ++j) {
                if (fms[j])
                    fms[j] = ((rqs[j] & HALO) ? f.hent[(size_t)f.hidx[qs[j]] * (GXF_HDR + f.rw) + 1] : f.fmask[p][vqs[j]]) &
                             M & gxf_slot_sets(f, fis[j] & 0xFFu);
            }
          } else {  // one engine: the frontier bit of every peer first, the slots of the senders in it
#pragma unroll
            for (int j = 0; j < B; ++j)
                fms[j] = rqs[j] != NO_PAIR && ((f.fbit[p][vqs[j] >> 6] >> (vqs[j] & 63)) & 1);
#pragma unroll
            for (int j = 0; j < B; ++j) {
                if (!fms[j]) continue;
                const uint64_t q = qs[j];
                fis[j] = (fo_ready ? (uint32_t)f.fout[rqs[j]] : gxf_fout_bits(s, h, f, (uint64_t)rqs[j], vqs[j])) |
                         ((!(h.eflags[q] & EDGE_DIRECT) && s.score[q] < h.graylist) ? GXF_GRAY : 0u);  // AcceptFrom at x
                fms[j] = f.fmask[p][vqs[j]] & M & gxf_slot_sets(f, fis[j] & 0xFFu);
            }
          }
          for (int j = 0; j < B; ++j) {  // the rounds in sender order
            const int64_t qb = qb0 + j * G;
            if (qb >= e1) break;
            const int64_t q = qs[j];
            const uint32_t fi = fis[j];
            const uint32_t r = (fi & 0xFFu) ? rqs[j] : NO_PAIR;
            const uint32_t v = (fi & 0xFFu) ? vqs[j] : 0u;
            const uint64_t fv = fms[j];
            if (!gxf_gor<G>(fv)) continue;  // no sender of the round sends anything new
            const uint64_t* hdr = (fv && (r & HALO)) ? f.hent + (size_t)f.hidx[q] * (GXF_HDR + f.rw) : nullptr;
            const bool gray = (fi & GXF_GRAY) != 0;  // AcceptFrom at x
            for (uint32_t ts = 0; ts < f.n_slots; ++ts) {
                const uint64_t sm = fv & f.slot_sets[ts];
                const uint64_t smg = gxf_gor<G>(sm);
                if (!smg) continue;
                const uint32_t t = f.slot_topic[ts];
                uint32_t n1 = 0, dt = 0, dw = 0, g = 0;
                for (uint64_t mm = smg; mm; mm &= mm - 1) {
                    const uint32_t si = (uint32_t)__builtin_ctzll(mm);
                    const GxFwdSet& S = f.sets[si];
                    const uint32_t W = S.n_words;
                    const bool mine = (sm >> si) & 1;
                    const uint64_t* F = !mine ? nullptr : hdr ? hdr + GXF_HDR + S.woff : S.fr[p] + (size_t)v * W;
                    uint64_t* X = S.x + (size_t)x * W;
                    const uint64_t* A = S.all + (size_t)x * W;
                    uint64_t* NF = S.fr[pw] + (size_t)x * W;
                    const bool isrc = (srcm >> si) & 1;
                    for (uint32_t w = 0; w < W; ++w) {
                        uint64_t snd = mine ? F[w] : 0ull;
                        if (isrc && snd) snd &= ~gxf_origin(S, x + h.node_lo, w);  // not back to the origin (:1006-1009)
                        if (gray) {
                            g += (uint32_t)__popcll(snd);
                            snd = 0;  // dropped at x: delivers nothing
                        }
                        // a word no sender of the round sends: nothing to receive or count
                        if (!((__ballot(snd != 0) >> (__lane_id() & ~(uint32_t)(G - 1))) & ((1ull << G) - 1))) continue;
                        const uint64_t xw = X[w], have = A[w] | xw;
                        uint64_t incl = snd;  // the group's sends so far, in sender order
#pragma unroll
                        for (int o = 1; o < G; o <<= 1) {
                            const uint64_t y = (uint64_t)__shfl_up((unsigned long long)incl, o, G);
                            if (lc >= (uint32_t)o) incl |= y;
                        }
                        uint64_t excl = (uint64_t)__shfl_up((unsigned long long)incl, 1, G);
                        if (lc == 0) excl = 0;
                        const uint64_t all_g = (uint64_t)__shfl((unsigned long long)incl, G - 1, G);
                        const uint64_t nw = snd & ~(have | excl);  // not seen, not from a lower sender
                        const uint64_t dup = snd & ~nw;
                        dt += (uint32_t)__popcll(dup);
                        // in-window duplicates: those x got this round (before this hop, or first
                        // from a lower sender of this one); an old copy by its validation time
                        const uint64_t cur = dup & (xw | (excl & ~have));
                        if (MIX) dw += (uint32_t)__popcll(cur | old_inside(S.old_in, S.vc, (size_t)x * W + w, dup & ~cur));
                        else dw += (uint32_t)__popcll(S.old_in ? dup : cur);
                        n1 += (uint32_t)__popcll(nw);
                        const uint64_t gn = all_g & ~have;  // the group's first receipts of the word
                        if (gn) {
                            X[w] = xw | gn;
                            if (!((newsets >> si) & 1)) {  // x's first receipt of the set this hop: its row
                                newsets |= 1ull << si;      // written whole (no read of the word back)
                                for (uint32_t z = 0; z < W; ++z) NF[z] = z == w ? gn : 0ull;
                            } else {
                                NF[w] |= gn;
                            }
                        }
                    }
                }
                if (!sm) continue;  // (this lane's pair sends nothing of the slot)
                // the copies v would send back to x: the first receipts v took from x last hop
                uint32_t back = 0, back_w = 0;
                if (hdr) {  // counted by the sender's rank (k_gxf_halo)
                    back = (uint32_t)(hdr[2 + ts / 4] >> (16 * (ts % 4))) & 0xFFFFu;
                    back_w = (uint32_t)(hdr[4 + ts / 4] >> (16 * (ts % 4))) & 0xFFFFu;
                } else {
                    gxf_back(h, f, hop, r, (uint64_t)q, ts, back, back_w);
                }
                if (gray) {
                    g -= back;
                } else {
                    dt -= back;
                    dw -= back_w;
                }
                c_new += n1;
                c_dup += dt;
                c_gray += g;
                if (n1 | dw) {
                    gx_credit(s, (uint64_t)q, t, n1, dw, 0);
                    if (h.gx_mark) h.gx_mark[q] = 1;
                }
                if (n1) {
                    const uint64_t bi = gxf_bidx((uint64_t)q, r);
                    if (f.bst[pw][bi] != seq_cur) {
                        f.bst[pw][bi] = seq_cur;
                        for (uint32_t z = 0; z < GXF_SLOTS; ++z) f.bcnt[pw][bi * GXF_SLOTS + z] = 0;
                    }
                    f.bcnt[pw][bi * GXF_SLOTS + ts] = (uint16_t)n1;
                }
            }
          }
        }
        const uint32_t slot_x = wave_append(&f.fcnt[hop], newsets != 0 && lc == 0);
        if (!newsets) continue;
        if (lc == 0) {
            for (uint64_t mm = newsets; mm; mm &= mm - 1) {  // (read first: one writer in a thousand stores)
                uint8_t* gp = f.sets[__builtin_ctzll(mm)].got;
                if (!*gp) *gp = 1;
            }
            f.fmask[pw][x] = newsets;
            f.flist[pw][slot_x] = x;
            atomicOr(reinterpret_cast<unsigned long long*>(&f.fbit[pw][x >> 6]), 1ull << (x & 63));
            if (h.gx_touch) atomicOr(reinterpret_cast<unsigned long long*>(&h.gx_touch[x >> 6]), 1ull << (x & 63));
        }
        // fulfillPromise (:119-126): x's promises of messages it now has (a pair's
        // promises are its own: the group's lanes take x's pairs c, c + G, ...)
        for (int64_t qq = r0 + lc; qq < r1; qq += G) {
            if (!h.prom_any[qq]) continue;  // no promise on this pair
            for (uint64_t z = (uint64_t)qq * S_; z < (uint64_t)(qq + 1) * S_; ++z) {
                if (h.prom_e[z] == 0) continue;
                const uint64_t hd = h.prom_h[z];
                const uint32_t ser = (uint32_t)(hd >> 32), k = (uint32_t)hd;
                for (uint64_t mm = newsets; mm; mm &= mm - 1) {
                    const GxFwdSet& S = f.sets[__builtin_ctzll(mm)];
                    if (S.serial != ser) continue;
                    if (k < S.n_msgs && ((S.x[(size_t)x * S.n_words + k / 64] >> (k % 64)) & 1)) h.prom_e[z] = 0;
                    break;
                }
            }
        }
    }
    unsigned long long vv[3] = {c_new, c_dup, c_gray};
    const uint32_t slot[3] = {HB_FWD_DELIVERED, HB_FWD_DUPLICATES, HB_FWD_GRAYLISTED};
    block_count<3>(vv, h.stats, slot);
}
// GS lanes per receiver on a sparse hop (few receivers: a row spread over
// more lanes), GD on a dense one (every node: more receivers per wave; measured
// on the heartbeat's forwarding, 1M nodes: GD = 2 pulls a dense hop ~8 % faster
// than 4, GS = 4 a sparse one faster than 2).  The hop's kind is uniform.
template <int GS, int GD, int B, bool MIX>
__global__ __launch_bounds__(256) void k_gxf_pull_g(DevState s, HbState h, GxFwd f, uint32_t hop) {
    if (gxf_dense(f, hop, h.n_nodes)) gxf_pull_run<GD, B, MIX>(s, h, f, hop, true);
    else gxf_pull_run<GS, B, MIX>(s, h, f, hop, false);
}

// ---- the exchange across range shards (gsx_gx_*; gsx.h) -------------------------
//
// Everything (D) computes belongs to the receiver of an IHAVE (its counters,
// promises, records, receipts and cache), so a cross-shard pair needs from the
// sender's rank only: the topics of the IHAVE and whether the sender answers
// IWANTs (its score of the receiver), and the sender's cache rows of the
// advertised batches when they hold an uncommon message (gx_rhm over the
// common words of every rank).  The forwarding needs per cross-shard pair the
// sender's topic slots (fout) once per run, and per hop the sender's frontier
// rows with its back-send counts: all fixed-size entries routed by the shard
// plan's receive slots.


__global__ __launch_bounds__(256) void k_gxs_pack_ihave(DevState s, HbState h, GxsPlan P, uint64_t* out) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < P.n_send; j += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = P.send_pair[j];
        uint64_t w0 = 0, w1 = 0;
        if (r != NO_PAIR) {
            w0 = h.gxs_out[r];
            w1 = !(s.score[r] < h.gossip_threshold);  // handleIWant's gate at the sender (:683-688)
        }
        out[2 * j] = w0;
        out[2 * j + 1] = w1;
    }
}

__global__ __launch_bounds__(256) void k_gxs_recv_ihave(HbState h, const uint64_t* in, const uint32_t* halo_pair,
                                                        uint64_t n_recv) {
    for (uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x; k < n_recv; k += (uint64_t)gridDim.x * 256u) {
        const uint32_t q = halo_pair[k];
        h.ihave_bits[q] = in[2 * k];
        h.gxs_rans[q] = (uint8_t)(in[2 * k + 1] & 1);
        h.gxs_hidx[q] = NO_PAIR;
    }
}

// out null: count the entries per destination; else pack them at off[dest].
__global__ __launch_bounds__(256) void k_gxs_rows(HbState h, GxsPlan P, const GxBatch* __restrict__ gx, uint32_t n_gx,
                                                  unsigned long long* cnt, const uint64_t* off, uint64_t* out) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < P.n_send; j += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = P.send_pair[j];
        if (r == NO_PAIR || !h.gxs_out[r]) continue;
        const uint32_t v = P.pair_obs[r];
        if (!h.gx_rhm[v]) continue;  // only common messages in v's rows: nothing to ask
        const uint32_t d = P.send_dest[j];
        const unsigned long long k = atomicAdd(&cnt[d], 1ull);
        if (!out) continue;
        uint64_t* e = out + (size_t)(off[d] + k) * gxs_ew(h);
        e[0] = P.dest_halo_base[d] + (j - P.send_base[d]);  // the receive slot at the destination
        // a truncated list reaches the receiver as its subset: the rows of that
        // topic's batches go masked with the subset row v kept for this pair, so
        // the receiver's handleIHave sees exactly the ids of the IHAVE it got
        const uint64_t tro = h.gxs_tro ? h.gxs_tro[r] : 0ull;
        for (uint32_t g = 0; g < n_gx; ++g) {
            const GxBatch& b = gx[g];
            const uint64_t* sub = nullptr;
            if ((tro >> b.topic) & 1) {
                const GxSub& G = h.gsubs[b.topic];
                sub = G.pool + (size_t)G.idx[r] * G.tw + b.row_off;
            }
            for (uint32_t w = 0; w < b.n_words; ++w) {
                uint64_t m = b.mem[(size_t)v * b.n_words + w];
                if (sub) m &= sub[w];
                e[1 + b.woff + w] = m;
                // the mixed sets: which of v's copies are inside the window at v (hop-1 back-sends)
                if (h.gxs_vin) e[b.vin_off + w] = b.old_in == 2 ? vc_inside(b.vc, (size_t)v * b.n_words + w, m) : 0ull;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_gxs_rows_recv(HbState h, const uint64_t* in, uint64_t n,
                                                       const uint32_t* halo_pair) {
    for (uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256u)
        h.gxs_hidx[halo_pair[in[k * gxs_ew(h)]]] = (uint32_t)k;
}

__global__ __launch_bounds__(256) void k_gxf_pack_fout(GxFwd f, GxsPlan P, uint64_t* out) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < P.n_send; j += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = P.send_pair[j];
        out[j] = r == NO_PAIR ? 0ull : f.fout[r];
    }
}

__global__ __launch_bounds__(256) void k_gxf_recv_fout(GxFwd f, const uint64_t* in, const uint32_t* halo_pair,
                                                       uint64_t n_recv) {
    for (uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x; k < n_recv; k += (uint64_t)gridDim.x * 256u)
        f.fin[halo_pair[k]] |= (uint16_t)(in[k] & 0xFFu);
}

// A hop's frontier entries of this rank's senders to remote receivers (out
// null: counted per destination).
__global__ __launch_bounds__(256) void k_gxf_halo(HbState h, GxFwd f, GxsPlan P, uint32_t hop,
                                                  unsigned long long* cnt, const uint64_t* off, uint64_t* out) {
    const uint32_t p = (hop - 1) & 1;
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < P.n_send; j += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = P.send_pair[j];
        if (r == NO_PAIR) continue;
        const uint32_t fo = f.fout[r];
        if (!fo) continue;
        const uint32_t v = P.pair_obs[r];
        if (!((f.fbit[p][v >> 6] >> (v & 63)) & 1)) continue;
        const uint64_t M = f.fmask[p][v] & gxf_slot_sets(f, fo);
        if (!M) continue;
        const uint32_t d = P.send_dest[j];
        const unsigned long long k = atomicAdd(&cnt[d], 1ull);
        if (!out) continue;
        uint64_t* e = out + (size_t)(off[d] + k) * (GXF_HDR + f.rw);
        e[0] = P.dest_halo_base[d] + (j - P.send_base[d]);
        e[1] = M;
        uint64_t b01[2] = {0, 0}, w01[2] = {0, 0};
        for (uint32_t ts = 0; ts < f.n_slots; ++ts) {
            uint32_t back, back_w;
            gxf_back(h, f, hop, r, r, ts, back, back_w);  // (x remote: the counts are at r)
            b01[ts / 4] |= (uint64_t)back << (16 * (ts % 4));
            w01[ts / 4] |= (uint64_t)back_w << (16 * (ts % 4));
        }
        e[2] = b01[0];
        e[3] = b01[1];
        e[4] = w01[0];
        e[5] = w01[1];
        for (uint32_t si = 0; si < f.n_sets; ++si) {
            const GxFwdSet& S = f.sets[si];
            const bool in = (M >> si) & 1;
            for (uint32_t w = 0; w < S.n_words; ++w)
                e[GXF_HDR + S.woff + w] = in ? S.fr[p][(size_t)v * S.n_words + w] : 0ull;
        }
    }
}

// The entries other ranks sent for this hop: per receive slot the entry, and
// its receiver marked (sparse hops; a dense hop pulls at every node).
__global__ __launch_bounds__(256) void k_gxf_halo_recv(HbState h, GxFwd f, uint32_t hop, const uint64_t* in,
                                                       uint64_t n, const uint32_t* halo_pair,
                                                       const uint32_t* halo_node) {
    const bool dense = (uint64_t)f.fcnt[hop - 1] * f.dense_div > h.n_nodes;
    for (uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256u) {
        const uint64_t* e = in + (size_t)k * (GXF_HDR + f.rw);
        const uint64_t slot = e[0];
        const uint32_t q = halo_pair[slot], x = halo_node[slot];
        f.hstamp[q] = f.seq + hop;
        f.hidx[q] = (uint32_t)k;
        if (dense) continue;
        const unsigned long long old = atomicOr(reinterpret_cast<unsigned long long*>(&f.rmask[x]), e[1]);
        const uint32_t at = wave_append(&f.rcnt[hop], old == 0);
        if (old == 0) f.rlist[at] = x;
    }
}

// (entries for rank d, this rank's frontier of the hop before) per destination
// (gsx_gxf_pack_dev: one all-to-all of these pairs tells every rank its entry
// splits and, summed, whether the last hop left a frontier anywhere).
__global__ void k_gxf_pack_counts(const unsigned long long* __restrict__ cnt, const uint32_t* __restrict__ front,
                                  uint32_t world, int64_t* __restrict__ out) {
    const uint32_t d = threadIdx.x;
    if (d >= world) return;
    out[2 * d] = (int64_t)cnt[d];
    out[2 * d + 1] = (int64_t)*front;
}

static inline unsigned gx_blocks(uint64_t n, unsigned bs, unsigned cap) {
    const uint64_t b = (n + bs - 1) / bs;
    return (unsigned)(b < cap ? b : cap);
}

hipError_t launch_gx_promises(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gx_promises, dim3(gx_blocks(h.n_pairs, 256, COUNTER_GRID)), dim3(256), 0, st, s, h);
    return hipGetLastError();
}

hipError_t launch_gx_rhm(const GxBatch* gx, uint32_t n_gx, uint32_t n_nodes, uint64_t* rhm, hipStream_t st) {
    if (n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gx_rhm, dim3(gx_blocks(n_nodes, 256, 4096)), dim3(256), 0, st, gx, n_gx, n_nodes, rhm);
    return hipGetLastError();
}

hipError_t launch_gx_setprep(const GxSetPrep* sets, uint32_t n_sets, uint32_t n_nodes, hipStream_t st) {
    if (n_sets == 0 || n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gx_setprep, dim3(gx_blocks(n_nodes, 256, 512), n_sets), dim3(256), 0, st, sets, n_nodes);
    return hipGetLastError();
}

hipError_t launch_gx_merge_sets(const GxSetMerge* sets, uint32_t n_sets, uint32_t n_nodes, hipStream_t st) {
    if (n_sets == 0 || n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gx_merge_sets, dim3(gx_blocks(n_nodes, 256, 512), n_sets), dim3(256), 0, st, sets, n_nodes);
    return hipGetLastError();
}

hipError_t launch_gx_exchange(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gx_ask, dim3(gx_blocks(h.n_nodes, 64, 8192)), dim3(64), 0, st, s, h);
    // the listed nodes (their count is on the device): a wave each, grid-stride
    if (h.gx_mixed) hipLaunchKernelGGL(k_gx_node<true>, dim3(8192), dim3(64), 0, st, s, h);
    else hipLaunchKernelGGL(k_gx_node<false>, dim3(8192), dim3(64), 0, st, s, h);
    return hipGetLastError();
}

hipError_t launch_gxf_init(const DevState& s, const HbState& h, const GxFwd& f, uint32_t n_src_total,
                           hipStream_t st) {
    const uint64_t n = std::max<uint64_t>(h.n_nodes, n_src_total);
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxf_init, dim3(gx_blocks(n, 256, 4096)), dim3(256), 0, st, s, h, f, h.n_nodes, n_src_total,
                       h.node_lo);
    if (f.fin) hipLaunchKernelGGL(k_gxf_fin, dim3(gx_blocks(h.n_pairs, 256, 8192)), dim3(256), 0, st, s, h, f);
    return hipGetLastError();
}

// One hop (hop >= 1): its grids are sized for the largest frontier / receiver
// list (the counts are on the device: an empty hop's threads exit at once).
hipError_t launch_gxf_hop(const DevState& s, const HbState& h, const GxFwd& f, uint32_t hop, hipStream_t st) {
    if (hop == 1 && f.fent && f.fin)  // the shard's eligible senders (the remote ones' fin bits have arrived by now)
        hipLaunchKernelGGL(k_gxf_compact, dim3(gx_blocks(h.n_nodes, 256, 4096)), dim3(256), 0, st, s, h, f);
    if (f.fout_lazy) hipLaunchKernelGGL(k_gxf_fout_pre, dim3(gx_blocks(h.n_nodes, 256, 2048)), dim3(256), 0, st, s, h, f, hop);
    hipLaunchKernelGGL(k_gxf_mark, dim3(gx_blocks(h.n_nodes, 256, 4096)), dim3(256), 0, st, s, h, f, hop);
    static const int gl = [] {  // receivers' lanes: GSX_GXF_G = 1 (k_gxf_pull), 2, 4 (default), 8
        const char* v = getenv("GSX_GXF_G");
        return v ? atoi(v) : 4;
    }();
    static const int gd = [] {  // GSX_GXF_GD = 4: G = 4 on dense hops too (default 2 there)
        const char* v = getenv("GSX_GXF_GD");
        return v ? atoi(v) : 2;
    }();
    static const int gb = [] {  // GSX_GXF_B = 2: filter batches of two rounds (G = 4)
        const char* v = getenv("GSX_GXF_B");
        return v ? atoi(v) : 1;
    }();
    static const unsigned gcap = [] {  // GSX_GXF_GRID: the pull's block cap (A/B)
        const char* v = getenv("GSX_GXF_GRID");
        return v && atoi(v) > 0 ? (unsigned)atoi(v) : 2048u;
    }();
    const unsigned gp = gx_blocks(h.n_nodes, 256 / gl, gcap);
#define GXF_PULL(G_, GD_, B_)                                                                                 \
    do {                                                                                                      \
        if (f.mixed) hipLaunchKernelGGL((k_gxf_pull_g<G_, GD_, B_, true>), dim3(gp), dim3(256), 0, st, s, h, f, hop); \
        else hipLaunchKernelGGL((k_gxf_pull_g<G_, GD_, B_, false>), dim3(gp), dim3(256), 0, st, s, h, f, hop);        \
    } while (0)
    if (gl == 8) GXF_PULL(8, 8, 1);
    else if (gl == 4 && gb == 2) GXF_PULL(4, 4, 2);
    else if (gl == 4 && gd == 4) GXF_PULL(4, 4, 1);
    else if (gl == 4) GXF_PULL(4, 2, 1);
    else if (gl == 2) GXF_PULL(2, 2, 1);
    else if (!f.fin) GXF_PULL(1, 1, 1);
    else hipLaunchKernelGGL(k_gxf_pull, dim3(gp), dim3(256), 0, st, s, h, f, hop);
#undef GXF_PULL
    return hipGetLastError();
}

static inline unsigned gx_grid(uint64_t n) { return gx_blocks(n ? n : 1, 256, 4096); }

hipError_t launch_gxs_pack_ihave(const DevState& s, const HbState& h, const GxsPlan& P, uint64_t* out, hipStream_t st) {
    if (P.n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxs_pack_ihave, dim3(gx_grid(P.n_send)), dim3(256), 0, st, s, h, P, out);
    return hipGetLastError();
}
hipError_t launch_gxs_recv_ihave(const HbState& h, const uint64_t* in, const uint32_t* halo_pair, uint64_t n_recv,
                                 hipStream_t st) {
    if (n_recv == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxs_recv_ihave, dim3(gx_grid(n_recv)), dim3(256), 0, st, h, in, halo_pair, n_recv);
    return hipGetLastError();
}
hipError_t launch_gxs_rows(const HbState& h, const GxsPlan& P, const GxBatch* gx, uint32_t n_gx,
                           unsigned long long* cnt, const uint64_t* off, uint64_t* out, hipStream_t st) {
    if (P.n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxs_rows, dim3(gx_grid(P.n_send)), dim3(256), 0, st, h, P, gx, n_gx, cnt, off, out);
    return hipGetLastError();
}
hipError_t launch_gxs_rows_recv(const HbState& h, const uint64_t* in, uint64_t n, const uint32_t* halo_pair,
                                hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxs_rows_recv, dim3(gx_grid(n)), dim3(256), 0, st, h, in, n, halo_pair);
    return hipGetLastError();
}
hipError_t launch_gxf_pack_fout(const GxFwd& f, const GxsPlan& P, uint64_t* out, hipStream_t st) {
    if (P.n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxf_pack_fout, dim3(gx_grid(P.n_send)), dim3(256), 0, st, f, P, out);
    return hipGetLastError();
}
hipError_t launch_gxf_recv_fout(const GxFwd& f, const uint64_t* in, const uint32_t* halo_pair, uint64_t n_recv,
                                hipStream_t st) {
    if (n_recv == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxf_recv_fout, dim3(gx_grid(n_recv)), dim3(256), 0, st, f, in, halo_pair, n_recv);
    return hipGetLastError();
}
hipError_t launch_gxf_halo(const HbState& h, const GxFwd& f, const GxsPlan& P, uint32_t hop, unsigned long long* cnt,
                           const uint64_t* off, uint64_t* out, hipStream_t st) {
    if (P.n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxf_halo, dim3(gx_grid(P.n_send)), dim3(256), 0, st, h, f, P, hop, cnt, off, out);
    return hipGetLastError();
}
hipError_t launch_gxf_pack_counts(const unsigned long long* cnt, const uint32_t* front, uint32_t world, int64_t* out,
                                  hipStream_t st) {
    hipLaunchKernelGGL(k_gxf_pack_counts, dim3(1), dim3(MAX_RANKS), 0, st, cnt, front, world, out);
    return hipGetLastError();
}

hipError_t launch_gxf_halo_recv(const HbState& h, const GxFwd& f, uint32_t hop, const uint64_t* in, uint64_t n,
                                const uint32_t* halo_pair, const uint32_t* halo_node, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gxf_halo_recv, dim3(gx_grid(n)), dim3(256), 0, st, h, f, hop, in, n, halo_pair, halo_node);
    return hipGetLastError();
}

hipError_t launch_gx_broken(const HbState& h, uint32_t* counts, hipStream_t st) {
    if (h.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gx_broken, dim3(gx_blocks(h.n_pairs, 256, COUNTER_GRID)), dim3(256), 0, st, h, counts);
    return hipGetLastError();
}

hipError_t launch_gx_count(const HbState& h, unsigned long long* n, hipStream_t st) {
    if (h.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gx_count, dim3(gx_blocks(h.n_pairs * h.prom_slots, 256, COUNTER_GRID)), dim3(256), 0, st, h, n);
    return hipGetLastError();
}

hipError_t launch_gx_prom_grow(const uint64_t* h_in, const int64_t* e_in, uint32_t from, uint64_t* h_out,
                               int64_t* e_out, uint32_t to, uint64_t n_pairs, hipStream_t st) {
    if (n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gx_prom_grow, dim3(gx_blocks(n_pairs * to, 256, 8192)), dim3(256), 0, st, h_in, e_in, from,
                       h_out, e_out, to, n_pairs);
    return hipGetLastError();
}


}  // namespace gsx
