// gsx_propagate.hip — message propagation over the overlay (A13-A14).
//
// Bit-sliced, pull-based frontier expansion: messages travel in 64-message
// words; per node the engine keeps `seen`, `origin` and the current frontier
// as node-major word rows ([node][word]), so one gather brings every word of
// a neighbour.  One launch per hop: thread u walks its own pairs (u -> v) in
// ascending neighbour order and pulls v's frontier row through the reverse
// pair (v -> u) — its eligibility (read through u's own pair, pin) and the
// origin rows; the `from` exclusion is settled without a lookup (see
// k_prop_hop) — so the first deliverer
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

#include <cstdlib>

#ifndef GSX_FAST_U
#define GSX_FAST_U 4
#endif

namespace gsx {

// Eligibility of every pair (v -> u) for this call (topic, router, scores),
// and FWD_GIN: gossipsub's AcceptFrom at the pair's observer drops every RPC
// of the pair's neighbour (score < GraylistThreshold, not a direct peer;
// gossipsub.go:583-594 -> pubsub.go:1014-1017: the payload is never pushed,
// so no seen mark, no trace, no P2/P3/P4).  Floodsub and RandomSub accept all.
// The score is the one of the call start, like the publishThreshold tests.
__device__ __forceinline__ uint8_t fwd_byte(const PropState& ps, const DevState& s, uint64_t r) {
    const uint8_t pf = s.pflags[r];
    const uint8_t ef = ps.eflags[r];
    uint8_t out = 0;
    if ((pf & (PAIR_PRESENT | PAIR_CONNECTED)) == (PAIR_PRESENT | PAIR_CONNECTED) &&
        topic_peer(ps.psub, r, ps.topic)) {  // in ps.topics[topic]
        if (ps.router == ROUTER_FLOODSUB) {  // every topic peer (floodsub.go:81-90)
            out = FWD_FORWARD | FWD_PUBLISH;
        } else if (ps.router == ROUTER_RANDOMSUB) {  // FloodSub peers always, the rest by draw (randomsub.go:112-143)
            out = (ef & EDGE_FLOODSUB) ? (FWD_FORWARD | FWD_PUBLISH) : FWD_RSUB_CAND;
        } else {  // gossipsub
            const bool direct = ef & EDGE_DIRECT;
            // the score is read only where a threshold decides (floodsub peers, flood publish)
            const bool need_score = !direct && (!(ef & EDGE_GOSSIPSUB) || ps.flood_publish);
            const bool above = need_score && s.score[r] >= ps.publish_threshold;
            bool fwd = direct || (!(ef & EDGE_GOSSIPSUB) && above);  // direct + floodsub peers (:962-975)
            if (!fwd && ps.topic < s.n_topics)  // mesh peers, or the fanout when not joined (:977-999)
                fwd = joined_node(ps.sub, ps.pair_obs[r], ps.topic)
                          ? (s.rflags[flag_index(r, ps.topic, s.n_topics)] & REC_IN_MESH) != 0
                          : ((ps.fanout[r] >> ps.topic) & 1) != 0;
            const bool pub = ps.flood_publish ? (direct || above) : fwd;  // flood publish (:953-960)
            out = (fwd ? FWD_FORWARD : 0) | (pub ? FWD_PUBLISH : 0);
        }
    }
    // Score() of a peer without peerStats is 0 (score.go:247-256), never below the
    // (non-positive) threshold; the score vector holds 0 for those pairs.
    if (ps.gate && !(ef & EDGE_DIRECT) && s.score[r] < ps.graylist_threshold) out |= FWD_GIN;
    return out;
}

__global__ __launch_bounds__(256) void k_prop_fwd(PropState ps, DevState s) {
    unsigned long long n_gray[1] = {0};
    for (uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x; r < s.n_pairs; r += (uint64_t)gridDim.x * 256u) {
        const uint8_t out = fwd_byte(ps, s, r);
        if (out & FWD_GIN) ++n_gray[0];
        if (ps.inc) {  // the pins of the last call stand but for the pairs whose byte changed
            if (ps.fwd[r] != out) {
                const uint32_t k = atomicAdd(ps.nchg, 1u);
                if (k < ps.chg_cap) ps.chg[k] = (uint32_t)r;
                ps.fwd[r] = out;
            }
        } else {
            ps.fwd[r] = out;
        }
    }
    const uint32_t slot[1] = {0};
    block_count<1>(n_gray, ps.gray_pairs, slot);
}

// pin[q], per call, for the receiver's pair q = (u -> v): what the hop
// kernel needs to pull from v in one coalesced word — NO_PAIR if v never
// sends to u (no reverse pair, or not in v's targets), HALO | slot if v is
// remote, else (fwd & 3) << 29 | v_local (FORWARD / PUBLISH bits; RandomSub
// candidates have neither and go through `sel`).  (Gathering fwd per q here
// is cheaper than scattering pin from k_prop_fwd: 1-byte reads from a small
// array vs 4-byte partial-line writes.)
// Also keeps rfwd[q] = fwd[rev q], the reverse pair's byte (k_prop_dups reads
// it coalesced instead of gathering it).
__device__ __forceinline__ uint32_t pin_of(const PropState& ps, uint64_t q) {
    const uint32_t r = ps.rev[q];
    const bool gin = ps.fwd[q] & FWD_GIN;  // u drops whatever v sends (AcceptFrom)
    uint32_t out = NO_PAIR;
    uint8_t rf = 0;
    if (r != NO_PAIR) {
        if (r & HALO) {
            // remote v: its rank packs what it sends either way; u counts the
            // copies it drops (k_prop_hop).  (Replicated frontier: the pin comes
            // with v's fwd byte, k_rep_fwd_recv.)
            out = ps.rep ? NO_PAIR : gin ? (r | HALO_GRAY) : r;
        } else {
            const uint8_t fw = ps.fwd[r];
            rf = fw;
            if (!gin && (fw & FWD_SEND))
                out = ((uint32_t)(fw & (FWD_FORWARD | FWD_PUBLISH)) << PIN_FWD_SHIFT) | ((fw & FWD_GIN) ? PIN_RDROP : 0u) |
                      ((uint32_t)ps.col[q] - (ps.rep ? 0u : ps.node_lo));  // (replicated frontier: global ids)
        }
    }
    ps.rfwd[q] = rf;
    return out;
}

// Every pin (first call, or more changed fwd bytes than the change list
// holds), or (ps.inc) only the pins a changed byte feeds: pin[r] (its GIN
// bit) and pin[rev r] (what it lets through), marking their observers for
// k_prop_compact.  One launch over all pairs either way; in the incremental
// case every thread past the list returns at once.
// (A grid-stride loop on a capped grid: an incremental pass of a few changes
// costs a few waves, not a launch over every pair.)
__global__ __launch_bounds__(256) void k_prop_pin(PropState ps) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    const uint32_t n = ps.inc ? *ps.nchg : 0;
    if (!ps.inc || n > ps.chg_cap) {
        for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < ps.n_pairs; q += stride) ps.pin[q] = pin_of(ps, q);
        return;
    }
    for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < n; q += stride) {
        const uint32_t r = ps.chg[q];
        ps.pin[r] = pin_of(ps, r);
        const uint32_t v = ps.pair_obs[r];
        atomicOr((unsigned long long*)&ps.ndirty[v / 64], 1ull << (v % 64));
        const uint32_t q2 = ps.rev[r];
        if (q2 != NO_PAIR && !(q2 & HALO)) {
            ps.pin[q2] = pin_of(ps, q2);
            const uint32_t u = ps.pair_obs[q2];
            atomicOr((unsigned long long*)&ps.ndirty[u / 64], 1ull << (u % 64));
        }
    }
}

// Node u's compacted senders (ps.cent / ps.cend): every node after a full
// pin pass, else the nodes k_prop_pin marked (their marks cleared here).
__device__ __forceinline__ void compact_node(const PropState& ps, uint32_t u) {
    const int64_t q0 = ps.row_ptr[u], q1 = ps.row_ptr[u + 1];
    int64_t k = q0;
    for (int64_t q = q0; q < q1; ++q) {
        const uint32_t pn = ps.pin[q];
        if (pn != NO_PAIR) ps.cent[k++] = make_uint2(pn, (uint32_t)q);
    }
    ps.cend[u] = (uint32_t)k;
}
// (incremental: a thread per 64-node word of marks, the marked nodes only;
// the marks are cleared here, and the change list emptied by the last wave)
__global__ __launch_bounds__(256) void k_prop_compact(PropState ps) {
    const bool full = !ps.inc || *ps.nchg > ps.chg_cap;
    const uint32_t stride = gridDim.x * 256u;
    if (full) {
        for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < ps.n_nodes; u += stride) compact_node(ps, u);
        return;
    }
    const uint32_t nw = (ps.n_nodes + 63) / 64;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nw; i += stride) {
        uint64_t w = ps.ndirty[i];
        if (!w) continue;
        ps.ndirty[i] = 0;
        for (; w; w &= w - 1) compact_node(ps, i * 64 + (uint32_t)__builtin_ctzll(w));
    }
}
__global__ __launch_bounds__(256) void k_prop_compact_done(PropState ps) {
    const uint32_t stride = gridDim.x * 256u;
    const bool full = !ps.inc || *ps.nchg > ps.chg_cap;  // (an incremental compact cleared its marks)
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; full && i < (ps.n_nodes + 63) / 64; i += stride) ps.ndirty[i] = 0;
}
__global__ void k_prop_nchg_reset(PropState ps) { *ps.nchg = 0; }  // the next call's change list starts empty

// The origin and hop-0 rows are read only for nodes with their row-0
// occupancy bit (the call's sources), so only the sources' rows are cleared
// (k_prop_zero_src), not the whole [node][W] arrays.
__global__ __launch_bounds__(256) void k_prop_zero_src(PropState ps, uint64_t* front) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint32_t W = ps.n_words;
    if (i >= (uint64_t)ps.n_msgs * W) return;
    const uint32_t src = ps.msgs[i / W].source;
    if (src < ps.node_lo || src - ps.node_lo >= ps.n_nodes) return;
    const size_t r = (size_t)(src - ps.node_lo) * W + i % W;
    ps.origin[r] = 0;
    front[r] = 0;
}

// Sources on this shard: seen / frontier / origin bits and hop 0 (the local publish).
// The per-call clears of gsx_propagate in one launch (was a memset each):
// seen rows, first-receipt counts (and their last-hop words, the per-hop
// back-send corrections when those are used), occupancy row 0, both touch
// buffers and the counters.
__global__ __launch_bounds__(256) void k_prop_clear(PropState ps, uint32_t clear_flast, uint32_t clear_corr) {
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    const size_t nseen = (size_t)ps.n_words * ps.n_nodes;
    size_t n = nseen > ps.n_pairs ? nseen : ps.n_pairs;
    if (n < STAT_WORDS) n = STAT_WORDS;  // (tiny overlays: the stat words are the longest array)
    const size_t stride = (size_t)gridDim.x * 256u;
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < n; i += stride) {
        if (i < nseen) ps.seen[i] = 0;
        if (i < ps.n_pairs) {
            ps.fcnt[i] = 0;
            if (clear_flast) ps.flast[i] = 0;
            if (clear_corr) ps.corr[i] = 0;
        }
        if (i < occ_row) {
            ps.occ[i] = 0;
            ps.touch[i] = 0;
            ps.touch[occ_row + i] = 0;
        }
        if (i < STAT_WORDS) ps.stats[i] = 0;
    }
}

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
    atomicOr((unsigned long long*)&ps.occ[u / 64], 1ull << (u % 64));  // occupancy row 0
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

// Frontier-history row h of node v is valid only where occupancy row h has
// v's bit (a hop writes the rows of the nodes it touched; every other row
// is empty whatever the memory holds).
__device__ __forceinline__ bool occ_bit(const uint64_t* __restrict__ occ, uint32_t v) {
    return (occ[v / 64] >> (v % 64)) & 1;
}

// ---- RandomSub's draw: the canonical RNG with tag 7 (gsx_ops.h) ----------
constexpr uint64_t TAG_RANDOMSUB = 7;

// For every frontier vertex v and message m of this hop (randomsub.go:112-143):
// candidates = its non-FloodSub topic peers except `from` and the origin, in
// ascending order; above RandomSubD they are shuffled (shufflePeers,
// gossipsub.go:1890-1895) and the first max(6, ceil(sqrt(size))) kept.  The
// kept pairs get message m's bit in `sel`.
__global__ __launch_bounds__(64) void k_rsub_select(PropState ps, const uint64_t* __restrict__ front,
                                                   const uint64_t* __restrict__ front_occ) {
    const uint32_t v = blockIdx.x * 64u + threadIdx.x;
    if (v >= ps.n_nodes || !occ_bit(front_occ, v)) return;
    const int64_t r0 = ps.row_ptr[v], r1 = ps.row_ptr[v + 1];
    const uint32_t W = ps.n_words;
    uint32_t* const cand = ps.rcand + r0;  // the node's own pair range: no degree limit
    for (uint32_t w = 0; w < W; ++w) {
        uint64_t f = front[(size_t)v * W + w];
        while (f) {
            const int b = __builtin_ctzll(f);
            f &= f - 1;
            const uint32_t k = w * 64 + b;
            const uint32_t origin = ps.msgs[k].source;
            int n = 0;
            for (int64_t r = r0; r < r1; ++r) {
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

// Very sparse hops (at most n/16 first receipts last hop): the frontier
// pushes "you have a sender" bits to its neighbours, so the hop kernel
// skips every other node with one bitmap load instead of walking its pairs.
// The touch bitmap was cleared before this hop (and before the halo scatter,
// which marks the receivers of remote rows).
__device__ __forceinline__ bool mark_hop(const PropState& ps, uint32_t h) {
    const unsigned long long prev = h >= 2 ? ps.stats[STAT_HOP0 + h - 1] : ps.n_msgs;
    // (replicated frontier: the remote rows of the hop mark their receivers too)
    if (ps.rep) return !ps.rep_rows && prev + (h >= 2 ? ps.rep_in : 0) < ps.n_nodes / ps.mark_div;
    return prev < ps.n_nodes / ps.mark_div && !(ps.halo && !ps.halo_tag);
}
// Range shards: can a remote sender's row reach this hop?  The compacted
// exchange counts the hop's scattered entries (STAT_HALO0); the dense one
// (every cross pair's row, untagged) always may.
__device__ __forceinline__ bool halo_rows(const PropState& ps, uint32_t h) {
    return ps.halo && (!ps.halo_tag || ps.stats[STAT_HALO0 + h] != 0);
}
// A remote sender's row of hop h, words w0 .. w0 + CW: the compacted
// exchange's tagged row (empty unless its tag is this hop's), or the dense
// exchange's row as received.
template <int CW>
__device__ __forceinline__ void halo_row(const PropState& ps, uint32_t slot, uint32_t h, uint32_t w0,
                                         uint64_t (&c)[CW]) {
    const uint32_t W = ps.n_words;
    if (ps.halo_tag) {
        const uint64_t* r = ps.halo + (size_t)slot * (W + 1);
        if (CW == 1 && W == 1) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(r);
            c[0] = x.x == (ps.halo_tag | h) ? x.y : 0ull;
            return;
        }
        const bool live = r[0] == (ps.halo_tag | h);
#pragma unroll
        for (int i = 0; i < CW; ++i) c[i] = live ? r[1 + w0 + i] : 0ull;
    } else {
#pragma unroll
        for (int i = 0; i < CW; ++i) c[i] = ps.halo[(size_t)slot * W + w0 + i];
    }
}
// ---- shard exchange: pack what each cross-shard pair (v -> u) sends ---------------
// One thread per send slot (the order the receiving rank asked for).  The
// receiver applies only its own origin mask; eligibility, RandomSub draws
// and the `from` exclusion are the sender's and are applied here.
__global__ __launch_bounds__(256) void k_prop_pack(PropState ps, const uint64_t* __restrict__ front,
                                                   const uint64_t* __restrict__ front_occ, uint64_t* __restrict__ send) {
    const uint32_t W = ps.n_words;
    unsigned long long cnt[1] = {0};
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < ps.n_send; j += (uint64_t)gridDim.x * 256u) {
        uint64_t* out = send + j * W;
        const uint32_t r = ps.send_pair[j];
        const uint32_t v = r == NO_PAIR ? 0 : ps.pair_obs[r];
        if (r == NO_PAIR || !occ_bit(front_occ, v)) {  // no pair, or v received nothing last hop
            for (uint32_t w = 0; w < W; ++w) out[w] = 0;
            continue;
        }
        const uint8_t fw = ps.fwd[r];
        // messages v first got from u at the frontier's hop (u is remote: the
        // receive slot of pair r), never sent back (floodsub.go:82)
        const uint64_t* hf = ps.hfrom + (size_t)r * W;  // (v's own pair for u: hfrom is per pair)
        for (uint32_t w = 0; w < W; ++w) {
            const uint64_t f = front[(size_t)v * W + w];
            uint64_t c = 0;
            if (f) {
                const uint64_t own = occ_bit(ps.occ, v) ? ps.origin[(size_t)v * W + w] : 0;  // rows of sources only
                uint64_t el = elig_word(fw, own);
                if (ps.sel) el |= ps.sel[(size_t)r * W + w];
                c = f & el;
                cnt[0] += c != 0;
                if (c) c &= ~hf[w];
            }
            out[w] = c;
        }
    }
    const uint32_t slot[1] = {STAT_EDGE_SENDS};
    block_count<1>(cnt, ps.stats, slot);
}

// Compacted exchange: only the non-empty rows travel, as entries
// [halo slot at the receiver][W words]; each destination rank d owns the
// entry range of its dense send segment (send_base[d] .. +send_count[d]).
// The pack walks the hop's FRONTIER, not the send slots: a node whose
// frontier row is empty (one occupancy bit; a wave of 64 nodes per word) costs
// nothing, so the sparse first and last hops of a call pack in microseconds.
// Two passes over the same nodes: k_pack_front<false> counts each block's
// entries per destination (LDS counters), k_pack_scan turns the counts into
// per-(block, destination) offsets and the destinations' totals (dcount),
// k_pack_front<true> recomputes the rows (cache-hot) and writes each entry at
// its block's offset plus a position from an LDS counter.  The order of the
// entries inside a block's range is not deterministic, but each carries its
// slot and the receiver only scatters them (k_halo_scatter), so the hop is.
constexpr uint32_t PACK_NPB = 256;  // nodes per block (few: the walk is a chain of dependent loads, latency-bound)
constexpr uint32_t PACK_G = 4;       // lanes per node
static inline uint32_t pack_blocks(uint32_t n_nodes) { return (n_nodes + PACK_NPB - 1) / PACK_NPB; }

// What pair r = (v -> u), u remote, sends at this hop, word w (0: nothing):
// v's frontier through the pair's eligibility (and RandomSub's draw), minus
// what v first got from u (floodsub.go:82; hfrom of r, v's own pair for u).
__device__ __forceinline__ uint64_t pack_word(const PropState& ps, const uint64_t* __restrict__ front, uint32_t v,
                                              bool v_src, uint64_t r, uint8_t fw, const uint64_t* __restrict__ hf,
                                              uint32_t w, uint64_t* elig_send) {
    const uint32_t W = ps.n_words;
    const uint64_t f = front[(size_t)v * W + w];
    if (!f) return 0;
    uint64_t el = elig_word(fw, v_src ? ps.origin[(size_t)v * W + w] : 0);
    if (ps.sel) el |= ps.sel[(size_t)r * W + w];
    const uint64_t c = f & el;
    if (elig_send) *elig_send += c != 0;
    return c & ~hf[w];
}

template <bool WRITE>
__global__ __launch_bounds__(256) void k_pack_front(PropState ps, const uint64_t* __restrict__ front,
                                                    const uint64_t* __restrict__ front_occ, uint32_t* __restrict__ tab,
                                                    uint64_t* __restrict__ out) {
    __shared__ uint32_t cnt[MAX_RANKS];
    __shared__ uint64_t base[MAX_RANKS];  // WRITE: this block's first entry per destination
    const uint32_t W = ps.n_words, R = ps.n_ranks;
    const uint32_t b = blockIdx.x;
    if (threadIdx.x < R) {
        cnt[threadIdx.x] = 0;
        if (WRITE) base[threadIdx.x] = ps.send_base[threadIdx.x] + tab[(size_t)b * R + threadIdx.x];
    }
    __syncthreads();
    uint64_t nsend = 0;
    const uint32_t u0 = b * PACK_NPB;
    // PACK_G lanes per node split its pairs (lane c: pairs c, c + PACK_G, ...), so a
    // node's per-pair reads (rev, send_slot, fwd, hfrom) are adjacent across its lanes
    const uint32_t gi = threadIdx.x / PACK_G, lc = threadIdx.x % PACK_G;
    for (uint32_t v = u0 + gi; v < u0 + PACK_NPB && v < ps.n_nodes; v += 256 / PACK_G) {
        if (!occ_bit(front_occ, v)) continue;  // v received nothing last hop (the whole wave, usually)
        const bool v_src = occ_bit(ps.occ, v);
        for (int64_t r = ps.row_ptr[v] + lc; r < ps.row_ptr[v + 1]; r += PACK_G) {
            const uint32_t rv = ps.rev[r];
            if (rv == NO_PAIR || !(rv & HALO)) continue;  // a local receiver pulls v's row itself
            const uint32_t j = ps.send_slot[r];
            if (j == NO_PAIR) continue;  // nobody asked for the pair (no reverse pair at u)
            const uint8_t fw = ps.fwd[r];
            if (!(fw & FWD_SEND)) continue;
            const uint64_t* hf = ps.hfrom + (size_t)r * W;
            bool nz = false;
            for (uint32_t w = 0; w < W; ++w) nz |= pack_word(ps, front, v, v_src, r, fw, hf, w, WRITE ? nullptr : &nsend) != 0;
            if (!nz) continue;
            const uint32_t d = ps.send_dest[j];
            const uint32_t pos = atomicAdd(&cnt[d], 1u);
            if (WRITE) {
                uint64_t* e = out + (base[d] + pos) * (uint64_t)(W + 1);
                e[0] = ps.dest_halo_base[d] + (j - ps.send_base[d]);
                for (uint32_t w = 0; w < W; ++w) e[1 + w] = pack_word(ps, front, v, v_src, r, fw, hf, w, nullptr);
            }
        }
    }
    if (!WRITE) {
        __syncthreads();
        if (threadIdx.x < R) tab[(size_t)b * R + threadIdx.x] = cnt[threadIdx.x];
        unsigned long long c1[1] = {nsend};
        const uint32_t slot[1] = {STAT_EDGE_SENDS};
        block_count<1>(c1, ps.stats, slot);
    }
}
// Per destination (one block each): exclusive scan of the blocks' counts in
// place, the destination's total into dcount[d].
__global__ __launch_bounds__(1024) void k_pack_scan(uint32_t* __restrict__ tab, uint32_t n_blocks, uint32_t R,
                                                    unsigned long long* __restrict__ dcount) {
    __shared__ uint32_t part[1024];
    const uint32_t d = blockIdx.x;
    uint64_t carry = 0;
    for (uint32_t b0 = 0; b0 < n_blocks; b0 += 1024) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t x = b < n_blocks ? tab[(size_t)b * R + d] : 0u;
        part[threadIdx.x] = x;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
            const uint32_t y = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
            __syncthreads();
            part[threadIdx.x] += y;
            __syncthreads();
        }
        if (b < n_blocks) tab[(size_t)b * R + d] = (uint32_t)(carry + part[threadIdx.x] - x);
        carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) dcount[d] = carry;
}

// Receiver (compacted exchange): each entry's row goes to its receive slot
// as [hop tag | W words] (PropState::halo_tag); a row whose tag is not the
// hop's is empty, so nothing is cleared between hops or calls.  On a hop the
// receivers will mark (mark_hop), the entries also mark their receivers.
__global__ __launch_bounds__(256) void k_halo_scatter(PropState ps, uint64_t* __restrict__ halo,
                                                      const uint64_t* __restrict__ ent, uint64_t n, uint32_t h) {
    const uint32_t W = ps.n_words;
    const uint64_t tag = ps.halo_tag | h;
    const bool mark = mark_hop(ps, h);
    uint64_t* touch = ps.touch + (size_t)(h & 1) * (((size_t)ps.n_nodes + 63) / 64);  // the coming hop h's buffer
    if (blockIdx.x == 0 && threadIdx.x == 0) ps.stats[STAT_HALO0 + h] = n;  // (launched only for n > 0)
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const uint64_t* e = ent + i * (uint64_t)(W + 1);
        const uint32_t slot = (uint32_t)e[0];
        uint64_t* r = halo + (size_t)slot * (W + 1);
        if (W == 1) {
            *reinterpret_cast<ulonglong2*>(r) = make_ulonglong2(tag, e[1]);  // (16-B aligned rows)
        } else {
            r[0] = tag;
            for (uint32_t w = 0; w < W; ++w) r[1 + w] = e[1 + w];
        }
        if (mark) {
            const uint32_t u = ps.halo_node[slot];
            atomicOr((unsigned long long*)&touch[u / 64], 1ull << (u % 64));  // u has a sender this hop
        }
    }
}

__global__ __launch_bounds__(256) void k_prop_mark(PropState ps, uint32_t h, const uint64_t* __restrict__ front_occ) {
    // housekeeping of this hop: its occupancy row (the hop ORs bits in) and
    // the other touch buffer (the next hop's, marked by its halo scatter and
    // its own k_prop_mark) start empty
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    uint64_t* occ_h = ps.occ + (size_t)h * occ_row;
    uint64_t* touch_next = ps.touch + (size_t)((h + 1) & 1) * occ_row;
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < occ_row; i += (size_t)gridDim.x * 256u) {
        occ_h[i] = 0;
        touch_next[i] = 0;
    }
    if (ps.rep) {  // the replicated rows of hop h: this hop writes this rank's part, k_rep_scatter the rest
        const size_t og_row = ((size_t)ps.n_total + 63) / 64 + 1;
        uint64_t* og = ps.occ_g + (size_t)(h & 1) * og_row;
        for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < og_row; i += (size_t)gridDim.x * 256u) og[i] = 0;
    }
    const unsigned long long prev = h >= 2 ? ps.stats[STAT_HOP0 + h - 1] : ps.n_msgs;
    if (ps.hop_flag && blockIdx.x == 0 && threadIdx.x == 0)  // hop h - 1 is complete: tell the launching host
        __hip_atomic_store(ps.hop_flag + (h - 1), (ps.hop_seq << 1) | (prev != 0 ? 1u : 0u), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    if (!mark_hop(ps, h) || (!ps.sharded && h > 1 && prev == 0)) return;
    uint64_t* touch = ps.touch + (size_t)(h & 1) * occ_row;
    for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < ps.n_nodes; v += gridDim.x * 256u) {
        if (!((front_occ[v / 64] >> (v % 64)) & 1)) continue;
        for (int64_t r = ps.row_ptr[v]; r < ps.row_ptr[v + 1]; ++r) {
            const uint32_t q = ps.rev[r];
            if (q == NO_PAIR || (q & HALO) || !(ps.fwd[r] & FWD_SEND)) continue;  // v sends nothing to a local u
            const uint32_t u = (uint32_t)ps.col[r] - ps.node_lo;
            atomicOr((unsigned long long*)&touch[u / 64], 1ull << (u % 64));
        }
    }
}

// ---- one hop ----------------------------------------------------------------
// `front` holds the messages each vertex first received at hop h-1; `nxt`
// receives those first received now.  A node is handled by a group of LPN
// lanes (1, 2 or 4): lane c of the group owns the CW-word chunks c, c + LPN,
// ... of every row, so the group reads a neighbour's row as LPN adjacent
// chunks of one line (LPN = 4 at 1024 messages: the whole 128-B line of a
// gathered row is used, where a one-lane walk over 32-B chunks used a
// quarter of every line it pulled).  Everything per pair (pins, occupancy
// tests, eligibility) is the same in every lane of a group, so the group
// walks the pairs in lock step and sums its per-pair counts with shuffles.
template <int CW>
__device__ __forceinline__ void load_words(uint64_t (&d)[CW], const uint64_t* p) {
#pragma unroll
    for (int i = 0; i < CW; ++i) d[i] = p[i];
}

// Sum over the LPN lanes of a group (aligned), every lane gets the sum.
// Groups of 2 and 4 use DPP quad permutes (a VALU operand modifier, no LDS
// crossbar); wider groups fall back to ds_bpermute shuffles.
// flast of pair q after `fresh` more first receipts at hop h: hop << 32 |
// count.  When a lane walks the pairs once per chunk of its row (rows longer
// than LPN * CW words), the chunks of one hop add up.
__device__ __forceinline__ uint64_t last_count(const PropState& ps, uint64_t q, uint32_t h, uint32_t fresh,
                                               bool chunks) {
    uint32_t base = 0;
    if (chunks) {
        const uint64_t fl = ps.flast[q];
        if ((uint32_t)(fl >> 32) == h) base = (uint32_t)fl;
    }
    return ((uint64_t)h << 32) | (base + fresh);
}

template <int LPN>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
    if (LPN == 2 || LPN == 4) {
        x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
        if (LPN == 4) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
        return x;
    }
#pragma unroll
    for (int o = 1; o < LPN; o <<= 1) x += __shfl_xor(x, o, LPN);
    return x;
}

// Bits of up to 64 consecutive nodes starting at global node g0 into a
// global occupancy row (g0 need not be 64-aligned: a shard's range starts
// anywhere; the row has one spare word).
__device__ __forceinline__ void occ_g_or(uint64_t* og, uint32_t g0, uint64_t bits) {
    const uint32_t sh = g0 % 64;
    atomicOr((unsigned long long*)&og[g0 / 64], (unsigned long long)(bits << sh));
    if (sh && (bits >> (64 - sh))) atomicOr((unsigned long long*)&og[g0 / 64 + 1], (unsigned long long)(bits >> (64 - sh)));
}

// The common case as its own lean kernel (k_prop_hop_fast): no RandomSub
// draws, no first-deliverer rows, and late duplicate accounting (every
// duplicate inside the P3 window, or no credits), so the hop only moves
// first receipts: per pair and word, eligibility, "not seen, not from a lower
// sender", and a popcount.  Same results as k_prop_hop.
// SH (range shards): a compacted sender may be remote (pin HALO | slot): its
// row comes from the halo, already filtered by the sender's rank (eligibility
// and the `from` exclusion, k_prop_pack[_compact]); u masks its own messages
// off it, its copies are counted as duplicates here (k_prop_dups sees only
// local senders), a graylisted one's copies as STAT_GRAY, and its first
// receipts go to hfrom for u's own pack.  A hop with no local frontier still
// runs while remote rows arrived (halo_rows).
template <int CW, int LPN, bool DROP, int SH>
__global__ __launch_bounds__(256) void k_prop_hop_fast(PropState ps, uint32_t h, const uint64_t* __restrict__ front,
                                                       uint64_t* __restrict__ nxt) {
    constexpr int U = GSX_FAST_U;
    constexpr uint32_t NB = 256 / LPN;
    constexpr uint32_t NW = 64 / LPN;
    const uint32_t W = ps.n_words;
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    const uint64_t* __restrict__ occ_src = ps.occ;
    const uint64_t* __restrict__ occ_front = ps.occ + (size_t)(h - 1) * occ_row;
    uint64_t* __restrict__ occ_nxt = ps.occ + (size_t)h * occ_row;
    const unsigned long long prev = h >= 2 ? ps.stats[STAT_HOP0 + h - 1] : ps.n_msgs;
    if (h > 1 && prev == 0 && !(SH == 1 && halo_rows(ps, h)) && !(SH == 2 && ps.rep_in)) return;
    // (hop 1 always: the rows of hop 0 are written for the sources only; the
    // replicated rows always: a remote row is valid only under its bit)
    const bool use_occ = SH == 2 || h == 1 || prev < ps.n_nodes / ps.occ_div;
    const bool use_mark = mark_hop(ps, h);
    // rows of hop h - 1 can be stale only if that hop left nodes untouched
    const bool check_rows = !use_occ && h >= 2 && mark_hop(ps, h - 1);
    const uint64_t* __restrict__ touch_h = ps.touch + (size_t)(h & 1) * occ_row;
    // SH == 2: the replicated rows of hop h - 1 (read) and h (this rank's part written)
    const size_t occ_g_row = ((size_t)ps.n_total + 63) / 64 + 1;
    const uint64_t* __restrict__ rg_front = SH == 2 ? ps.front_g + (size_t)((h - 1) & 1) * ps.n_total * W : nullptr;
    const uint64_t* __restrict__ og_front = SH == 2 ? ps.occ_g + (size_t)((h - 1) & 1) * occ_g_row : nullptr;
    uint64_t* __restrict__ rg_nxt = SH == 2 ? ps.front_g + (size_t)(h & 1) * ps.n_total * W : nullptr;
    uint64_t* __restrict__ og_nxt = SH == 2 ? ps.occ_g + (size_t)(h & 1) * occ_g_row : nullptr;
    const uint32_t gi = threadIdx.x / LPN, lc = threadIdx.x % LPN;
    unsigned long long n_new = 0, n_send = 0, n_vnew = 0, n_rej = 0, n_ign = 0, n_dup = 0, n_gray = 0;
    for (uint32_t tile = blockIdx.x * NB; tile < ps.n_nodes; tile += gridDim.x * NB) {
        const uint32_t u = tile + gi;
        bool any_new = false;
        bool touch = u < ps.n_nodes;
        if (touch && use_mark) touch = occ_bit(touch_h, u);
        if (touch) {
            // only the pairs whose neighbour sends to u at all (compacted, k_prop_compact)
            const int64_t q0 = ps.row_ptr[u], q1 = ps.cend[u];
            const size_t un = (size_t)u * W;
            // (u's own messages need no mask for local senders: they are in `seen`
            // since hop 0, and those duplicates are counted at the end of the call)
            const bool u_src = SH == 1 && occ_bit(occ_src, u);
            for (uint32_t w0 = lc * CW; w0 < W; w0 += LPN * CW) {
                uint64_t seen[CW], sa[CW], drp[CW], rej[CW], mine[CW];
                load_words<CW>(seen, ps.seen + un + w0);
                if (DROP) {  // messages validation does not accept: seen, not delivered, not forwarded
                    load_words<CW>(drp, ps.drop + w0);
                    load_words<CW>(rej, ps.reject + w0);
                }
#pragma unroll
                for (int i = 0; i < CW; ++i) {
                    sa[i] = seen[i];
                    mine[i] = 0;
                }
                if (SH == 1 && u_src) load_words<CW>(mine, ps.origin + un + w0);
                uint2 pn[U];
#pragma unroll
                for (int j = 0; j < U; ++j) pn[j] = q0 + j < q1 ? ps.cent[q0 + j] : make_uint2(NO_PAIR, 0u);
                for (int64_t qb = q0; qb < q1; qb += U) {
                    uint32_t pv[U], qv[U];
                    uint64_t c[U][CW];
#pragma unroll
                    for (int j = 0; j < U; ++j) {
                        pv[j] = pn[j].x;
                        qv[j] = pn[j].y;
                        // (a remote row's own tag says whether it arrived this hop: halo_row)
                        if (use_occ && pv[j] != NO_PAIR && !(SH == 1 && (pv[j] & HALO)) &&
                            !occ_bit(SH == 2 ? og_front : occ_front, pv[j] & PIN_NODE_MASK))
                            pv[j] = NO_PAIR;
                    }
#pragma unroll
                    for (int j = 0; j < U; ++j) {
                        if (pv[j] == NO_PAIR) {
#pragma unroll
                            for (int i = 0; i < CW; ++i) c[j][i] = 0;
                        } else if (SH == 1 && (pv[j] & HALO)) {
                            halo_row<CW>(ps, pv[j] & HALO_SLOT, h, w0, c[j]);
                        } else {
                            load_words<CW>(c[j], (SH == 2 ? rg_front : front) + (size_t)(pv[j] & PIN_NODE_MASK) * W + w0);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < U; ++j) pn[j] = qb + U + j < q1 ? ps.cent[qb + U + j] : make_uint2(NO_PAIR, 0u);
                    if (check_rows)
#pragma unroll
                        for (int j = 0; j < U; ++j)
                            if (pv[j] != NO_PAIR && !(SH == 1 && (pv[j] & HALO)) && !occ_bit(occ_front, pv[j] & PIN_NODE_MASK))
#pragma unroll
                                for (int i = 0; i < CW; ++i) c[j][i] = 0;
#pragma unroll
                    for (int j = 0; j < U; ++j) {
                        if (__ballot(pv[j] != NO_PAIR) == 0) continue;  // no lane of the wave has pair j
                        // (the same in every lane of a group: the group walks pair j together)
                        const bool hl = SH == 1 && pv[j] != NO_PAIR && (pv[j] & HALO);
                        // branch-free over the lanes: an absent pair carries an empty row
                        uint32_t m = (pv[j] == NO_PAIR || hl) ? 0u : pv[j] >> PIN_FWD_SHIFT;  // FORWARD | PUBLISH
                        if (SH == 2) {
                            // a sender's row of hop h - 1 holds only what it published (h = 1) or
                            // only what it received (h >= 2), so the pair lets it through whole
                            // or not at all: PUBLISH at hop 1, FORWARD after (elig_word on that row)
                            const bool pass = (m & (h == 1 ? FWD_PUBLISH : FWD_FORWARD)) != 0;
#pragma unroll
                            for (int i = 0; i < CW; ++i) c[j][i] = pass ? c[j][i] : 0ull;
                            m = 0;  // (no origin row to read)
                        }
                        // eligibility: FORWARD lets through what v received, PUBLISH what v
                        // published.  An absent pair's row is empty and a FORWARD|PUBLISH pair
                        // passes everything, so only a wave holding a one-sided pair masks.
                        if (__ballot(m == FWD_FORWARD || m == FWD_PUBLISH)) {
                            uint64_t own[CW];
#pragma unroll
                            for (int i = 0; i < CW; ++i) own[i] = 0;
                            const uint32_t v = pv[j] & PIN_NODE_MASK;
                            if ((m == FWD_FORWARD || m == FWD_PUBLISH) && occ_bit(occ_src, v))
                                load_words<CW>(own, ps.origin + (size_t)v * W + w0);
                            // (a remote sender's row is filtered already: it passes whole)
                            const uint64_t fmask = (hl || (m & FWD_FORWARD)) ? ~0ull : 0ull;
                            const uint64_t pmask = (hl || (m & FWD_PUBLISH)) ? ~0ull : 0ull;
#pragma unroll
                            for (int i = 0; i < CW; ++i) c[j][i] &= (fmask & ~own[i]) | (pmask & own[i]);
                        }
                        if (SH == 1 && hl) {  // never sent back to the origin; AcceptFrom drops a graylisted sender's
#pragma unroll
                            for (int i = 0; i < CW; ++i) c[j][i] &= ~mine[i];
                            if (pv[j] & HALO_GRAY) {
#pragma unroll
                                for (int i = 0; i < CW; ++i) {
                                    n_gray += __popcll(c[j][i]);
                                    c[j][i] = 0;
                                }
                            }
                        }
                        uint32_t fresh = 0, inv = 0, pc = 0;
                        uint64_t nbs[CW];
#pragma unroll
                        for (int i = 0; i < CW; ++i) {
                            const uint64_t cc = c[j][i];
                            if (!hl) n_send += cc != 0;  // (a remote sender's are counted at its pack)
                            const uint64_t nb = cc & ~sa[i];  // not seen, not from a lower sender
                            nbs[i] = nb;
                            sa[i] |= nb;
                            if (DROP) {
                                const uint64_t dv = nb & drp[i];
                                n_rej += __popcll(dv & rej[i]);
                                n_ign += __popcll(dv & ~rej[i]);
                                inv += __popcll(dv & rej[i]);
                                fresh += __popcll(nb & ~drp[i]);
                                if (SH == 1) pc += __popcll(cc & ~drp[i]);
                            } else {
                                fresh += __popcll(nb);
                                if (SH == 1) pc += __popcll(cc);
                            }
                        }
                        n_new += fresh;
                        uint32_t dup = 0;
                        if (SH == 1) {
                            dup = hl ? pc - fresh : 0u;  // a remote sender's duplicates, this hop
                            n_dup += dup;
                            if (hl) {  // what u must not send back to it (k_prop_pack)
                                bool rx = false;
#pragma unroll
                                for (int i = 0; i < CW; ++i) rx |= nbs[i] != 0;
                                if (rx) {
                                    uint64_t* hf = ps.hfrom + (size_t)qv[j] * W + w0;
#pragma unroll
                                    for (int i = 0; i < CW; ++i) hf[i] = nbs[i];
                                }
                            }
                        }
                        if (LPN > 1) fresh = group_sum<LPN>(fresh);
                        if (DROP && LPN > 1) inv = group_sum<LPN>(inv);
                        if (SH == 1 && LPN > 1) dup = group_sum<LPN>(dup);
                        if (lc == 0 && fresh) {
                            // first receipts from the pair: an add at L2, nothing read back
                            // (every pair has one writer per hop, but no load round trip)
                            const uint32_t q = qv[j];
                            atomicAdd(&ps.fcnt[q], fresh);
                            // the last hop's receipts matter only if that hop is the
                            // max_hops cut (a run that ends with an empty hop forwarded
                            // everything, k_prop_dups); flast is zeroed per call
                            if (h == ps.max_hops || ps.flast_every)
                                ps.flast[q] = last_count(ps, q, h, fresh, W > LPN * CW);
                        }
                        if (SH == 1 && lc == 0 && dup && ps.credit) ps.dupcnt[qv[j]] += dup;  // (one writer per pair)
                        if (DROP && lc == 0 && inv && ps.credit) ps.invcnt[qv[j]] += inv;  // P4
                    }
                }
#pragma unroll
                for (int i = 0; i < CW; ++i) {
                    const uint64_t acc = sa[i] ^ seen[i];
                    const uint64_t fwd_row = DROP ? acc & ~drp[i] : acc;
                    nxt[un + w0 + i] = fwd_row;
                    if (SH == 2) rg_nxt[(size_t)(ps.node_lo + u) * W + w0 + i] = fwd_row;  // (this rank's part)
                    if (acc) {
                        ps.seen[un + w0 + i] = sa[i];
                        ++n_vnew;
                    }
                    if (fwd_row) any_new = true;
                }
            }
        }
        if (LPN > 1) any_new = group_sum<LPN>(any_new ? 1u : 0u) != 0;
        uint64_t wb = __ballot(any_new && lc == 0);
        if (LPN > 1) {
            uint64_t r = 0;
#pragma unroll
            for (uint32_t i = 0; i < NW; ++i) r |= ((wb >> (i * LPN)) & 1ull) << i;
            wb = r;
        }
        const uint32_t u0 = tile + (threadIdx.x / 64) * NW;
        if ((threadIdx.x & 63) == 0 && wb) {
            atomicOr((unsigned long long*)&occ_nxt[u0 / 64], (unsigned long long)(wb << (u0 % 64)));
            if (SH == 2) occ_g_or(og_nxt, ps.node_lo + u0, wb);
        }
    }
    if (SH == 1) {
        unsigned long long cnt[7] = {n_new, n_send, n_vnew, n_rej, n_ign, n_dup, n_gray};
        const uint32_t slot[7] = {STAT_HOP0 + h, STAT_EDGE_SENDS, STAT_NEW_WORDS, STAT_REJECTED, STAT_IGNORED,
                                  STAT_DUPS, STAT_GRAY};
        block_count<7>(cnt, ps.stats, slot);
    } else {
        unsigned long long cnt[5] = {n_new, n_send, n_vnew, n_rej, n_ign};
        const uint32_t slot[5] = {STAT_HOP0 + h, STAT_EDGE_SENDS, STAT_NEW_WORDS, STAT_REJECTED, STAT_IGNORED};
        block_count<5>(cnt, ps.stats, slot);
    }
}

// k_prop_hop_fast for one-word rows (64-message calls): a group of 4 lanes
// per node splits the node's compacted SENDERS (lane c takes senders c, c +
// 4, ...) instead of row words, two rounds of 4 in flight.  The group reads
// 4 consecutive sender entries at once and runs to the longest of 16 nodes
// per wave instead of 64; "not from a lower sender" becomes an exclusive
// prefix-OR over the quad.  Same results as k_prop_hop_fast<1, 1, DROP, SH>
// (SH: remote senders through the halo, as there).
template <bool DROP, int G, int R, int SH>  // lanes per node, rounds of G senders in flight
__global__ __launch_bounds__(256) void k_prop_hop_fast1(PropState ps, uint32_t h, const uint64_t* __restrict__ front,
                                                        uint64_t* __restrict__ nxt) {
    constexpr uint32_t NB = 256 / G, NW = 64 / G;
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    const uint64_t* __restrict__ occ_src = ps.occ;
    const uint64_t* __restrict__ occ_front = ps.occ + (size_t)(h - 1) * occ_row;
    uint64_t* __restrict__ occ_nxt = ps.occ + (size_t)h * occ_row;
    const unsigned long long prev = h >= 2 ? ps.stats[STAT_HOP0 + h - 1] : ps.n_msgs;
    if (h > 1 && prev == 0 && !(SH == 1 && halo_rows(ps, h)) && !(SH == 2 && ps.rep_in)) return;
    const bool use_occ = SH == 2 || h == 1 || prev < ps.n_nodes / ps.occ_div;
    const bool use_mark = mark_hop(ps, h);
    const bool check_rows = !use_occ && h >= 2 && mark_hop(ps, h - 1);
    const uint64_t* __restrict__ touch_h = ps.touch + (size_t)(h & 1) * occ_row;
    const size_t occ_g_row = ((size_t)ps.n_total + 63) / 64 + 1;
    const uint64_t* __restrict__ rg_front = SH == 2 ? ps.front_g + (size_t)((h - 1) & 1) * ps.n_total : nullptr;
    const uint64_t* __restrict__ og_front = SH == 2 ? ps.occ_g + (size_t)((h - 1) & 1) * occ_g_row : nullptr;
    uint64_t* __restrict__ rg_nxt = SH == 2 ? ps.front_g + (size_t)(h & 1) * ps.n_total : nullptr;
    uint64_t* __restrict__ og_nxt = SH == 2 ? ps.occ_g + (size_t)(h & 1) * occ_g_row : nullptr;
    const uint32_t gi = threadIdx.x / G, lc = threadIdx.x % G;
    const uint64_t drp = DROP ? ps.drop[0] : 0ull, rej = DROP ? ps.reject[0] : 0ull;
    unsigned long long n_new = 0, n_send = 0, n_vnew = 0, n_rej = 0, n_ign = 0, n_dup = 0, n_gray = 0;
    for (uint32_t tile = blockIdx.x * NB; tile < ps.n_nodes; tile += gridDim.x * NB) {
        const uint32_t u = tile + gi;
        bool any_new = false;
        bool touch = u < ps.n_nodes;
        if (touch && use_mark) touch = occ_bit(touch_h, u);
        if (touch) {
            int64_t q0 = ps.row_ptr[u], q1 = ps.cend[u];
            const uint64_t seen = ps.seen[u];
            // a receiver that has seen every message of the call gets nothing new: its walk is
            // skipped (its senders' STAT_EDGE_SENDS are counted at the call's end: edge_late)
            if (SH != 1 && ps.edge_late && seen == ps.full1) q1 = q0;
            const uint64_t mine = (SH == 1 && occ_bit(occ_src, u)) ? ps.origin[u] : 0ull;  // (remote rows only)
            uint64_t sa = seen;
            uint2 pn[R];
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int64_t j = q0 + k * G + lc;
                pn[k] = j < q1 ? ps.cent[j] : make_uint2(NO_PAIR, 0u);
            }
            for (int64_t qb = q0; qb < q1; qb += R * G) {
                uint32_t pv[R], qv[R];
                uint64_t c[R];
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    pv[k] = pn[k].x;
                    qv[k] = pn[k].y;
                    if (use_occ && pv[k] != NO_PAIR && !(SH == 1 && (pv[k] & HALO)) &&
                        !occ_bit(SH == 2 ? og_front : occ_front, pv[k] & PIN_NODE_MASK))
                        pv[k] = NO_PAIR;  // (a remote row's tag says whether it arrived: halo_row)
                }
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    uint64_t x[1] = {0ull};
                    if (pv[k] == NO_PAIR) {
                    } else if (SH == 1 && (pv[k] & HALO)) {
                        halo_row<1>(ps, pv[k] & HALO_SLOT, h, 0, x);
                    } else {
                        x[0] = (SH == 2 ? rg_front : front)[pv[k] & PIN_NODE_MASK];
                    }
                    c[k] = x[0];
                }
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const int64_t j = qb + R * G + k * G + lc;
                    pn[k] = j < q1 ? ps.cent[j] : make_uint2(NO_PAIR, 0u);
                }
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const bool hl = SH == 1 && pv[k] != NO_PAIR && (pv[k] & HALO);
                    if (check_rows && pv[k] != NO_PAIR && !hl && !occ_bit(occ_front, pv[k] & PIN_NODE_MASK)) c[k] = 0;
                    const uint32_t m = (pv[k] == NO_PAIR || hl) ? 0u : pv[k] >> PIN_FWD_SHIFT;  // FORWARD | PUBLISH
                    if (SH == 2) {  // (rows of hop h - 1: published at h = 1, received after; k_prop_hop_fast)
                        if (!(m & (h == 1 ? FWD_PUBLISH : FWD_FORWARD))) c[k] = 0;
                    } else if (m == FWD_FORWARD || m == FWD_PUBLISH) {  // one-sided eligibility
                        const uint32_t v = pv[k] & PIN_NODE_MASK;
                        const uint64_t own = occ_bit(occ_src, v) ? ps.origin[v] : 0ull;
                        c[k] &= m == FWD_FORWARD ? ~own : own;
                    }
                    if (SH == 1 && hl) {  // never sent back to the origin; AcceptFrom drops a graylisted sender's
                        c[k] &= ~mine;
                        if (pv[k] & HALO_GRAY) {
                            n_gray += __popcll(c[k]);
                            c[k] = 0;
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < R; ++k) {  // round k: the quad's senders in order
                    const uint64_t x = c[k];
                    const bool hl = SH == 1 && pv[k] != NO_PAIR && (pv[k] & HALO);
                    if (!hl && !(SH != 1 && ps.edge_late)) n_send += x != 0;  // (a remote sender's are counted at its pack)
                    uint64_t incl = x;
#pragma unroll
                    for (uint32_t off = 1; off < (uint32_t)G; off <<= 1) {
                        const uint64_t y = __shfl_up(incl, off, G);
                        if (lc >= off) incl |= y;
                    }
                    uint64_t excl = __shfl_up(incl, 1, G);
                    if (lc == 0) excl = 0;
                    const uint64_t nb = x & ~sa & ~excl;  // not seen, not from a lower sender
                    sa |= __shfl(incl, G - 1, G);
                    uint32_t fresh, inv = 0;
                    if (DROP) {
                        const uint64_t dv = nb & drp;
                        n_rej += __popcll(dv & rej);
                        n_ign += __popcll(dv & ~rej);
                        inv = __popcll(dv & rej);
                        fresh = __popcll(nb & ~drp);
                    } else {
                        fresh = __popcll(nb);
                    }
                    n_new += fresh;
                    if (fresh) {
                        atomicAdd(&ps.fcnt[qv[k]], fresh);
                        if (h == ps.max_hops || ps.flast_every) ps.flast[qv[k]] = last_count(ps, qv[k], h, fresh, false);
                    }
                    if (DROP && inv && ps.credit) ps.invcnt[qv[k]] += inv;  // P4
                    if (SH == 1 && hl) {  // a remote sender: its duplicates this hop, and u's `from` row for it
                        const uint32_t dup = __popcll(DROP ? x & ~drp : x) - fresh;
                        n_dup += dup;
                        if (dup && ps.credit) ps.dupcnt[qv[k]] += dup;
                        if (nb) ps.hfrom[qv[k]] = nb;
                    }
                }
            }
            const uint64_t acc = sa ^ seen;
            const uint64_t fwd_row = DROP ? acc & ~drp : acc;
            if (lc == 0) {
                nxt[u] = fwd_row;
                if (SH == 2) rg_nxt[ps.node_lo + u] = fwd_row;  // (this rank's part of the replicated rows)
                if (acc) {
                    ps.seen[u] = sa;
                    ++n_vnew;
                }
            }
            any_new = fwd_row != 0;
        }
        uint64_t wb = __ballot(any_new && lc == 0);
        uint64_t r = 0;
#pragma unroll
        for (uint32_t i = 0; i < NW; ++i) r |= ((wb >> (i * G)) & 1ull) << i;
        const uint32_t u0 = tile + (threadIdx.x / 64) * NW;
        if ((threadIdx.x & 63) == 0 && r) {
            atomicOr((unsigned long long*)&occ_nxt[u0 / 64], (unsigned long long)(r << (u0 % 64)));
            if (SH == 2) occ_g_or(og_nxt, ps.node_lo + u0, r);
        }
    }
    if (SH == 1) {
        unsigned long long cnt[7] = {n_new, n_send, n_vnew, n_rej, n_ign, n_dup, n_gray};
        const uint32_t slot[7] = {STAT_HOP0 + h, STAT_EDGE_SENDS, STAT_NEW_WORDS, STAT_REJECTED, STAT_IGNORED,
                                  STAT_DUPS, STAT_GRAY};
        block_count<7>(cnt, ps.stats, slot);
    } else {
        unsigned long long cnt[5] = {n_new, n_send, n_vnew, n_rej, n_ign};
        const uint32_t slot[5] = {STAT_HOP0 + h, STAT_EDGE_SENDS, STAT_NEW_WORDS, STAT_REJECTED, STAT_IGNORED};
        block_count<5>(cnt, ps.stats, slot);
    }
}

// The `from` exclusion (floodsub.go:82, gossipsub.go:1007, randomsub.go:113)
// is never looked up here: a message v would send back to the peer u it
// first got it from is one u has already seen, so it can only ever count as
// a duplicate at u.  Duplicates are accounted in one of two ways:
//  * late (ps.late: every duplicate is inside the P3 window, or no credits):
//    not per hop at all — k_prop_dups derives each pair's duplicates at the
//    end of the call as sends - first receipts, where a pair's sends over
//    the call are v's forwarded set through its eligibility, minus `from`;
//  * per hop (a window shorter than the run): duplicates are counted as they
//    arrive, and the hop that gives v a message subtracts the back-send u will
//    make one hop later (v forwards received messages to u iff its pair
//    (v -> u) has FORWARD; v first got them at h - 1, so they are inside v's
//    window iff 2 * latency <= window) — from the duplicate counter and,
//    through corr[(v -> u)], from u's P3 count at the end of the call.
// Cross-shard sends arrive packed with the exclusion applied (k_prop_pack)
// and are counted per hop in both modes.
//
// occ (one bit per node and hop, [hop][node / 64]) marks non-empty frontier
// rows, so the sparse first and last hops skip the row gathers.
template <int CW, int LPN, bool TRACK>
__global__ __launch_bounds__(256) void k_prop_hop(PropState ps, uint32_t h, const uint64_t* __restrict__ front,
                                                  uint64_t* __restrict__ nxt) {
    constexpr int U = 4;               // pairs whose rows are in flight together (memory-level parallelism)
    constexpr uint32_t NB = 256 / LPN; // nodes per block tile
    constexpr uint32_t NW = 64 / LPN;  // nodes per wave (a power of two: its occupancy bits stay in one word)
    const uint32_t W = ps.n_words;
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    const uint64_t* __restrict__ occ_src = ps.occ;  // row 0: the nodes that published in this call
    const uint64_t* __restrict__ occ_front = ps.occ + (size_t)(h - 1) * occ_row;
    uint64_t* __restrict__ occ_nxt = ps.occ + (size_t)h * occ_row;
    const unsigned long long prev = h >= 2 ? ps.stats[STAT_HOP0 + h - 1] : ps.n_msgs;
    // nothing arrived last hop (and, on a range shard, no remote row this hop):
    // empty frontier, row h unused
    if (h > 1 && prev == 0 && !(ps.sharded && halo_rows(ps, h))) return;
    // Sparse frontier (at most a quarter of the rows can be non-empty): a row
    // is gathered only after its occupancy bit.  Very sparse (k_prop_mark):
    // a node no sender marked is left untouched (no row loads, no row
    // writes, occupancy bit 0).  Dense: rows are gathered beside their
    // occupancy bits.
    // (hop 1 always: the rows of hop 0 are written for the sources only)
    const bool use_occ = h == 1 || prev < ps.n_nodes / 4;
    const bool use_mark = mark_hop(ps, h);
    // rows of hop h - 1 can be stale only if that hop left nodes untouched
    const bool check_rows = !use_occ && h >= 2 && mark_hop(ps, h - 1);
    // Back-sends of this hop's first receipts would happen at hop h + 1 (if
    // it runs).  At h = 1 the receipts are the sender's own publishes, which
    // nobody sends back to their origin anyway.
    const bool backsend = !ps.late && h >= 2 && h < ps.max_hops;
    const bool credit_back = backsend && ps.credit && ps.back_in_window;
    // DuplicateMessage -> markDuplicateMessageDelivery with the record
    // validated at u's first receipt (score.go:806-809, 965): in the window
    // iff (h - h0) * latency <= window, i.e. u first got it at one of the
    // last win_hops hops.  A duplicate at u is a copy of a message u first
    // got earlier (seen) or this hop from a lower sender; with dm = ~seen |
    // (rows of the window hops), the in-window duplicates of a pair are
    // popcount(c & dm) - first receipts, and all its duplicates
    // popcount(c) - first receipts.
    const bool want_inwin = ps.credit && !ps.all_dups_in_window;
    const uint32_t h_lo = h > ps.win_hops ? h - ps.win_hops : 0;
    const uint32_t gi = threadIdx.x / LPN, lc = threadIdx.x % LPN;  // node of the tile, lane in the group
    unsigned long long n_new = 0, n_dup = 0, n_send = 0, n_vnew = 0, n_back = 0, n_rej = 0, n_ign = 0, n_gray = 0;
    for (uint32_t tile = blockIdx.x * NB; tile < ps.n_nodes; tile += gridDim.x * NB) {
        const uint32_t u = tile + gi;
        bool any_new = false;
        bool touch = u < ps.n_nodes;
        if (touch && use_mark) touch = occ_bit(ps.touch + (size_t)(h & 1) * occ_row, u);
        if (touch) {
            const int64_t q0 = ps.row_ptr[u], q1 = ps.row_ptr[u + 1];
            const size_t un = (size_t)u * W;
            // a node that published in this call masks its own messages off
            // every received row (never sent back to the origin); rare, so the
            // origin chunk is re-read (cache-hot) rather than held
            const bool u_src = occ_bit(occ_src, u);
            for (uint32_t w0 = lc * CW; w0 < W; w0 += LPN * CW) {
                uint64_t seen[CW], sa[CW], dm[CW], drp[CW], rej[CW];
                load_words<CW>(seen, ps.seen + un + w0);
                if (ps.drop) {  // messages validation does not accept (rare; both rows are per call)
                    load_words<CW>(drp, ps.drop + w0);
                    load_words<CW>(rej, ps.reject + w0);
                } else {
#pragma unroll
                    for (int i = 0; i < CW; ++i) drp[i] = rej[i] = 0;
                }
#pragma unroll
                for (int i = 0; i < CW; ++i) {
                    sa[i] = seen[i];  // seen | this hop's receipts so far
                    dm[i] = 0;
                }
                if (want_inwin) {
                    for (uint32_t h0 = h_lo; h0 < h; ++h0) {
                        if (!occ_bit(ps.occ + (size_t)h0 * occ_row, u)) continue;  // untouched: empty row
                        const uint64_t* row = ps.hist + (size_t)h0 * ps.n_nodes * W + un + w0;
#pragma unroll
                        for (int i = 0; i < CW; ++i) dm[i] |= row[i];
                    }
#pragma unroll
                    for (int i = 0; i < CW; ++i) dm[i] |= ~seen[i];
                }
                // software pipeline: the next block's pins are in flight
                // while this block's rows are merged
                uint32_t pn[U];
#pragma unroll
                for (int j = 0; j < U; ++j) pn[j] = q0 + j < q1 ? ps.pin[q0 + j] : NO_PAIR;
                for (int64_t qb = q0; qb < q1; qb += U) {
                    uint32_t pv[U];
                    uint64_t c[U][CW];
#pragma unroll
                    for (int j = 0; j < U; ++j) pv[j] = pn[j];
                    if (use_occ) {
#pragma unroll
                        for (int j = 0; j < U; ++j)
                            if (pv[j] != NO_PAIR) {
                                // (a remote row's tag says whether it arrived: halo_row)
                                const bool live = (pv[j] & HALO) || occ_bit(occ_front, pv[j] & PIN_NODE_MASK);
                                if (!live) pv[j] = NO_PAIR;  // the sender's row is empty
                            }
                    }
#pragma unroll
                    for (int j = 0; j < U; ++j) {
                        if (pv[j] == NO_PAIR) {
#pragma unroll
                            for (int i = 0; i < CW; ++i) c[j][i] = 0;
                        } else if (pv[j] & HALO) {  // remote sender: its rank packed exactly what it sends
                            halo_row<CW>(ps, pv[j] & HALO_SLOT, h, w0, c[j]);
                        } else {
                            load_words<CW>(c[j], front + (size_t)(pv[j] & PIN_NODE_MASK) * W + w0);
                        }
                    }
                    bool dead[U];  // rows of senders the previous hop left untouched are empty
#pragma unroll
                    for (int j = 0; j < U; ++j)
                        dead[j] = check_rows && pv[j] != NO_PAIR && !(pv[j] & HALO) &&
                                  !occ_bit(occ_front, pv[j] & PIN_NODE_MASK);
                    // the block's per-pair counters travel with its rows (group lane 0
                    // keeps them): no load-then-store chain per pair below
                    uint32_t fc[U], dc[U];
                    uint8_t fq[U];
#pragma unroll
                    for (int j = 0; j < U; ++j) {
                        const bool mine0 = pv[j] != NO_PAIR && lc == 0;
                        fc[j] = mine0 ? ps.fcnt[qb + j] : 0;
                        dc[j] = mine0 && ps.credit && (!ps.late || (pv[j] & HALO)) ? ps.dupcnt[qb + j] : 0;
                        fq[j] = mine0 && backsend ? ps.fwd[qb + j] : 0;
                    }
#pragma unroll
                    for (int j = 0; j < U; ++j) pn[j] = qb + U + j < q1 ? ps.pin[qb + U + j] : NO_PAIR;
#pragma unroll
                    for (int j = 0; j < U; ++j) {
                        const uint32_t p = pv[j];
                        if (p == NO_PAIR) continue;  // the same in every lane of the group
                        const int64_t q = qb + j;
                        const bool halo = p & HALO;
                        if (dead[j])
#pragma unroll
                            for (int i = 0; i < CW; ++i) c[j][i] = 0;
                        if (!halo) {  // v's frontier row through the pair's eligibility
                            const uint32_t v = p & PIN_NODE_MASK;
                            const uint8_t m = (uint8_t)(p >> PIN_FWD_SHIFT);
                            uint64_t own[CW], sl[CW];
                            if ((m == FWD_FORWARD || m == FWD_PUBLISH) && occ_bit(occ_src, v))
                                load_words<CW>(own, ps.origin + (size_t)v * W + w0);
                            else
#pragma unroll
                                for (int i = 0; i < CW; ++i) own[i] = 0;
                            if (ps.sel) load_words<CW>(sl, ps.sel + (size_t)ps.rev[q] * W + w0);
                            else
#pragma unroll
                                for (int i = 0; i < CW; ++i) sl[i] = 0;
#pragma unroll
                            for (int i = 0; i < CW; ++i) {
                                c[j][i] &= elig_word(m, own[i]) | sl[i];
                                n_send += c[j][i] != 0;
                            }
                        }
                        if (u_src) {
                            uint64_t mine[CW];
                            load_words<CW>(mine, ps.origin + un + w0);
#pragma unroll
                            for (int i = 0; i < CW; ++i) c[j][i] &= ~mine[i];
                        }
                        if (halo && (p & HALO_GRAY)) {  // u's AcceptFrom drops the remote sender's RPCs whole
                            // (bit 30 of a local pin is FWD_PUBLISH: tested under HALO only)
#pragma unroll
                            for (int i = 0; i < CW; ++i) n_gray += __popcll(c[j][i]);
                            continue;  // the same in every lane of the group
                        }
                        uint64_t nb[CW];
                        uint32_t fresh = 0, pc = 0, kw = 0, inv = 0;
                        bool rx = false;  // any first receipt, delivered or dropped
#pragma unroll
                        for (int i = 0; i < CW; ++i) {
                            nb[i] = c[j][i] & ~sa[i];  // first receipts: not seen, not from a lower sender
                            sa[i] |= nb[i];
                            rx |= nb[i] != 0;
                            // a message validation does not accept is seen but not delivered
                            // (RejectMessage); it only ever arrives from its source, at hop 1
                            const uint64_t dv = nb[i] & drp[i];
                            n_rej += __popcll(dv & rej[i]);
                            n_ign += __popcll(dv & ~rej[i]);
                            inv += __popcll(dv & rej[i]);
                            fresh += __popcll(nb[i] & ~drp[i]);
                            const uint64_t cv = c[j][i] & ~drp[i];
                            pc += __popcll(cv);
                            if (want_inwin) kw += __popcll(cv & dm[i]);
                        }
                        n_new += fresh;
                        uint32_t k = 0;
                        if (!ps.late || halo) {  // duplicates counted here (late: k_prop_dups)
                            n_dup += pc - fresh;
                            if (ps.credit) k = (want_inwin ? kw : pc) - fresh;
                        }
                        if (rx) {
                            if (TRACK) {  // first deliverers tracked: the pair's cumulative row
                                uint64_t* fr = ps.from_mask + (size_t)q * W + w0;
                                uint64_t o[CW];
                                load_words<CW>(o, fr);
#pragma unroll
                                for (int i = 0; i < CW; ++i) fr[i] = o[i] | nb[i];
                            }
                            if (halo) {  // what u must not send back to this remote sender (k_prop_pack)
                                uint64_t* hf = ps.hfrom + (size_t)q * W + w0;
#pragma unroll
                                for (int i = 0; i < CW; ++i) hf[i] = nb[i];
                            }
                        }
                        if (LPN > 1) {  // converged: every lane of the group is here for pair q
                            k = group_sum<LPN>(k);
                            fresh = group_sum<LPN>(fresh);
                            if (ps.drop) inv = group_sum<LPN>(inv);
                        }
                        if (lc == 0) {
                            if (inv && ps.credit) ps.invcnt[q] += inv;  // markInvalidMessageDelivery, P4
                            if (k) ps.dupcnt[q] = dc[j] + k;
                            if (fresh) {  // first receipts from v: this call's count and the last hop's
                                ps.fcnt[q] = fc[j] + fresh;
                                ps.flast[q] = last_count(ps, q, h, fresh, W > LPN * CW);
                                if (backsend && !halo && (fq[j] & FWD_FORWARD) && !(p & PIN_RDROP)) {
                                    // u forwards them to v at hop h + 1 and v counts duplicates:
                                    // the `from` exclusion's whole effect, taken back here
                                    n_back += fresh;
                                    if (credit_back) ps.corr[q] += fresh;
                                }
                            }
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < CW; ++i) {
                    const uint64_t acc = sa[i] ^ seen[i];
                    nxt[un + w0 + i] = acc & ~drp[i];  // this hop's frontier row (touched nodes only): forwarded
                    if (acc) {
                        ps.seen[un + w0 + i] = sa[i];
                        ++n_vnew;
                    }
                    if (acc & ~drp[i]) any_new = true;
                }
            }
        }
        // occupancy of this hop's rows (cleared before the hop): the group's
        // lanes OR their bits, the wave's NW nodes become NW bits of one word
        if (LPN > 1) any_new = group_sum<LPN>(any_new ? 1u : 0u) != 0;
        uint64_t wb = __ballot(any_new && lc == 0);
        if (LPN > 1) {
            uint64_t r = 0;
#pragma unroll
            for (uint32_t i = 0; i < NW; ++i) r |= ((wb >> (i * LPN)) & 1ull) << i;
            wb = r;
        }
        const uint32_t u0 = tile + (threadIdx.x / 64) * NW;  // the wave's first node
        if ((threadIdx.x & 63) == 0 && wb) atomicOr((unsigned long long*)&occ_nxt[u0 / 64], (unsigned long long)(wb << (u0 % 64)));
    }
    unsigned long long cnt[8] = {n_new, n_dup, n_send, n_vnew, n_back, n_rej, n_ign, n_gray};
    const uint32_t slot[8] = {STAT_HOP0 + h, STAT_DUPS, STAT_EDGE_SENDS, STAT_NEW_WORDS, STAT_BACKSENDS,
                              STAT_REJECTED, STAT_IGNORED, STAT_GRAY};
    block_count<8>(cnt, ps.stats, slot);
}

struct DupsLast {  // the last hop run and its frontier rows
    uint32_t h_run;
    bool empty;
    const uint64_t* row;
    const uint64_t* occ;
};
__device__ __forceinline__ DupsLast dups_last(const PropState& ps, uint32_t h_run) {
    // rows after the first hop that delivered nothing were never written
    // (skipped hops); that hop's row is empty and nothing was first received
    // later, so v forwarded its whole seen set
    for (uint32_t hh = 1; hh < h_run && !ps.sharded; ++hh)
        if (ps.stats[STAT_HOP0 + hh] == 0) {
            h_run = hh;
            break;
        }
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    DupsLast L;
    L.h_run = h_run;
    L.row = ps.hist + (size_t)h_run * ps.n_nodes * ps.n_words;
    L.occ = ps.occ + (size_t)h_run * occ_row;
    L.empty = ps.stats[STAT_HOP0 + h_run] == 0 && (!ps.sharded || h_run < ps.max_hops);
    return L;
}

// Per sender v: the size of its forwarded set (seen minus the last hop's
// receipts) and the part of it v published, packed n_all | n_own << 32.  L
// lanes per node, 4 words each per step, summed with shuffles.
template <int L>
__global__ __launch_bounds__(256) void k_prop_vcount(PropState ps, uint32_t h_run, uint64_t* __restrict__ vcnt,
                                                     bool gray_only) {
    if (gray_only && *ps.gray_pairs == 0) return;  // no gated pair: k_prop_dups<true> has nothing to count
    const DupsLast L_ = dups_last(ps, h_run);
    const uint32_t W = ps.n_words;
    const uint32_t lc = threadIdx.x % L;
    const uint32_t CWv = L > 1 ? 4 : W;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t / L < ps.n_nodes; t += gridDim.x * 256u) {
        const uint32_t v = t / L;
        const bool v_src = occ_bit(ps.occ, v);
        const bool v_last = !L_.empty && occ_bit(L_.occ, v);
        uint32_t n_all = 0, n_own = 0;
        for (uint32_t w0 = lc * CWv; w0 < W; w0 += L * CWv)
            for (uint32_t w = w0; w < w0 + CWv; ++w) {
                const size_t vw = (size_t)v * W + w;
                uint64_t s = ps.seen[vw];
                if (ps.drop) s &= ~ps.drop[w];  // never forwarded, not even by their source's peers
                if (v_last) s &= ~L_.row[vw];
                n_all += __popcll(s);
                if (v_src) n_own += __popcll(s & ps.origin[vw]);
            }
        if (L > 1) {
            n_all = group_sum<L>(n_all);
            n_own = group_sum<L>(n_own);
        }
        uint64_t fh = 0;  // edge_late: the hops 2 .. h_run at which v forwarded received messages
        if (ps.edge_late && lc == 0) {
            const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
            for (uint32_t hh = 1; hh + 1 <= L_.h_run; ++hh) fh += occ_bit(ps.occ + (size_t)hh * occ_row, v);
        }
        if (lc == 0) vcnt[v] = (uint64_t)n_all | ((uint64_t)n_own << 32) | (fh << 56);
    }
}

// One thread per sender pair; the sends land in corr[r] (unused by the late
// accounting otherwise) and k_prop_count moves them to the receiver's pair,
// so no thread scatters into another pair's counter.  A pair takes the
// per-word path only for RandomSub draws, tracked `from` rows, or a
// publishing u; every other pair reads its class's count from vcnt.
// Batches of DU pairs per thread (q0 + i * stride): the loads of a batch are
// issued together, so a thread waits for one round of latencies per batch
// rather than one per pair.
constexpr int DU = 4;
constexpr int FH = 2;  // fold_rescore_1: pairs whose loads are in flight together
// With the graylist gate (ps.gate), a pair whose receiver drops the sender's
// RPCs (FWD_GIN on the receiver's pair q) sends the same copies, but they are
// dropped at u before pushMsg: they count as STAT_GRAY, never as duplicates,
// and leave no correction in corr[r].  Those copies include the messages v
// published that validation does not accept (their copies to accepting
// receivers are rejected/ignored receipts of the hop kernels).  GRAY_ONLY
// (per-hop accounting, where duplicates are counted on arrival) visits only
// the gated pairs.
template <bool GRAY_ONLY, int DD = DU>
__global__ __launch_bounds__(256) void k_prop_dups(PropState ps, uint32_t h_run, const uint64_t* __restrict__ vcnt) {
    if (GRAY_ONLY && *ps.gray_pairs == 0) return;
    unsigned long long cnt[4] = {0, 0, 0, 0};
    const uint32_t W = ps.n_words;
    const DupsLast L = dups_last(ps, h_run);
    h_run = L.h_run;
    const uint64_t* src_occ = ps.occ;  // row 0: nodes that published in this call
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t r0 = (uint64_t)blockIdx.x * 256u + threadIdx.x; r0 < ps.n_pairs; r0 += stride * DD) {
        uint32_t qa[DD], va[DD], ua[DD], af[DD], as_[DD];
        uint8_t fa[DD];
#pragma unroll
        for (int i = 0; i < DD; ++i) {
            const uint64_t r = r0 + i * stride;
            const bool in = r < ps.n_pairs;
            qa[i] = in ? ps.rev[r] : NO_PAIR;  // the receiver's pair (u -> v)
            fa[i] = in ? ps.fwd[r] : 0;
            va[i] = in ? ps.pair_obs[r] : 0;
            ua[i] = in ? (uint32_t)ps.col[r] - ps.node_lo : 0;
            // deferred folds: the pair's sums, loaded with the rest (written back below)
            af[i] = (!GRAY_ONLY && ps.acc_f && in) ? ps.acc_f[r] : 0u;
            as_[i] = (!GRAY_ONLY && ps.acc_s && in) ? ps.acc_s[r] : 0u;
        }
        bool ga[DD];  // u drops v's copies: the GIN bit of u's pair (v's reverse), kept beside r by k_prop_pin
#pragma unroll
        for (int i = 0; i < DD; ++i) {
            const uint64_t r = r0 + i * stride;
            const bool local = qa[i] != NO_PAIR && !(qa[i] & HALO) && (fa[i] & FWD_SEND);
            ga[i] = local && ps.gate && (ps.rfwd[r] & FWD_GIN);
            if (GRAY_ONLY && !ga[i]) qa[i] = NO_PAIR;
        }
        uint64_t vca[DD], fla[DD];
        uint32_t fca[DD];
#pragma unroll
        for (int i = 0; i < DD; ++i) {
            const uint64_t r = r0 + i * stride;
            const bool live = qa[i] != NO_PAIR && !(qa[i] & HALO) && (fa[i] & FWD_SEND);
            vca[i] = live ? vcnt[va[i]] : 0;
            const bool fl = live && !ps.from_mask && (fa[i] & FWD_FORWARD) && h_run >= 1;
            fca[i] = (fl || (ps.acc_f && r < ps.n_pairs)) ? ps.fcnt[r] : 0;
            fla[i] = (fl && ps.flast_live) ? ps.flast[r] : 0;
        }
        if (!GRAY_ONLY && ps.edge_late) {  // STAT_EDGE_SENDS of one-word calls (k_prop_hop_fast1 skips
                                           // saturated receivers): per pair u's pin lets through, the hops at
                                           // which v's row was non-empty: hop 1 its publishes, later ones
                                           // its receipts of the hop before (vcount's forwarding hops)
#pragma unroll
            for (int i = 0; i < DD; ++i) {
                const uint64_t r = r0 + i * stride;
                if (qa[i] == NO_PAIR || (qa[i] & HALO) || !(fa[i] & FWD_SEND) || ga[i] || (ps.rfwd[r] & FWD_GIN))
                    continue;
                cnt[3] += ((fa[i] & FWD_PUBLISH) && h_run >= 1 && occ_bit(src_occ, va[i]) ? 1u : 0u) +
                          ((fa[i] & FWD_FORWARD) ? (uint32_t)(vca[i] >> 56) : 0u);
            }
        }
        if (!GRAY_ONLY && ps.acc_f) {  // deferred folds: r as a receiver pair — its first receipts join its sum
#pragma unroll
            for (int i = 0; i < DD; ++i) {
                const uint64_t r = r0 + i * stride;
                if (r >= ps.n_pairs || !fca[i]) continue;
                ps.acc_f[r] = af[i] + fca[i];
                const uint32_t rr = ps.rev[r];
                if (rr != NO_PAIR && !(rr & HALO)) cnt[2] += fca[i];  // the back-sends (k_prop_count's count)
            }
        }
#pragma unroll
        for (int i = 0; i < DD; ++i) {
            const uint64_t r = r0 + i * stride;
            const uint32_t q = qa[i];
            const uint8_t fw = fa[i];
            if (q == NO_PAIR || (q & HALO) || !(fw & FWD_SEND)) continue;
            const uint32_t v = va[i], u = ua[i];
            const bool u_src = occ_bit(src_occ, u);
            const bool v_src = occ_bit(src_occ, v);
            uint32_t sends = 0, pub = 0;
            if (!u_src && !ps.sel && !ps.from_mask) {
                const uint64_t vc = vca[i];
                const uint32_t n_all = (uint32_t)vc, n_own = (uint32_t)(vc >> 32) & 0xFFFFFFu;
                const uint8_t m = fw & (FWD_FORWARD | FWD_PUBLISH);
                sends = m == (FWD_FORWARD | FWD_PUBLISH) ? n_all : m == FWD_FORWARD ? n_all - n_own
                      : m == FWD_PUBLISH ? n_own : 0;
            } else {
                const bool v_last = !L.empty && occ_bit(L.occ, v);
                for (uint32_t w = 0; w < W; ++w) {
                    const size_t vw = (size_t)v * W + w;
                    uint64_t sb = ps.seen[vw];
                    if (v_last) sb &= ~L.row[vw];
                    sb &= elig_word(fw, v_src ? ps.origin[vw] : 0);
                    if (ps.sel) sb |= ps.sel[r * W + w];
                    if (ps.from_mask) sb &= ~ps.from_mask[r * W + w];
                    if (ps.drop) sb &= ~ps.drop[w];  // copies of dropped messages are receipts, not deliveries
                    if (u_src) {
                        const uint64_t ou = ps.origin[(size_t)u * W + w] & (ps.drop ? ~ps.drop[w] : ~0ull);
                        sb &= ~ou;
                        pub += __popcll(ou);
                    }
                    sends += __popcll(sb);
                }
            }
            if (!ps.from_mask && (fw & FWD_FORWARD) && h_run >= 1) {
                const uint64_t fl = fla[i];
                const uint32_t from_last = (!L.empty && (uint32_t)(fl >> 32) == h_run) ? (uint32_t)fl : 0;
                // u's own messages v first got from u: all of them iff u publishes to v
                // and v accepts u's RPCs (pub != 0 only if u published)
                const uint32_t from_pub = (pub && (ps.fwd[q] & FWD_PUBLISH) && !(fw & FWD_GIN)) ? pub : 0;
                sends -= fca[i] - from_last - from_pub + ((h_run == 1 && !L.empty) ? from_pub : 0);
            }
            if (ga[i]) {
                if (ps.drop && v_src && (fw & FWD_PUBLISH))  // v's own unaccepted messages, sent at hop 1
                    for (uint32_t w = 0; w < W; ++w) sends += __popcll(ps.origin[(size_t)v * W + w] & ps.drop[w]);
                cnt[1] += sends;
                if (!GRAY_ONLY) ps.corr[r] = 0;
            } else {
                cnt[0] += sends;
                if (ps.acc_s) {  // deferred folds: the sends join the sender pair's sum
                    if (sends) ps.acc_s[r] = as_[i] + sends;
                } else {
                    ps.corr[r] = sends;
                }
            }
        }
    }
    const uint32_t slot[4] = {STAT_DUPS, STAT_GRAY, STAT_BACKSENDS, STAT_EDGE_SENDS};
    block_count<4>(cnt, ps.stats, slot);
}

// ---- range shards, replicated frontier (PropState::rep) -------------------------
// The lean calls (late duplicate accounting, no RandomSub draws, no
// first-deliverer rows) on range shards keep every node's frontier row of the
// last two hops on every rank (front_g / occ_g, global node ids), so a remote
// sender's row is gathered exactly as a local one and nothing per pair
// crosses shards during the hops:
//  * hop 0 (the call's publishes) is known everywhere: every rank writes row 0
//    of every source from the message list (k_rep_init);
//  * after hop h each rank contributes the rows of its nodes that received at
//    h (k_rep_pack: entries [global id][W words]) and the others' entries are
//    scattered into row h (k_rep_scatter); the driver moves them with one
//    all-gather per hop;
//  * the eligibility of a remote pair (v -> u) comes with v's fwd byte once per
//    call (k_rep_fwd_pack / k_rep_fwd_recv build u's pin from it);
//  * the `from` exclusion never changes a first receipt (a message v sends back
//    to u is one u has seen), so it is settled at the call's end like the local
//    pairs' (k_prop_dups): v's rank computes what each cross pair sent over the
//    call (k_rep_sends) and u's rank turns it into duplicates or graylisted
//    copies (k_rep_sends_recv).
__global__ __launch_bounds__(256) void k_rep_zero_src(PropState ps) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint32_t W = ps.n_words;
    if (i >= (uint64_t)ps.n_msgs * W) return;
    ps.front_g[(size_t)ps.msgs[i / W].source * W + i % W] = 0;  // (parity 0)
}
// The first entry of rmark_v equal to g (n_rmark if none): the receivers of a
// remote sender g are rmark_u[lo .. while rmark_v == g].
__device__ __forceinline__ uint64_t rmark_lower(const PropState& ps, uint32_t g) {
    uint64_t lo = 0, hi = ps.n_rmark;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (ps.rmark_v[mid] < g) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ void rep_mark_receivers(const PropState& ps, uint32_t g, uint64_t* touch) {
    for (uint64_t i = rmark_lower(ps, g); i < ps.n_rmark && ps.rmark_v[i] == g; ++i) {
        const uint32_t u = ps.rmark_u[i];
        atomicOr((unsigned long long*)&touch[u / 64], 1ull << (u % 64));
    }
}
__global__ __launch_bounds__(256) void k_rep_init(PropState ps) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= ps.n_msgs) return;
    const uint32_t W = ps.n_words, g = ps.msgs[k].source;
    atomicOr((unsigned long long*)&ps.front_g[(size_t)g * W + k / 64], 1ull << (k % 64));
    atomicOr((unsigned long long*)&ps.occ_g[g / 64], 1ull << (g % 64));
    atomicOr((unsigned long long*)&ps.src_bits[g / 64], 1ull << (g % 64));
    // hop 1's very sparse marking (mark_hop): a remote source marks its receivers here
    // (a local one is marked by k_prop_mark(1) with the rest of the local frontier)
    const bool remote = g < ps.node_lo || g - ps.node_lo >= ps.n_nodes;
    if (remote && mark_hop(ps, 1)) rep_mark_receivers(ps, g, ps.touch + (((size_t)ps.n_nodes + 63) / 64));
}
// This rank's entries of hop h: its nodes whose row h is non-empty, in node
// order (a block scan places each thread's run of four nodes), so a
// receiver's wave meets runs of neighbouring ids (k_rep_scatter's occupancy
// words and row stores).
__global__ __launch_bounds__(256) void k_rep_pack(PropState ps, uint32_t h, uint64_t* __restrict__ out,
                                                  unsigned long long* __restrict__ cnt) {
    __shared__ uint32_t wsum[4];
    __shared__ uint64_t base;
    const uint32_t W = ps.n_words;
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    const uint64_t* occ_h = ps.occ + (size_t)h * occ_row;
    const uint64_t* row_h = ps.hist + (size_t)h * ps.n_nodes * W;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t u0 = blockIdx.x * 1024u; u0 < ps.n_nodes; u0 += gridDim.x * 1024u) {
        const uint32_t ub = u0 + threadIdx.x * 4;  // this thread's four nodes
        uint32_t bits = 0;
        if (ub < ps.n_nodes) {
            const uint64_t ow = occ_h[ub / 64] >> (ub % 64);  // (4 | 64: the four share a word)
            bits = (uint32_t)(ow & 0xF);
            if (ub + 4 > ps.n_nodes) bits &= (1u << (ps.n_nodes - ub)) - 1;
        }
        const uint32_t mine = __popc(bits);
        uint32_t incl = mine;  // inclusive scan over the wave
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            before += k < wv ? wsum[k] : 0u;
            tot += wsum[k];
        }
        if (threadIdx.x == 0) base = tot ? atomicAdd(cnt, (unsigned long long)tot) : 0ull;
        __syncthreads();
        uint64_t pos = base + before + incl - mine;
        for (uint32_t i = 0; i < 4; ++i) {
            if (!((bits >> i) & 1)) continue;
            const uint32_t u = ub + i;
            uint64_t* e = out + pos++ * (uint64_t)(W + 1);
            e[0] = ps.node_lo + u;
            for (uint32_t w = 0; w < W; ++w) e[1 + w] = row_h[(size_t)u * W + w];
        }
        __syncthreads();  // (wsum / base are reused by the next chunk)
    }
}
__device__ __forceinline__ uint64_t wave_or(uint64_t x) {
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) x |= __shfl_xor(x, o, 64);
    return x;
}
// Another rank's entries of hop h into the replicated rows of hop h (parity
// h & 1), their occupancy bits (the lanes of a wave that share a word OR
// their bits first: one atomic per word, not per entry), and (when hop h + 1
// is very sparse) the marks of their local receivers.
__global__ __launch_bounds__(256) void k_rep_scatter(PropState ps, uint32_t h, RepParts parts) {
    const uint64_t n = parts.off[parts.n];
    const uint32_t W = ps.n_words;
    const size_t occ_g_row = ((size_t)ps.n_total + 63) / 64 + 1;
    uint64_t* rg = ps.front_g + (size_t)(h & 1) * ps.n_total * W;
    uint64_t* og = ps.occ_g + (size_t)(h & 1) * occ_g_row;
    const bool mark = mark_hop(ps, h + 1);
    uint64_t* touch = ps.touch + (size_t)((h + 1) & 1) * (((size_t)ps.n_nodes + 63) / 64);
    const uint32_t lane = threadIdx.x & 63;
    // (a whole-wave loop: every lane runs the same trip count, the ballots stay uniform)
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256u + (threadIdx.x & ~63u); i0 < n; i0 += (uint64_t)gridDim.x * 256u) {
        const uint64_t i = i0 + lane;
        const bool valid = i < n;
        uint32_t g = 0;
        if (valid) {
            uint32_t k = 0;  // the part holding entry i (every rank's entries in one launch)
            while (parts.off[k + 1] <= i) ++k;
            const uint64_t* e = parts.p[k] + (i - parts.off[k]) * (uint64_t)(W + 1);
            g = (uint32_t)e[0];
            for (uint32_t w = 0; w < W; ++w) rg[(size_t)g * W + w] = e[1 + w];
            if (mark) rep_mark_receivers(ps, g, touch);
        }
        uint64_t todo = __ballot(valid);
        while (todo) {
            const uint32_t leader = (uint32_t)__builtin_ctzll(todo);
            const uint32_t lw = __shfl(g / 64, leader, 64);
            const bool same = valid && g / 64 == lw;
            const uint64_t bits = wave_or(same ? 1ull << (g % 64) : 0ull);
            if (lane == leader) atomicOr((unsigned long long*)&og[lw], (unsigned long long)bits);
            todo &= ~__ballot(same);
        }
    }
}
// Once per call: the fwd byte of every pair a remote receiver asked for, in
// send-slot order, and on the receiving side the pins they give.
__global__ __launch_bounds__(256) void k_rep_fwd_pack(PropState ps, uint8_t* __restrict__ out) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < ps.n_send; j += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = ps.send_pair[j];
        out[j] = r == NO_PAIR ? 0 : ps.fwd[r];
    }
}
// (pair order: a receive slot's pairs come ascending per owner rank, so the
// slot reads run forward while the pair's own arrays are read coalesced)
__global__ __launch_bounds__(256) void k_rep_fwd_recv(PropState ps, const uint8_t* __restrict__ in) {
    for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < ps.n_pairs; q += (uint64_t)gridDim.x * 256u) {
        const uint32_t rv = ps.rev[q];
        if (rv == NO_PAIR || !(rv & HALO)) continue;
        const uint8_t fw = in[rv & HALO_SLOT];
        const bool gin = ps.fwd[q] & FWD_GIN;  // u drops whatever v sends (AcceptFrom)
        ps.pin[q] = (!gin && (fw & (FWD_FORWARD | FWD_PUBLISH)))
                        ? ((uint32_t)(fw & (FWD_FORWARD | FWD_PUBLISH)) << PIN_FWD_SHIFT) | (uint32_t)ps.col[q]
                        : NO_PAIR;
        ps.rfwd[q] = fw;
    }
}
// The origin row word w of a (possibly remote) node g: the messages it published.
__device__ __forceinline__ uint64_t rep_origin(const PropState& ps, uint32_t g, uint32_t w) {
    if (!((ps.src_bits[g / 64] >> (g % 64)) & 1)) return 0;
    uint32_t lo = 0, hi = ps.n_src;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        if (ps.src_ids[mid] < g) lo = mid + 1;
        else hi = mid;
    }
    return ps.src_rows[(size_t)lo * ps.n_words + w];
}
// At the call's end, per send slot j (pair r = (v -> u), v here, u remote):
// v's sends to u over the call, as k_prop_dups computes them for a local
// receiver (its forwarded set through the pair's eligibility, minus what it
// first got from u and never sends back, minus u's own messages), low word;
// high word: v's own unaccepted messages it sent u at hop 1 (copies a
// graylisting u drops too).  u's own messages v first got from u (from_pub)
// are the ones in v's hop-1 row: only u had them at hop 1.
__global__ __launch_bounds__(256) void k_rep_sends(PropState ps, uint32_t h_run, const uint64_t* __restrict__ vcnt,
                                                   uint64_t* __restrict__ out) {
    const uint32_t W = ps.n_words;
    const DupsLast L = dups_last(ps, h_run);
    h_run = L.h_run;
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    // (pair order: the pair's own arrays are read along the sender's row; one
    // scattered store per cross pair)
    for (uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x; r < ps.n_pairs; r += (uint64_t)gridDim.x * 256u) {
        const uint32_t j = ps.send_slot[r];
        if (j == NO_PAIR) continue;  // a local receiver (k_prop_dups), or nobody asked
        const uint8_t fw = ps.fwd[r];
        if (!(fw & FWD_SEND)) {
            out[j] = 0;
            continue;
        }
        const uint32_t v = ps.pair_obs[r], g = (uint32_t)ps.col[r];
        const bool v_src = occ_bit(ps.occ, v);
        const bool u_src = (ps.src_bits[g / 64] >> (g % 64)) & 1;
        uint32_t sends = 0, pub = 0, from_pub = 0, xdrop = 0;
        if (!u_src) {
            const uint64_t vc = vcnt[v];
            const uint32_t n_all = (uint32_t)vc, n_own = (uint32_t)(vc >> 32) & 0xFFFFFFu;
            const uint8_t m = fw & (FWD_FORWARD | FWD_PUBLISH);
            sends = m == (FWD_FORWARD | FWD_PUBLISH) ? n_all : m == FWD_FORWARD ? n_all - n_own
                  : m == FWD_PUBLISH ? n_own : 0;
        } else {
            const bool v_last = !L.empty && occ_bit(L.occ, v);
            const bool v_h1 = occ_bit(ps.occ + occ_row, v);
            for (uint32_t w = 0; w < W; ++w) {
                const size_t vw = (size_t)v * W + w;
                uint64_t sb = ps.seen[vw];
                if (v_last) sb &= ~L.row[vw];
                sb &= elig_word(fw, v_src ? ps.origin[vw] : 0);
                if (ps.drop) sb &= ~ps.drop[w];
                const uint64_t ou = rep_origin(ps, g, w) & (ps.drop ? ~ps.drop[w] : ~0ull);
                sends += __popcll(sb & ~ou);
                pub += __popcll(ou);
                if (v_h1) from_pub += __popcll(ps.hist[(size_t)ps.n_nodes * W + vw] & ou);
            }
        }
        if ((fw & FWD_FORWARD) && h_run >= 1) {
            const uint64_t fl = ps.flast[r];
            const uint32_t from_last = (!L.empty && (uint32_t)(fl >> 32) == h_run) ? (uint32_t)fl : 0;
            if (!pub) from_pub = 0;
            sends -= ps.fcnt[r] - from_last - from_pub + ((h_run == 1 && !L.empty) ? from_pub : 0);
        }
        if (ps.drop && v_src && (fw & FWD_PUBLISH))
            for (uint32_t w = 0; w < W; ++w) xdrop += __popcll(ps.origin[(size_t)v * W + w] & ps.drop[w]);
        // edge_late (one-word calls: at most 64 sends and 64 own copies: 16-bit fields): the
        // hops at which v's row to u was non-empty, as k_prop_dups counts a local pair's —
        // hop 1 its publishes, later ones its receipts of the hop before (vcount's hops);
        // the receiver's rank drops them with the sends when it graylists v
        uint64_t edges = 0;
        if (ps.edge_late)
            edges = ((fw & FWD_PUBLISH) && h_run >= 1 && v_src ? 1u : 0u) +
                    ((fw & FWD_FORWARD) ? (uint32_t)(vcnt[v] >> 56) : 0u);
        out[j] = ps.edge_late ? (uint64_t)sends | ((uint64_t)xdrop << 16) | (edges << 32)
                              : (uint64_t)sends | ((uint64_t)xdrop << 32);
    }
}
// At u's rank, per receive slot (pair q = (u -> v), v remote): v's sends
// become duplicates (P3 credits through the pending counts: sends minus u's
// first receipts from v) or, when u's AcceptFrom drops v, graylisted copies.
__global__ __launch_bounds__(256) void k_rep_sends_recv(PropState ps, const uint64_t* __restrict__ in) {
    unsigned long long cnt[3] = {0, 0, 0};
    for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < ps.n_pairs; q += (uint64_t)gridDim.x * 256u) {
        const uint32_t rv = ps.rev[q];
        if (rv == NO_PAIR || !(rv & HALO)) continue;
        const uint64_t x = in[rv & HALO_SLOT];
        if (!x) continue;
        const uint32_t sends = ps.edge_late ? (uint32_t)x & 0xFFFFu : (uint32_t)x;
        const uint32_t xdrop = ps.edge_late ? (uint32_t)(x >> 16) & 0xFFFFu : (uint32_t)(x >> 32);
        const uint32_t edges = ps.edge_late ? (uint32_t)(x >> 32) : 0u;
        const bool gin = (ps.fwd[q] & FWD_GIN) != 0;  // u drops v's RPCs
        if (ps.gate && gin) {
            cnt[1] += sends + xdrop;
        } else {
            const uint32_t dup = sends - ps.fcnt[q];
            cnt[0] += dup;
            if (dup && ps.credit) ps.dupcnt[q] += dup;
        }
        if (!gin) cnt[2] += edges;  // (one engine's compacted senders leave a graylisted sender out)
    }
    const uint32_t slot[3] = {STAT_DUPS, STAT_GRAY, STAT_EDGE_SENDS};
    block_count<3>(cnt, ps.stats, slot);
}

// ---- P2/P3 credits ------------------------------------------------------------
// Per receiver pair q = (u -> v), add this call's first receipts from v (the
// hop kernel's fcnt) and in-window duplicates to the pending counts.
// Fold pending counts: k1 first receipts, k2 duplicates inside the window.
// markFirstMessageDelivery: fmd k1 steps of +1 then cap, mmd too when in
// mesh; markDuplicateMessageDelivery: mmd k2 more steps when in mesh
// (score.go:912-974).  All steps are identical, so their order does not
// matter; add_ones_capped gives the result of the steps one by one.
__device__ __forceinline__ void fold_pair(const PropState& ps, const DevState& s, uint64_t q, uint32_t k1, uint32_t k2,
                                          uint32_t k4 = 0) {
    const DevTopicParams& tp = s.tp[ps.topic];
    const size_t b = rec_index(q, ps.topic, s.n_topics, FMD);
    // markInvalidMessageDelivery (score.go:894-907): k4 steps of +1, no cap
    if (k4) s.rec[b + IMD * TILE] = add_ones_capped(s.rec[b + IMD * TILE], k4, __builtin_inf());
    if (k1 == 0 && k2 == 0) return;
    s.rec[b + FMD * TILE] = add_ones_capped(s.rec[b + FMD * TILE], k1, tp.cap2);
    if (!(s.rflags[flag_index(q, ps.topic, s.n_topics)] & REC_IN_MESH)) return;
    s.rec[b + MMD * TILE] = add_ones_capped(s.rec[b + MMD * TILE], k1 + k2, tp.cap3);
}

// Per receiver pair q = (u -> v): this call's first receipts from v (the hop
// kernel's fcnt) and in-window duplicates join the pending counts; with FOLD
// (GSX_CREDIT_NOW) they are folded into the record at once.  RESCORE (the
// scores were exact when the call started, the last fwd pass used this
// call's settings): a folded pair is re-scored here, its forwarding byte
// recomputed and, when it changed, listed for the next call's pins — the only
// scores and bytes the credits can change, so neither a full re-score nor a
// k_prop_fwd pass is needed before the next call (or heartbeat).
// score(q) after a fold of topic ps.topic, through the topic-term cache
// (PropState::tterm): a pair whose terms are current re-reads only the folded
// topic's record; any other computes and stores every term.  Either way the
// terms are summed from 0 in ascending topic order, as eval_pair does.
__device__ __forceinline__ double eval_pair_cached(const PropState& ps, const DevState& s, const DevPeerParams& pp,
                                                   uint64_t q) {
    const uint32_t T = s.n_topics;
    double* tt = ps.tterm + q * T;
    double score = 0.0;
    if (ps.tgen[q] == ps.tepoch) {
        for (uint32_t t = 0; t < T; ++t) {
            const DevTopicParams& tp = s.tp[t];
            if (!tp.scored) continue;
            double term;
            if (t == ps.topic) {
                const uint8_t fl = s.rflags[flag_index(q, t, T)];
                const size_t b = rec_index(q, t, T, FMD);
                term = topic_score(tp, fl, mesh_time_of(s, fl, q, t), s.rec[b], s.rec[b + MMD * TILE],
                                   s.rec[b + MFP * TILE], s.rec[b + IMD * TILE]);
                tt[t] = term;
            } else {
                term = tt[t];
            }
            score += term;
        }
    } else {
        for (uint32_t t = 0; t < T; ++t) {
            const DevTopicParams& tp = s.tp[t];
            if (!tp.scored) continue;
            const uint8_t fl = s.rflags[flag_index(q, t, T)];
            const size_t b = rec_index(q, t, T, FMD);
            const double term = topic_score(tp, fl, mesh_time_of(s, fl, q, t), s.rec[b], s.rec[b + MMD * TILE],
                                            s.rec[b + MFP * TILE], s.rec[b + IMD * TILE]);
            tt[t] = term;
            score += term;
        }
        ps.tgen[q] = ps.tepoch;
    }
    return score_tail(s, pp, q, score, s.bp[q]);
}

// k_prop_count's fold + re-score for one topic (the propagation engines'
// shape), DU pairs at a time in three phases — the counts, then every load
// the fold, score() and the forwarding byte need, then the arithmetic and the
// stores — so a thread waits for one round of latencies per batch, not three
// per pair (the stores of one pair no longer order the next pair's loads).
// Bit-identical to fold_pair + eval_pair + fwd_byte pair by pair: the same
// operations on the same values in the same order.
__device__ __forceinline__ void fold_rescore_1(const PropState& ps, const DevState& s, const DevPeerParams& pp,
                                               uint64_t q0, uint64_t stride, const uint32_t (&k1a)[DU],
                                               const uint32_t (&ra)[DU], const uint32_t (&ca)[DU], bool fold_topic,
                                               unsigned long long& backsends) {
    const uint32_t t = ps.topic;
    uint32_t fa[DU], da[DU], k4a[DU];
    bool doit[DU];
#pragma unroll
    for (int i = 0; i < DU; ++i) {  // counts (as the general loop)
        const uint64_t q = q0 + i * stride;
        doit[i] = false;
        fa[i] = da[i] = k4a[i] = 0;
        if (q >= ps.n_pairs) continue;
        const uint32_t k1 = k1a[i], r = ra[i];
        const bool local = r != NO_PAIR && !(r & HALO);
        if (ps.credit) {
            const uint32_t f0 = ps.pending ? ps.firstcnt[q] : 0, d0 = ps.pending ? ps.dupcnt[q] : 0;
            uint32_t first = f0 + k1, dup = d0;
            if (local) {
                if (ps.late) dup += ca[i] - k1;
                else dup -= ca[i];
            }
            if (f0 | d0) {
                ps.firstcnt[q] = 0;
                ps.dupcnt[q] = 0;
            }
            uint32_t k4 = 0;
            if ((ps.drop || ps.pending) && (k4 = ps.invcnt[q])) ps.invcnt[q] = 0;
            fa[i] = first;
            da[i] = dup;
            k4a[i] = k4;
            doit[i] = (first | dup | k4) && fold_topic && (s.pflags[q] & PAIR_PRESENT);
        }
        if (ps.late && local) backsends += k1;
    }
    if (ps.stale) {  // lazy: credits only (no P4) of pairs at or above every threshold fold without a re-score
        bool lz[DU];
#pragma unroll
        for (int i = 0; i < DU; ++i) lz[i] = doit[i] && k4a[i] == 0 && s.score[q0 + i * stride] >= ps.lazy_thr;
#pragma unroll
        for (int i = 0; i < DU; ++i) {
            if (!lz[i]) continue;
            const uint64_t q = q0 + i * stride;
            doit[i] = false;
            ps.stale[q] = 1;
            if (!(fa[i] | da[i])) continue;
            const size_t b = rec_index(q, t, 1, FMD);
            const uint8_t fl = s.rflags[flag_index(q, t, 1)];
            s.rec[b + FMD * TILE] = add_ones_capped(s.rec[b + FMD * TILE], fa[i], s.tp[t].cap2);
            if (fl & REC_IN_MESH) s.rec[b + MMD * TILE] = add_ones_capped(s.rec[b + MMD * TILE], fa[i] + da[i], s.tp[t].cap3);
        }
    }
    for (int h0 = 0; h0 < DU; h0 += FH) {  // (halves: fewer live registers per batch)
    uint8_t fl[FH];
    double fmd[FH], mmd[FH], mfp[FH], imd[FH], app[FH], bp[FH];
    int64_t graft[FH];
    uint2 ipg[FH];
#pragma unroll
    for (int j = 0; j < FH; ++j) {  // every load of the half
        const int i = h0 + j;
        if (!doit[i]) continue;
        const uint64_t q = q0 + i * stride;
        const size_t b = rec_index(q, t, 1, FMD);
        fl[j] = s.rflags[flag_index(q, t, 1)];
        fmd[j] = s.rec[b + FMD * TILE];
        mmd[j] = s.rec[b + MMD * TILE];
        mfp[j] = s.rec[b + MFP * TILE];
        imd[j] = s.rec[b + IMD * TILE];
        graft[j] = reinterpret_cast<const int64_t*>(s.rec)[rec_index(q, t, 1, GRAFT)];
        app[j] = s.app[q];
        bp[j] = s.bp[q];
        if (pp.w6 != 0.0) ipg[j] = reinterpret_cast<const uint2*>(s.ipg)[q];
    }
    uint32_t ipc[FH][2];
    if (pp.w6 != 0.0) {
#pragma unroll
        for (int j = 0; j < FH; ++j) {
            const int i = h0 + j;
            ipc[j][0] = ipc[j][1] = 0;
            if (!doit[i]) continue;
            const uint32_t gs[2] = {ipg[j].x, ipg[j].y};
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (!(gs[k] == IPG_NONE || (gs[k] & IPG_WL))) ipc[j][k] = s.ipcount[gs[k]];
        }
    }
    const DevTopicParams& tp = s.tp[t];
#pragma unroll
    for (int j = 0; j < FH; ++j) {  // fold_pair, eval_pair, fwd_byte
        const int i = h0 + j;
        if (!doit[i]) continue;
        const uint64_t q = q0 + i * stride;
        const size_t b = rec_index(q, t, 1, FMD);
        const uint32_t k1 = fa[i], k2 = da[i], k4 = k4a[i];
        if (k4) {
            imd[j] = add_ones_capped(imd[j], k4, __builtin_inf());
            s.rec[b + IMD * TILE] = imd[j];
        }
        if (k1 | k2) {
            fmd[j] = add_ones_capped(fmd[j], k1, tp.cap2);
            s.rec[b + FMD * TILE] = fmd[j];
            if (fl[j] & REC_IN_MESH) {
                mmd[j] = add_ones_capped(mmd[j], k1 + k2, tp.cap3);
                s.rec[b + MMD * TILE] = mmd[j];
            }
        }
        const int64_t mt = (!(fl[j] & REC_IN_MESH) || (fl[j] & REC_FRESH)) ? 0 : s.last_refresh - graft[j];
        double score = 0.0;
        score += topic_score(tp, fl[j], mt, fmd[j], mmd[j], mfp[j], imd[j]);
        // score_tail with the loaded values
        if (pp.topic_score_cap > 0 && score > pp.topic_score_cap) score = pp.topic_score_cap;
        score += app[j] * pp.w5;
        if (pp.w6 != 0.0) {
            double p6 = 0.0;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t id = k ? ipg[j].y : ipg[j].x;
                if (id == IPG_NONE || (id & IPG_WL)) continue;
                const int64_t peers_in_ip = (int64_t)ipc[j][k];
                if (peers_in_ip > pp.thr6) {
                    const double surpluss = (double)(peers_in_ip - pp.thr6);
                    p6 += surpluss * surpluss;
                }
            }
            score += p6 * pp.w6;
        }
        if (bp[j] > pp.thr7) {
            const double excess = bp[j] - pp.thr7;
            const double p7 = excess * excess;
            score += p7 * pp.w7;
        }
        s.score[q] = score;
        const uint8_t ob = ps.fwd[q], nb = fwd_byte(ps, s, q);
        if (nb != ob) {
            ps.fwd[q] = nb;
            const uint32_t k = atomicAdd(ps.nchg, 1u);
            if (k < ps.chg_cap) ps.chg[k] = (uint32_t)q;
            if ((nb ^ ob) & FWD_GIN) atomicAdd(ps.gray_pairs, (nb & FWD_GIN) ? 1ull : ~0ull);  // (+1 / -1)
        }
    }
    }
}

template <bool FOLD, bool RESCORE, bool ONE_TOPIC = false>
__global__ __launch_bounds__(256) void k_prop_count(PropState ps, DevState s, DevPeerParams pp) {
    unsigned long long cnt[1] = {0};
    const bool fold_topic = FOLD && ps.topic < s.n_topics && s.tp[ps.topic].scored;
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t q0 = (uint64_t)blockIdx.x * 256u + threadIdx.x; q0 < ps.n_pairs; q0 += stride * DU) {
        uint32_t k1a[DU], ra[DU], ca[DU];
#pragma unroll
        for (int i = 0; i < DU; ++i) {
            const uint64_t q = q0 + i * stride;
            const bool in = q < ps.n_pairs;
            k1a[i] = in ? ps.fcnt[q] : 0;
            ra[i] = in ? ps.rev[q] : NO_PAIR;
        }
#pragma unroll
        for (int i = 0; i < DU; ++i) {  // the sender pair's sends (k_prop_dups), one gather per pair
            const uint64_t q = q0 + i * stride;
            const bool local = ra[i] != NO_PAIR && !(ra[i] & HALO);
            // late accounting: k_prop_dups wrote corr of the senders whose byte has SEND
            // (rfwd: the reverse pair's byte as this call's pins read it), nothing else
            const bool wrote = !ps.late || (q < ps.n_pairs && (ps.rfwd[q] & FWD_SEND));
            ca[i] = (local && ps.credit && wrote) ? ps.corr[ra[i]] : 0;
        }
        if (ONE_TOPIC) {  // the batched fold + re-score (its own instantiation: its registers do not
                          // cost the general loop occupancy)
            fold_rescore_1(ps, s, pp, q0, stride, k1a, ra, ca, fold_topic, cnt[0]);
            continue;
        }
#pragma unroll
        for (int i = 0; i < DU; ++i) {
            const uint64_t q = q0 + i * stride;
            if (q >= ps.n_pairs) break;
            const uint32_t k1 = k1a[i];
            const uint32_t r = ra[i];
            const bool local = r != NO_PAIR && !(r & HALO);
            if (ps.credit) {
                // (unsharded, late accounting, nothing deferred: the hops wrote no
                // pending counts and none were left, so they are not read)
                const uint32_t f0 = ps.pending ? ps.firstcnt[q] : 0, d0 = ps.pending ? ps.dupcnt[q] : 0;
                uint32_t first = f0 + k1, dup = d0;
                if (local) {
                    if (ps.late) dup += ca[i] - k1;  // k_prop_dups: every send from v, first receipts too
                    else dup -= ca[i];               // in-window back-sends taken back
                }
                if (FOLD) {  // GSX_CREDIT_NOW: fold at once (k_prop_fold) and leave the counts empty
                    if (f0 | d0) {
                        ps.firstcnt[q] = 0;
                        ps.dupcnt[q] = 0;
                    }
                    uint32_t k4 = 0;
                    if ((ps.drop || ps.pending) && (k4 = ps.invcnt[q])) ps.invcnt[q] = 0;
                    if ((first | dup | k4) && fold_topic && (s.pflags[q] & PAIR_PRESENT)) {
                        fold_pair(ps, s, q, first, dup, k4);
                        if (RESCORE && ps.stale && k4 == 0 && s.score[q] >= ps.lazy_thr) {  // lazy (PropState::stale)
                            ps.stale[q] = 1;
                            if (ps.tterm) ps.tgen[q] = 0;  // (its cached term of this topic is stale too)
                        } else if (RESCORE) {
                            s.score[q] = ps.tterm ? eval_pair_cached(ps, s, pp, q) : eval_pair(s, pp, q);
                            const uint8_t ob = ps.fwd[q], nb = fwd_byte(ps, s, q);
                            if (nb != ob) {
                                ps.fwd[q] = nb;
                                const uint32_t k = atomicAdd(ps.nchg, 1u);
                                if (k < ps.chg_cap) ps.chg[k] = (uint32_t)q;
                                if ((nb ^ ob) & FWD_GIN)
                                    atomicAdd(ps.gray_pairs, (nb & FWD_GIN) ? 1ull : ~0ull);  // (+1 / -1)
                            }
                        }
                    }
                } else {
                    ps.firstcnt[q] = first;
                    ps.dupcnt[q] = dup;
                }
            }
            if (ps.late && local) cnt[0] += k1;
        }
    }
    const uint32_t slot[1] = {STAT_BACKSENDS};
    block_count<1>(cnt, ps.stats, slot);
}

// Deferred folds, the call's pass (PropState::acc_s / acc_f): a pair folds
// now only if its score is below lazy_thr (its fwd bytes may depend on the
// credits) or it took a P4 credit this call (invalid deliveries lower a
// score); it folds its whole sums (earlier calls' too: identical +1 steps)
// and is re-scored with its fwd byte, as k_prop_count's RESCORE path does.
__global__ __launch_bounds__(256) void k_prop_defer(PropState ps, DevState s, DevPeerParams pp) {
    const bool fold_topic = ps.topic < s.n_topics && s.tp[ps.topic].scored;
    if (!fold_topic) return;
    // The score a pair's own fwd byte tests (fwd_byte): none for a direct peer;
    // AcceptFrom's graylist threshold; the publish threshold too for a floodsub
    // peer or flood publishing.  Credits only raise the score, so a pair at or
    // above its threshold keeps its byte while its sums wait; a graylisted pair
    // (FWD_GIN) accepts no copy of the sender, so it has no credits at all.
    const double thr_gs = ps.gate ? ps.graylist_threshold : -__builtin_inf();
    const double thr_all = ps.gate ? fmax(ps.graylist_threshold, ps.publish_threshold) : ps.publish_threshold;
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t q0 = (uint64_t)blockIdx.x * 256u + threadIdx.x; q0 < ps.n_pairs; q0 += stride * DU) {
        double sc[DU];
        uint32_t k4a[DU];
        uint8_t pf[DU], ef[DU], fb[DU];
#pragma unroll
        for (int i = 0; i < DU; ++i) {
            const uint64_t q = q0 + i * stride;
            const bool in = q < ps.n_pairs;
            k4a[i] = (in && ps.drop) ? ps.invcnt[q] : 0u;
            pf[i] = in ? s.pflags[q] : 0;
            ef[i] = in ? ps.eflags[q] : 0;
            fb[i] = in ? ps.fwd[q] : 0;
        }
        // The score decides only for a floodsub peer or under flood publish: a
        // gossipsub edge's own threshold is AcceptFrom's (FWD_GIN is exactly
        // score < graylist on the cached scores, and such pairs are skipped), so
        // its score is never read — most of the pass's bytes on a gossipsub overlay
#pragma unroll
        for (int i = 0; i < DU; ++i) {
            const uint64_t q = q0 + i * stride;
            const bool need = q < ps.n_pairs && (pf[i] & PAIR_PRESENT) && !k4a[i] && !(ef[i] & EDGE_DIRECT) &&
                              !(fb[i] & FWD_GIN) && (!(ef[i] & EDGE_GOSSIPSUB) || ps.flood_publish);
            sc[i] = need ? s.score[q] : __builtin_inf();
        }
        bool now_[DU];
#pragma unroll
        for (int i = 0; i < DU; ++i) {
            const uint64_t q = q0 + i * stride;
            now_[i] = false;
            if (q >= ps.n_pairs) continue;
            if (!(pf[i] & PAIR_PRESENT)) {  // no peerStats: nothing to credit (the sums are cleared at the fold)
                if (k4a[i]) ps.invcnt[q] = 0;
                continue;
            }
            if (k4a[i]) {  // invalid deliveries lower the score: fold now
                now_[i] = true;
                continue;
            }
            if ((ef[i] & EDGE_DIRECT) || (fb[i] & FWD_GIN)) continue;
            const double thr = (!(ef[i] & EDGE_GOSSIPSUB) || ps.flood_publish) ? thr_all : thr_gs;
            now_[i] = !(sc[i] >= thr);
        }
#pragma unroll
        for (int i = 0; i < DU; ++i) {
            if (!now_[i]) continue;
            const uint64_t q = q0 + i * stride;
            const uint32_t k1 = ps.acc_f[q];
            const uint32_t r = ps.rev[q];
            const bool local = r != NO_PAIR && !(r & HALO);
            const uint32_t sends = local ? ps.acc_s[r] : 0u;
            if (!(k1 | sends | k4a[i])) continue;
            if (k1) ps.acc_f[q] = 0;
            if (sends) ps.acc_s[r] = 0;
            if (k4a[i]) ps.invcnt[q] = 0;
            fold_pair(ps, s, q, k1, sends - k1, k4a[i]);
            s.score[q] = eval_pair(s, pp, q);
            const uint8_t ob = fb[i], nb = fwd_byte(ps, s, q);
            if (nb != ob) {
                ps.fwd[q] = nb;
                const uint32_t k = atomicAdd(ps.nchg, 1u);
                if (k < ps.chg_cap) ps.chg[k] = (uint32_t)q;
                if ((nb ^ ob) & FWD_GIN) atomicAdd(ps.gray_pairs, (nb & FWD_GIN) ? 1ull : ~0ull);  // (+1 / -1)
            }
        }
    }
}

// Every deferred sum folded (before a reader of records or scores); the
// folded pairs are marked stale for the caller's re-score.
__global__ __launch_bounds__(256) void k_prop_fold_acc(PropState ps, DevState s) {
    const bool fold_topic = ps.topic < s.n_topics && s.tp[ps.topic].scored;
    for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < ps.n_pairs; q += (uint64_t)gridDim.x * 256u) {
        const uint32_t k1 = ps.acc_f[q];
        const uint32_t r = ps.rev[q];
        const uint32_t sends = (r != NO_PAIR && !(r & HALO)) ? ps.acc_s[r] : 0u;
        if (!(k1 | sends) || !fold_topic || !(s.pflags[q] & PAIR_PRESENT)) continue;
        fold_pair(ps, s, q, k1, sends - k1, 0);
        ps.stale[q] = 1;
    }
}

// Fold of pending counts (gsx_prop_fold_credits; GSX_CREDIT_NOW folds in k_prop_count).
// The counts are left empty: only the nonzero ones are rewritten (no full clears).
__global__ __launch_bounds__(256) void k_prop_fold(PropState ps, DevState s, uint32_t* __restrict__ first,
                                                   uint32_t* __restrict__ dup) {
    const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= s.n_pairs) return;
    const uint32_t k1 = first[q];
    const uint32_t k2 = dup[q];
    const uint32_t k4 = ps.invcnt ? ps.invcnt[q] : 0;
    if (k1 == 0 && k2 == 0 && k4 == 0) return;
    if (k1 | k2) {
        first[q] = 0;
        dup[q] = 0;
    }
    if (k4) ps.invcnt[q] = 0;
    if (!(s.pflags[q] & PAIR_PRESENT) || ps.topic >= s.n_topics) return;
    if (!s.tp[ps.topic].scored) return;
    fold_pair(ps, s, q, k1, k2, k4);
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

// Arrival hops, [message][node] as the ABI lays them out: the hop whose
// frontier row holds the message's bit (0 at the source), 0xFF never.
// Thread per (node, word): the hops of its new bits (hist rows where the node
// is occupied) spread over the code planes; sources and messages the node
// never got keep code 0 (only old copies of received messages are looked up).
// The node's occupied rows are found first (one occ word per row, shared by
// the node's threads), then their words are loaded VB at a time, so a thread
// waits for one load latency per VB rows instead of two per row.
__global__ __launch_bounds__(256) void k_prop_vcodes(PropState ps, uint64_t* __restrict__ vc, uint32_t n_planes) {
    constexpr int VB = 8;
    const uint32_t W = ps.n_words;
    const size_t plane = (size_t)ps.n_nodes * W;
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    const uint32_t rows = ps.n_rows < 64 ? ps.n_rows : 64;  // (hop 64, GSX_MAX_HOPS, apart below)
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < plane; i += (size_t)gridDim.x * 256u) {
        const uint32_t u = (uint32_t)(i / W);
        uint64_t rm = 0;  // bit h: the node is occupied at hop h
        for (uint32_t h = 1; h < rows; ++h) rm |= (uint64_t)occ_bit(ps.occ + (size_t)h * occ_row, u) << h;
        uint64_t pl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (ps.n_rows > 64 && occ_bit(ps.occ + (size_t)64 * occ_row, u)) pl[6] = ps.hist[(size_t)64 * plane + i];
        while (rm) {
            uint32_t hs[VB];
            uint64_t x[VB];
#pragma unroll
            for (int j = 0; j < VB; ++j) {
                hs[j] = rm ? (uint32_t)__builtin_ctzll(rm) : 0u;
                rm &= rm - 1;
            }
#pragma unroll
            for (int j = 0; j < VB; ++j) x[j] = hs[j] ? ps.hist[(size_t)hs[j] * plane + i] : 0ull;
#pragma unroll
            for (int j = 0; j < VB; ++j)
#pragma unroll
                for (uint32_t b = 0; b < 8; ++b)
                    if ((hs[j] >> b) & 1) pl[b] |= x[j];
        }
#pragma unroll
        for (uint32_t b = 0; b < 8; ++b)
            if (b < n_planes) vc[b * plane + i] = pl[b];
    }
}

__global__ __launch_bounds__(256) void k_prop_hops_export(PropState ps, uint8_t* __restrict__ out) {
    const uint32_t u = blockIdx.x * 256u + threadIdx.x;
    const uint32_t w = blockIdx.y;
    if (u >= ps.n_nodes) return;
    const uint32_t W = ps.n_words;
    uint8_t hk[64];
#pragma unroll
    for (int b = 0; b < 64; ++b) hk[b] = 0xFF;
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    for (uint32_t h = 0; h < ps.n_rows; ++h) {
        if (!occ_bit(ps.occ + (size_t)h * occ_row, u)) continue;  // untouched at hop h: empty row
        uint64_t x = ps.hist[(size_t)h * ps.n_nodes * W + (size_t)u * W + w];
        while (x) {
            const int b = __builtin_ctzll(x);
            x &= x - 1;
            hk[b] = (uint8_t)h;
        }
    }
    if (ps.drop && ps.drop[w]) {  // not forwarded, so not in the frontier rows: received at hop 1
        uint64_t x = ps.dseen[(size_t)u * W + w];
        while (x) {
            const int b = __builtin_ctzll(x);
            x &= x - 1;
            hk[b] = 1;
        }
    }
    for (int b = 0; b < 64; ++b) {
        const uint32_t k = w * 64 + b;
        if (k < ps.n_msgs) out[(size_t)k * ps.n_nodes + u] = hk[b];
    }
}

// Duplicate receipts per pair (DUPLICATE_MESSAGE, trace.go:136-164): bit m
// of row q = (u -> v) when v sent u a copy of m that u had already seen
// (pushMsg's seenMessage test, pubsub.go:1046-1060).  v sends m at hop h + 1
// when it forwarded m at hop h (frontier-history row h: published at h = 0,
// accepted first receipts otherwise) and the call ran that hop (h <
// max_hops), through the eligibility of its pair (v -> u) or RandomSub's
// draw, never back to the peer it first got m from (from_mask of (v -> u))
// nor to m's origin (u's row 0).  The copy that gave u the message is the
// one recorded in from_mask of q; every other copy is a duplicate.  A pair
// whose copies u's AcceptFrom drops has pin NO_PAIR: no trace, as in
// pubsub.go:1014-1017.
__global__ __launch_bounds__(256) void k_prop_dup_rows(PropState ps, uint64_t* __restrict__ out) {
    const uint32_t W = ps.n_words;
    const size_t occ_row = ((size_t)ps.n_nodes + 63) / 64;
    const uint32_t h_end = ps.n_rows < ps.max_hops ? ps.n_rows : ps.max_hops;  // rows forwarded in a hop that ran
    for (uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x; q < ps.n_pairs; q += (uint64_t)gridDim.x * 256u) {
        const uint32_t pn = ps.pin[q];
        const uint32_t r = ps.rev[q];
        const uint32_t u = ps.pair_obs[q];
        const uint32_t v = pn & PIN_NODE_MASK;
        const bool sends = pn != NO_PAIR && r != NO_PAIR;
        const uint8_t fw = sends ? (uint8_t)(pn >> PIN_FWD_SHIFT) : 0;
        for (uint32_t w = 0; w < W; ++w) {
            uint64_t d = 0;
            if (sends) {
                uint64_t fset = 0, own = 0;
                for (uint32_t h = 0; h < h_end; ++h) {
                    if (!occ_bit(ps.occ + (size_t)h * occ_row, v)) continue;
                    const uint64_t x = ps.hist[(size_t)h * ps.n_nodes * W + (size_t)v * W + w];
                    fset |= x;
                    if (h == 0) own = x;
                }
                uint64_t el = elig_word(fw, own);
                if (ps.sel) el |= ps.sel[(size_t)r * W + w];
                const uint64_t own_u = occ_bit(ps.occ, u) ? ps.hist[(size_t)u * W + w] : 0;
                d = fset & el & ~ps.from_mask[(size_t)r * W + w] & ~own_u & ~ps.from_mask[q * W + w];
            }
            out[q * W + w] = d;
        }
    }
}
hipError_t launch_prop_dup_rows(const PropState& ps, uint64_t* out, hipStream_t st) {
    if (ps.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_dup_rows, dim3((unsigned)std::min<uint64_t>((ps.n_pairs + 255) / 256, 4096)), dim3(256), 0,
                       st, ps, out);
    return hipGetLastError();
}

// After a call with dropped messages: keep their hop-1 receipts for
// gsx_prop_results, and (gossipsub) take them out of the seen rows the
// message cache keeps, since Publish Puts only what a node processed
// (gossipsub.go:944): a dropped message stays in its source's row only.
__global__ __launch_bounds__(256) void k_prop_uncache(PropState ps, bool mask_cache) {
    const uint32_t W = ps.n_words;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < (uint64_t)ps.n_nodes * W; i += (uint64_t)gridDim.x * 256u) {
        const uint32_t w = (uint32_t)(i % W);
        const uint64_t d = ps.drop[w];
        const uint32_t u = (uint32_t)(i / W);
        const uint64_t rx = d & ps.seen[i] & ~(occ_bit(ps.occ, u) ? ps.origin[i] : 0ull);  // origin rows: sources only
        ps.dseen[i] = rx;
        if (mask_cache && rx) ps.seen[i] &= ~rx;
    }
}
hipError_t launch_prop_uncache(const PropState& ps, bool mask_cache, hipStream_t st) {
    if (!ps.drop || ps.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_uncache, dim3(std::min((unsigned)(((uint64_t)ps.n_nodes * ps.n_words + 255) / 256), COUNTER_GRID)),
                       dim3(256), 0, st, ps, mask_cache);
    return hipGetLastError();
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
    hipLaunchKernelGGL(k_prop_hops_export, dim3(nblk(ps.n_nodes, 256), ps.n_words), dim3(256), 0, st, ps, hop_mn);
    return hipGetLastError();
}
hipError_t launch_prop_vcodes(const PropState& ps, uint64_t* vc, uint32_t n_planes, hipStream_t st) {
    const uint64_t n = (uint64_t)ps.n_nodes * ps.n_words;
    if (n == 0 || n_planes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_vcodes, dim3(std::min<uint64_t>((n + 255) / 256, 16384)), dim3(256), 0, st, ps, vc,
                       n_planes);
    return hipGetLastError();
}
hipError_t launch_prop_fwd(const PropState& ps, const DevState& s, hipStream_t st, bool pins_only, bool compact) {
    if (s.n_pairs == 0) return hipSuccess;
    if (!pins_only)
        hipLaunchKernelGGL(k_prop_fwd, dim3(std::min(nblk(s.n_pairs, 256), COUNTER_GRID)), dim3(256), 0, st, ps, s);
    hipLaunchKernelGGL(k_prop_pin, dim3(std::min(nblk(s.n_pairs, 256), 8192u)), dim3(256), 0, st, ps);
    if (!compact) return hipGetLastError();  // (the caller compacts once more pins are in: k_rep_fwd_recv)
    return launch_prop_compact(ps, st);
}
hipError_t launch_prop_compact(const PropState& ps, hipStream_t st) {
    if (ps.n_nodes) {
        hipLaunchKernelGGL(k_prop_compact, dim3(std::min(nblk(ps.n_nodes, 256), 4096u)), dim3(256), 0, st, ps);
        hipLaunchKernelGGL(k_prop_compact_done, dim3(std::min(nblk((ps.n_nodes + 63) / 64, 256), 1024u)), dim3(256), 0,
                           st, ps);
    }
    hipLaunchKernelGGL(k_prop_nchg_reset, dim3(1), dim3(1), 0, st, ps);
    return hipGetLastError();
}
hipError_t launch_prop_init(const PropState& ps, uint64_t* front, hipStream_t st) {
    if (ps.n_msgs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_zero_src, dim3(nblk((uint64_t)ps.n_msgs * ps.n_words, 256)), dim3(256), 0, st, ps, front);
    hipLaunchKernelGGL(k_prop_init, dim3(nblk(ps.n_msgs, 256)), dim3(256), 0, st, ps, front);
    return hipGetLastError();
}
hipError_t launch_prop_clear(const PropState& ps, bool clear_flast, bool clear_corr, hipStream_t st) {
    const size_t n = std::max<size_t>({(size_t)ps.n_words * ps.n_nodes, (size_t)ps.n_pairs, (size_t)STAT_WORDS});
    hipLaunchKernelGGL(k_prop_clear, dim3(std::min(nblk(n, 256), 8192u)), dim3(256), 0, st, ps, clear_flast ? 1u : 0u,
                       clear_corr ? 1u : 0u);
    return hipGetLastError();
}
hipError_t launch_rsub_select(const PropState& ps, const uint64_t* front, const uint64_t* front_occ, hipStream_t st) {
    if (ps.n_nodes == 0 || !ps.sel) return hipSuccess;
    hipLaunchKernelGGL(k_rsub_select, dim3(nblk(ps.n_nodes, 64)), dim3(64), 0, st, ps, front, front_occ);
    return hipGetLastError();
}
hipError_t launch_prop_pack(const PropState& ps, const uint64_t* front, const uint64_t* front_occ, uint64_t* send,
                            hipStream_t st) {
    if (ps.n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_pack, dim3(std::min(nblk(ps.n_send, 256), COUNTER_GRID)), dim3(256), 0, st, ps, front,
                       front_occ, send);
    return hipGetLastError();
}
hipError_t launch_prop_pack_compact(const PropState& ps, const uint64_t* front, const uint64_t* front_occ,
                                    uint64_t* out, unsigned long long* dcount, uint32_t* tab, hipStream_t st) {
    if (ps.n_send == 0 || ps.n_nodes == 0) return hipSuccess;
    const uint32_t nb = pack_blocks(ps.n_nodes);
    hipLaunchKernelGGL(k_pack_front<false>, dim3(nb), dim3(256), 0, st, ps, front, front_occ, tab, out);
    hipLaunchKernelGGL(k_pack_scan, dim3(ps.n_ranks), dim3(1024), 0, st, tab, nb, ps.n_ranks, dcount);
    hipLaunchKernelGGL(k_pack_front<true>, dim3(nb), dim3(256), 0, st, ps, front, front_occ, tab, out);
    return hipGetLastError();
}
uint32_t pack_table_words(uint32_t n_nodes, uint32_t n_ranks) { return pack_blocks(n_nodes) * n_ranks; }
// The compacted exchange's count words, device-side: out[d] = (entries for
// rank d, this rank's first receipts of its latest hop), so that one
// all-to-all tells every receiver both its entry count and whether the hop
// before delivered anything anywhere (no host round trip in between).
__global__ void k_pack_counts(const unsigned long long* __restrict__ dcount,
                              const unsigned long long* __restrict__ hop_new, uint32_t world, int64_t* __restrict__ out) {
    const uint32_t d = threadIdx.x;
    if (d >= world) return;
    out[2 * d] = dcount ? (int64_t)dcount[d] : 0;
    out[2 * d + 1] = hop_new ? (int64_t)*hop_new : 0;
}
hipError_t launch_pack_counts(const unsigned long long* dcount, const unsigned long long* hop_new, uint32_t world,
                              int64_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_pack_counts, dim3(1), dim3(MAX_RANKS), 0, st, dcount, hop_new, world, out);
    return hipGetLastError();
}
hipError_t launch_halo_scatter(const PropState& ps, uint64_t* halo, const uint64_t* ent, uint64_t n, uint32_t h,
                               hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_halo_scatter, dim3(std::min(nblk(n, 256), COUNTER_GRID)), dim3(256), 0, st, ps, halo, ent, n, h);
    return hipGetLastError();
}
template <bool DROP, int G, int R>
static void fast1_launch(const PropState& ps, uint32_t h, const uint64_t* front, uint64_t* nxt, hipStream_t st) {
    const dim3 g1(std::min(nblk(ps.n_nodes, 256 / G), COUNTER_GRID)), b(256);
    if (ps.rep) hipLaunchKernelGGL((k_prop_hop_fast1<DROP, G, R, 2>), g1, b, 0, st, ps, h, front, nxt);
    else if (ps.sharded) hipLaunchKernelGGL((k_prop_hop_fast1<DROP, G, R, 1>), g1, b, 0, st, ps, h, front, nxt);
    else hipLaunchKernelGGL((k_prop_hop_fast1<DROP, G, R, 0>), g1, b, 0, st, ps, h, front, nxt);
}
template <int CW, int LPN, bool DROP>
static void fast_launch(const PropState& ps, uint32_t h, const uint64_t* front, uint64_t* nxt, hipStream_t st) {
    const dim3 g(std::min(nblk(ps.n_nodes, 256 / LPN), COUNTER_GRID)), b(256);
    if (ps.rep) hipLaunchKernelGGL((k_prop_hop_fast<CW, LPN, DROP, 2>), g, b, 0, st, ps, h, front, nxt);
    else if (ps.sharded) hipLaunchKernelGGL((k_prop_hop_fast<CW, LPN, DROP, 1>), g, b, 0, st, ps, h, front, nxt);
    else hipLaunchKernelGGL((k_prop_hop_fast<CW, LPN, DROP, 0>), g, b, 0, st, ps, h, front, nxt);
}
bool hop_lean(const PropState& ps) {
    static const bool no_fast = getenv("GSX_HOP_GENERAL") != nullptr;  // tuning / cross-checks
    return !ps.sel && !ps.from_mask && ps.late && !no_fast;
}
template <int CW, int LPN>
static void hop_launch(const PropState& ps, uint32_t h, const uint64_t* front, uint64_t* nxt, hipStream_t st) {
    const dim3 g(std::min(nblk(ps.n_nodes, 256 / LPN), COUNTER_GRID)), b(256);
    static const bool no_fast1 = getenv("GSX_HOP_NO_FAST1") != nullptr;  // tuning / cross-checks
    // (range shards take the lean kernels too: SH = 1 reads remote rows from the
    // halo, SH = 2 from the replicated frontier rows)
    if (hop_lean(ps) && ps.n_words == 1 && !no_fast1) {
        static const int gv = [] {  // lanes per node x rounds (tuning): 42 (default), 41, 81, 22, 82
            const char* v = getenv("GSX_HOP_GR");
            return v ? atoi(v) : 42;
        }();
#define GSX_FAST1(GG, RR)                                          \
    {                                                              \
        if (ps.drop) fast1_launch<true, GG, RR>(ps, h, front, nxt, st); \
        else fast1_launch<false, GG, RR>(ps, h, front, nxt, st);   \
    }
        if (gv == 41) GSX_FAST1(4, 1)
        else if (gv == 81) GSX_FAST1(8, 1)
        else if (gv == 82) GSX_FAST1(8, 2)
        else if (gv == 22) GSX_FAST1(2, 2)
        else GSX_FAST1(4, 2)
#undef GSX_FAST1
    } else if (hop_lean(ps)) {
        if (ps.drop) fast_launch<CW, LPN, true>(ps, h, front, nxt, st);
        else fast_launch<CW, LPN, false>(ps, h, front, nxt, st);
    }
    else if (ps.from_mask) hipLaunchKernelGGL((k_prop_hop<CW, LPN, true>), g, b, 0, st, ps, h, front, nxt);
    else hipLaunchKernelGGL((k_prop_hop<CW, LPN, false>), g, b, 0, st, ps, h, front, nxt);
}
hipError_t launch_prop_hop(const PropState& ps, uint32_t h, const uint64_t* front, uint64_t* nxt, hipStream_t st) {
    if (ps.n_nodes == 0) return hipSuccess;
    // n_words is 1, 2 or a multiple of 4 (the engine pads).  Words per lane
    // CW (GSX_HOP_CW = 2 or 4 overrides, for tuning) and lanes per node: the
    // largest of 4, 2, 1 whose chunks tile the row.
    static const int cw_env = [] {
        const char* v = getenv("GSX_HOP_CW");
        return v ? atoi(v) : 0;
    }();
    const uint32_t W = ps.n_words;
    if (W == 1) hop_launch<1, 1>(ps, h, front, nxt, st);
    else if (W == 2) hop_launch<2, 1>(ps, h, front, nxt, st);
    else if (cw_env == 2) {
        if (W % 16 == 0) hop_launch<2, 8>(ps, h, front, nxt, st);
        else if (W % 8 == 0) hop_launch<2, 4>(ps, h, front, nxt, st);
        else hop_launch<2, 2>(ps, h, front, nxt, st);
    } else {
        if (W % 16 == 0) hop_launch<4, 4>(ps, h, front, nxt, st);
        else if (W % 8 == 0) hop_launch<4, 2>(ps, h, front, nxt, st);
        else hop_launch<4, 1>(ps, h, front, nxt, st);
    }
    return hipGetLastError();
}
hipError_t launch_rep_init(const PropState& ps, hipStream_t st) {
    if (ps.n_msgs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rep_zero_src, dim3(nblk((uint64_t)ps.n_msgs * ps.n_words, 256)), dim3(256), 0, st, ps);
    hipLaunchKernelGGL(k_rep_init, dim3(nblk(ps.n_msgs, 256)), dim3(256), 0, st, ps);
    return hipGetLastError();
}
hipError_t launch_rep_pack(const PropState& ps, uint32_t h, uint64_t* out, unsigned long long* cnt, hipStream_t st) {
    if (ps.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rep_pack, dim3(std::min(nblk(ps.n_nodes, 1024), 4096u)), dim3(256), 0, st, ps, h, out, cnt);
    return hipGetLastError();
}
hipError_t launch_rep_scatter(const PropState& ps, uint32_t h, const RepParts& parts, hipStream_t st) {
    const uint64_t n = parts.off[parts.n];
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rep_scatter, dim3(std::min(nblk(n, 256), COUNTER_GRID)), dim3(256), 0, st, ps, h, parts);
    return hipGetLastError();
}
hipError_t launch_rep_fwd_pack(const PropState& ps, uint8_t* out, hipStream_t st) {
    if (ps.n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rep_fwd_pack, dim3(std::min(nblk(ps.n_send, 256), COUNTER_GRID)), dim3(256), 0, st, ps, out);
    return hipGetLastError();
}
hipError_t launch_rep_fwd_recv(const PropState& ps, const uint8_t* in, hipStream_t st) {
    if (ps.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rep_fwd_recv, dim3(std::min(nblk(ps.n_pairs, 256), COUNTER_GRID)), dim3(256), 0, st, ps, in);
    return hipGetLastError();
}
hipError_t launch_rep_sends(const PropState& ps, uint32_t h_run, uint64_t* vcnt, uint64_t* out, hipStream_t st) {
    if (ps.n_send == 0) return hipSuccess;
    const dim3 gv(std::min(nblk(ps.n_nodes, 256), COUNTER_GRID));
    if (ps.n_nodes) hipLaunchKernelGGL(k_prop_vcount<1>, gv, dim3(256), 0, st, ps, h_run, vcnt, false);
    (void)hipMemsetAsync(out, 0, 8 * ps.n_send, st);  // (slots whose pair does not exist stay 0)
    hipLaunchKernelGGL(k_rep_sends, dim3(std::min(nblk(ps.n_pairs, 256), COUNTER_GRID)), dim3(256), 0, st, ps, h_run,
                       vcnt, out);
    return hipGetLastError();
}
hipError_t launch_rep_sends_recv(const PropState& ps, const uint64_t* in, hipStream_t st) {
    if (ps.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rep_sends_recv, dim3(std::min(nblk(ps.n_pairs, 256), COUNTER_GRID)), dim3(256), 0, st, ps, in);
    return hipGetLastError();
}
hipError_t launch_prop_mark(const PropState& ps, uint32_t h, const uint64_t* front_occ, hipStream_t st) {
    if (ps.n_nodes == 0) return hipSuccess;
    // (GSX_MARK_GRID: A/B of the grid; 256 / 512 / 1024 blocks measured slower
    // than 2048 at 64 messages, 1.79 / 1.64 / 1.53 vs 1.50 ms per batch)
    static const unsigned mark_grid = [] {
        const char* v = getenv("GSX_MARK_GRID");
        return v && atoi(v) > 0 ? (unsigned)atoi(v) : COUNTER_GRID;
    }();
    hipLaunchKernelGGL(k_prop_mark, dim3(std::min(nblk(ps.n_nodes, 256), mark_grid)), dim3(256), 0, st, ps, h, front_occ);
    return hipGetLastError();
}
hipError_t launch_prop_dups(const PropState& ps, uint32_t h_run, uint64_t* vcnt, bool gray_only, hipStream_t st) {
    if (ps.n_pairs == 0) return hipSuccess;
    const uint32_t W = ps.n_words;
    const int L = W % 64 == 0 ? 16 : W % 32 == 0 ? 8 : W % 16 == 0 ? 4 : W % 8 == 0 ? 2 : 1;
    const dim3 gv(std::min(nblk((uint64_t)ps.n_nodes * L, 256), COUNTER_GRID));
    if (L == 16) hipLaunchKernelGGL(k_prop_vcount<16>, gv, dim3(256), 0, st, ps, h_run, vcnt, gray_only);
    else if (L == 8) hipLaunchKernelGGL(k_prop_vcount<8>, gv, dim3(256), 0, st, ps, h_run, vcnt, gray_only);
    else if (L == 4) hipLaunchKernelGGL(k_prop_vcount<4>, gv, dim3(256), 0, st, ps, h_run, vcnt, gray_only);
    else if (L == 2) hipLaunchKernelGGL(k_prop_vcount<2>, gv, dim3(256), 0, st, ps, h_run, vcnt, gray_only);
    else hipLaunchKernelGGL(k_prop_vcount<1>, gv, dim3(256), 0, st, ps, h_run, vcnt, gray_only);
    const dim3 gd(std::min(nblk(ps.n_pairs, 256), COUNTER_GRID));
    // A/B: GSX_DUPS_DU (pairs per thread batch: 1, 2 or 4) and GSX_DUPS_GRID (block cap)
    static const int dd = [] {
        const char* v = getenv("GSX_DUPS_DU");
        return v ? atoi(v) : DU;
    }();
    static const unsigned dgrid = [] {
        const char* v = getenv("GSX_DUPS_GRID");
        return v && atoi(v) > 0 ? (unsigned)atoi(v) : COUNTER_GRID;
    }();
    const dim3 gdd(std::min(nblk(ps.n_pairs, 256), dgrid));
    if (gray_only) hipLaunchKernelGGL(k_prop_dups<true>, gd, dim3(256), 0, st, ps, h_run, vcnt);
    else if (dd == 1) hipLaunchKernelGGL((k_prop_dups<false, 1>), gdd, dim3(256), 0, st, ps, h_run, vcnt);
    else if (dd == 2) hipLaunchKernelGGL((k_prop_dups<false, 2>), gdd, dim3(256), 0, st, ps, h_run, vcnt);
    else hipLaunchKernelGGL((k_prop_dups<false, 4>), gdd, dim3(256), 0, st, ps, h_run, vcnt);
    return hipGetLastError();
}
hipError_t launch_prop_count(const PropState& ps, const DevState& s, bool fold, bool rescore, const DevPeerParams& pp,
                             hipStream_t st) {
    if (ps.n_pairs == 0) return hipSuccess;
    const dim3 g(std::min(nblk(ps.n_pairs, 256), COUNTER_GRID)), b(256);
    if (fold && rescore && s.n_topics == 1) hipLaunchKernelGGL((k_prop_count<true, true, true>), g, b, 0, st, ps, s, pp);
    else if (fold && rescore) hipLaunchKernelGGL((k_prop_count<true, true>), g, b, 0, st, ps, s, pp);
    else if (fold) hipLaunchKernelGGL((k_prop_count<true, false>), g, b, 0, st, ps, s, pp);
    else hipLaunchKernelGGL((k_prop_count<false, false>), g, b, 0, st, ps, s, pp);
    return hipGetLastError();
}
hipError_t launch_prop_defer(const PropState& ps, const DevState& s, const DevPeerParams& pp, hipStream_t st) {
    if (ps.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_defer, dim3(std::min(nblk(ps.n_pairs, 256), COUNTER_GRID)), dim3(256), 0, st, ps, s, pp);
    return hipGetLastError();
}
hipError_t launch_prop_fold_acc(const PropState& ps, const DevState& s, hipStream_t st) {
    if (ps.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_fold_acc, dim3(std::min(nblk(ps.n_pairs, 256), 8192u)), dim3(256), 0, st, ps, s);
    return hipGetLastError();
}
hipError_t launch_prop_fold(const PropState& ps, const DevState& s, uint32_t* first, uint32_t* dup,
                            hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prop_fold, dim3(nblk(s.n_pairs, 256)), dim3(256), 0, st, ps, s, first, dup);
    return hipGetLastError();
}

}  // namespace gsx
