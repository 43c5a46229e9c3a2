// gsx_heartbeat.hip — the GossipSub heartbeat's mesh maintenance and IHAVE
// gossip as one synchronous round over the whole overlay (gsx.h,
// gsx_heartbeat).
//
//  (A) per topic t ascending:
//      k_hb_mesh — one lane per node v: the mesh maintenance of (v, t)
//        (gossipsub.go:1344-1510).  Everything it touches — the records,
//        backoff entries and control bits of v's own pairs for topic t —
//        belongs to it alone.  Mesh and candidate lists are <= HB_MAX_DEG u16
//        offsets in scratch.
//      k_hb_gossip — one lane per node: emitGossip (:1669-1723).  The IHAVE
//        list is the node's GetGossipIDs set (mcache.go:82-92) read straight
//        from the cached batches' seen words; its order is never observable
//        (handleIHave collects ids into a map, :641-650), so an untruncated
//        list is reported by its length and multiset digest and its shuffle
//        only advances the draw stream.  Nodes whose list exceeds
//        MaxIHaveLength (per-target reshuffle + truncation, :1708-1716) are
//        queued for k_hb_gossip_long, one wave per node with the list in LDS.
//  (B) k_hb_recv: one lane per receiving node u, senders in ascending order
//      (the Dhi check reads the mesh size the previous accepts left):
//      handleGraft / handlePrune, :718-843, AcceptFrom-gated (:582-593).
//  (C) k_hb_answer: one lane per pair, the GRAFT senders' handlePrune of the
//      PRUNE answers.
// Control messages are per-pair topic bitmasks (bit t of a u64), so a
// receiver reads one word per sender.  Round counters are summed per wave
// before one atomic each.  Integer/byte work with scattered reads of the
// per-pair score cache: latency-bound, no MFMA/LDS tiling applies.
#include "gsx_ops.h"

namespace gsx {

constexpr uint64_t TAG_HEARTBEAT = 8;

__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// Sums a per-lane counter over the wave; lane 0 adds it to the round total.
// Every lane of the wave must call it.
__device__ __forceinline__ void flush_count(unsigned long long* stats, int k, uint64_t c) {
    c = wave_sum64(c);
    if ((threadIdx.x % 64) == 0 && c) atomicAdd(&stats[k], (unsigned long long)c);
}

__device__ __forceinline__ bool hb_in_mesh(const DevState& s, uint64_t r, uint32_t t) {
    return (s.pflags[r] & PAIR_PRESENT) && (s.rflags[flag_index(r, t, s.n_topics)] & REC_IN_MESH);
}

// addBackoff / doAddBackoff, gossipsub.go:845-859 (0 = no entry; the zero
// time is before every expiry)
__device__ __forceinline__ void add_backoff(const HbState& h, uint64_t r, uint32_t t, int64_t interval) {
    int64_t* b = &h.backoff[(size_t)t * h.n_pairs + r];
    const int64_t expire = h.now + interval;
    if (*b == 0 || *b < expire) *b = expire;
}

// clearBackoff, gossipsub.go:1585-1604
__global__ __launch_bounds__(256) void k_hb_clear_backoff(HbState h, uint64_t n) {
    uint64_t cleared = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const int64_t b = h.backoff[i];
        if (b != 0 && b + 2 * HEARTBEAT_INTERVAL_NS < h.now) {
            h.backoff[i] = 0;
            ++cleared;
        }
    }
    flush_count(h.stats, HB_BACKOFF_CLEARED, cleared);
}

struct HbUnit {
    const DevState& s;
    const HbState& h;
    uint32_t t;
    int64_t r0;  // first pair of the row
    int deg;
    uint64_t grafts = 0, prunes = 0;

    __device__ bool in_mesh(int i) const { return hb_in_mesh(s, r0 + i, t); }
    __device__ uint8_t ef(int i) const { return h.eflags[r0 + i]; }
    __device__ double score(int i) const { return s.score[r0 + i]; }

    __device__ int mesh_list(uint16_t* out) const {
        int n = 0;
        for (int i = 0; i < deg; ++i)
            if (in_mesh(i)) out[n++] = (uint16_t)i;
        return n;
    }

    // getPeers, gossipsub.go:1852-1872: mesh-capable topic peers passing the
    // filter, ascending, shuffled, truncated to count.  score_cmp 0: score >=
    // ref, 1: score > ref.
    __device__ int get_peers(int count_max, bool outbound_only, int score_cmp, double ref, uint16_t* out,
                             Rng& g) const {
        int n = 0;
        for (int i = 0; i < deg; ++i) {
            const uint64_t r = r0 + i;
            if ((s.pflags[r] & (PAIR_PRESENT | PAIR_CONNECTED)) != (PAIR_PRESENT | PAIR_CONNECTED)) continue;
            const uint8_t f = ef(i);
            if (!(f & EDGE_GOSSIPSUB)) continue;
            if (in_mesh(i)) continue;
            if (h.backoff[(size_t)t * h.n_pairs + r] != 0) continue;  // map presence (:1377)
            if (f & EDGE_DIRECT) continue;
            if (outbound_only && !(f & EDGE_OUTBOUND)) continue;
            const double sc = score(i);
            if (score_cmp == 0 && !(sc >= ref)) continue;
            if (score_cmp == 1 && !(sc > ref)) continue;
            out[n++] = (uint16_t)i;
        }
        g.shuffle(out, n);
        if (count_max > 0 && n > count_max) n = count_max;
        return n;
    }

    // the receiver's pair (u -> v) of r = (v -> u) has control to read in (B)
    __device__ void mark_inbox(uint64_t r) const {
        const uint32_t q = h.rev[r];
        if (q != NO_PAIR && !(q & HALO)) h.inbox[q] = 1;
    }
    __device__ void graft(int i) {  // graftPeer, :1353-1359
        const uint64_t r = r0 + i;
        ev_graft(s, r, t, h.now);
        h.ctl_graft[r] |= 1ull << t;
        h.dirty[r] = 1;
        mark_inbox(r);
        ++grafts;
    }
    __device__ void prune(int i) {  // prunePeer, :1345-1351
        const uint64_t r = r0 + i;
        ev_prune(s, r, t);
        add_backoff(h, r, t, h.gp.prune_backoff_ns);
        h.ctl_prune[r] |= 1ull << t;
        h.dirty[r] = 1;
        mark_inbox(r);
        ++prunes;
    }

    // stable insertion sort by cached score
    __device__ void sort_by_score(uint16_t* a, int n, bool desc) const {
        for (int i = 1; i < n; ++i) {
            const uint16_t x = a[i];
            const double sx = score(x);
            int j = i - 1;
            while (j >= 0 && (desc ? score(a[j]) < sx : score(a[j]) > sx)) {
                a[j + 1] = a[j];
                --j;
            }
            a[j + 1] = x;
        }
    }

    __device__ static void rotate(uint16_t* a, int i) {  // :1411-1418
        const uint16_t p = a[i];
        for (int j = i; j > 0; --j) a[j] = a[j - 1];
        a[0] = p;
    }

    __device__ void maintain(Rng& g) {
        const DevGossipParams& gp = h.gp;
        uint16_t plst[HB_MAX_DEG], tmp[HB_MAX_DEG];
        // drop all peers with negative score, without PX (:1361-1368)
        int n = mesh_list(plst);
        for (int i = 0; i < n; ++i)
            if (score(plst[i]) < 0) prune(plst[i]);
        // do we have enough peers? (:1370-1385)
        n = mesh_list(plst);
        if (n < gp.d_lo) {
            const int k = get_peers(gp.d - n, false, 0, 0.0, tmp, g);
            for (int i = 0; i < k; ++i) graft(tmp[i]);
        }
        // do we have too many peers? (:1387-1448)
        n = mesh_list(plst);
        if (n > gp.d_hi) {
            g.shuffle(plst, n);
            sort_by_score(plst, n, true);
            g.shuffle(plst + gp.d_score, n - gp.d_score);
            int outbound = 0;
            for (int i = 0; i < gp.d; ++i)
                if (ef(plst[i]) & EDGE_OUTBOUND) ++outbound;
            if (outbound < gp.d_out) {
                if (outbound > 0) {
                    int ihave = outbound;
                    for (int i = 1; i < gp.d && ihave > 0; ++i)
                        if (ef(plst[i]) & EDGE_OUTBOUND) {
                            rotate(plst, i);
                            --ihave;
                        }
                }
                int ineed = gp.d_out - outbound;
                for (int i = gp.d; i < n && ineed > 0; ++i)
                    if (ef(plst[i]) & EDGE_OUTBOUND) {
                        rotate(plst, i);
                        --ineed;
                    }
            }
            for (int i = gp.d; i < n; ++i) prune(plst[i]);
        }
        // do we have enough outbound peers? (:1450-1476)
        n = mesh_list(plst);
        if (n >= gp.d_lo) {
            int outbound = 0;
            for (int i = 0; i < n; ++i)
                if (ef(plst[i]) & EDGE_OUTBOUND) ++outbound;
            if (outbound < gp.d_out) {
                const int k = get_peers(gp.d_out - outbound, true, 0, 0.0, tmp, g);
                for (int i = 0; i < k; ++i) graft(tmp[i]);
            }
        }
        // opportunistic grafting (:1478-1510)
        n = mesh_list(plst);
        if (gp.og_ticks && h.tick % gp.og_ticks == 0 && n > 1) {
            sort_by_score(plst, n, false);
            const double median = score(plst[n / 2]);
            if (median < h.og_threshold) {
                const int k = get_peers(gp.og_peers, false, 1, median, tmp, g);
                for (int i = 0; i < k; ++i) graft(tmp[i]);
            }
        }
    }
};

// Draws are keyed by the GLOBAL node id, so a range shard draws what the
// whole-overlay engine draws for the same node.
__device__ __forceinline__ Rng hb_rng(const HbState& h, uint32_t v, uint32_t t, uint32_t k) {
    return Rng{h.seed, TAG_HEARTBEAT, (uint64_t)h.node_lo + v, (h.tick << 32) | ((uint64_t)t << 24), k};
}

// One launch per topic, ascending: the maintenance of (v, t) for every v.
// A wave takes 64 consecutive nodes.  One pass over their pairs — coalesced,
// lane j reading pairs j, j + 64, ... of the wave's contiguous pair range,
// counted into the owner's LDS slot — decides whether any step of
// maintain() acts (a steady mesh: no negative score, Dlo <= |mesh| <= Dhi,
// enough outbound peers, not an opportunistic-graft tick); such a unit draws
// nothing and is done.  A graft step with no candidate (getPeers over an
// empty list) draws nothing either.  Lanes whose unit acts then run
// maintain() over their own row.
__global__ __launch_bounds__(64) void k_hb_mesh(DevState s, HbState h, uint32_t t) {
    __shared__ int64_t rs[65];    // row starts of the wave's nodes, rs[nv] = end
    __shared__ int cnt[5][64];    // per node: |mesh|, negative, outbound in mesh, candidates, outbound candidates
    uint64_t grafts = 0, prunes = 0;
    const DevGossipParams& gp = h.gp;
    const bool og_tick = gp.og_ticks && h.tick % gp.og_ticks == 0;
    const uint32_t lane = threadIdx.x;
    for (uint32_t v0 = blockIdx.x * 64u; v0 < h.n_nodes; v0 += gridDim.x * 64u) {
        const uint32_t nv = min(64u, h.n_nodes - v0);
        rs[lane] = h.row_ptr[v0 + min(lane, nv)];
        if (lane == 0) rs[64] = h.row_ptr[v0 + nv];
#pragma unroll
        for (int k = 0; k < 5; ++k) cnt[k][lane] = 0;
        __syncthreads();
        const int64_t pa = rs[0], pb = rs[64];
        for (int64_t r = pa + lane; r < pb; r += 64) {
            int lo = 0, hi = (int)nv;  // owner: rs[lo] <= r < rs[lo + 1]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (rs[mid] <= r) lo = mid;
                else hi = mid;
            }
            const uint8_t f = h.eflags[r];
            const uint8_t pf = s.pflags[r];
            if ((pf & PAIR_PRESENT) && (s.rflags[flag_index(r, t, s.n_topics)] & REC_IN_MESH)) {
                atomicAdd(&cnt[0][lo], 1);
                if (s.score[r] < 0) atomicAdd(&cnt[1][lo], 1);
                if (f & EDGE_OUTBOUND) atomicAdd(&cnt[2][lo], 1);
            } else if ((pf & (PAIR_PRESENT | PAIR_CONNECTED)) == (PAIR_PRESENT | PAIR_CONNECTED) &&
                       (f & EDGE_GOSSIPSUB) && !(f & EDGE_DIRECT) && h.backoff[(size_t)t * h.n_pairs + r] == 0 &&
                       s.score[r] >= 0.0) {  // getPeers' filter of the graft steps (:1370-1385, :1450-1476)
                atomicAdd(&cnt[3][lo], 1);
                if (f & EDGE_OUTBOUND) atomicAdd(&cnt[4][lo], 1);
            }
        }
        __syncthreads();
        if (lane < nv) {
            const uint32_t v = v0 + lane;
            const int n = cnt[0][lane], neg = cnt[1][lane], outb = cnt[2][lane];
            const int cand = cnt[3][lane], cand_out = cnt[4][lane];
            const bool grow = n < gp.d_lo && cand > 0;                               // :1370-1385
            const bool outbound = n >= gp.d_lo && outb < gp.d_out && cand_out > 0;  // :1450-1476
            if (!neg && n <= gp.d_hi && !grow && !outbound && !(og_tick && n > 1)) {
                h.rngk[v] = 0;
            } else {
                const int64_t r0 = rs[lane];
                HbUnit U{s, h, t, r0, (int)(rs[lane + 1] - r0)};
                Rng g = hb_rng(h, v, t, 0);
                U.maintain(g);
                h.rngk[v] = g.k;  // emitGossip continues this (node, topic) draw stream
                grafts += U.grafts;
                prunes += U.prunes;
            }
        }
        __syncthreads();  // rs / cnt are rewritten by the next wave-tile
    }
    flush_count(h.stats, HB_GRAFTS, grafts);
    flush_count(h.stats, HB_PRUNES, prunes);
}

// ---- emitGossip (gossipsub.go:1669-1723) --------------------------------------

// The live score of emitGossip (:1692): the heartbeat-start cache, except for
// pairs the node's maintenance of topics <= t has grafted or pruned.
__device__ __forceinline__ double live_score(const DevState& s, const HbState& h, uint64_t r) {
    return h.dirty[r] ? eval_pair(s, h.pp, r) : s.score[r];
}

// Eligible targets of (v, t), ascending: topic peers with the mesh feature,
// not in the mesh, not direct, live score >= GossipThreshold.
__device__ __forceinline__ bool gossip_target(const DevState& s, const HbState& h, uint64_t r, uint32_t t) {
    const uint8_t f = h.eflags[r];
    return (s.pflags[r] & (PAIR_PRESENT | PAIR_CONNECTED)) == (PAIR_PRESENT | PAIR_CONNECTED) &&
           (f & EDGE_GOSSIPSUB) && !(f & EDGE_DIRECT) && !hb_in_mesh(s, r, t) &&
           live_score(s, h, r) >= h.gossip_threshold;
}

__global__ __launch_bounds__(64) void k_hb_gossip(DevState s, HbState h, uint32_t t, const GossipBatch* __restrict__ gb,
                                                  uint32_t n_gb) {
    uint64_t msgs = 0, ids = 0;
    for (uint32_t v = blockIdx.x * 64u + threadIdx.x; v < h.n_nodes; v += gridDim.x * 64u) {
        // GetGossipIDs of (v, t): its length and multiset digest
        uint32_t L = 0;
        uint64_t dig = 0;
        for (uint32_t b = 0; b < n_gb; ++b) {
            const GossipBatch B = gb[b];
            for (uint32_t w = 0; w < B.n_words; ++w) {
                uint64_t word = B.seen[(size_t)v * B.n_words + w];
                L += (uint32_t)__popcll(word);
                // a node holding every message of the word (the common case once a
                // batch has spread) adds the word's precomputed digest sum
                const uint32_t left = B.n_msgs > w * 64 ? B.n_msgs - w * 64 : 0;
                const uint64_t full = left >= 64 ? ~0ull : ((1ull << left) - 1);
                if (word && word == full) {
                    dig += h.mc_digest[B.wdig_base + w];
                    continue;
                }
                while (word) {
                    dig += h.mc_digest[B.slot_base + w * 64 + (uint32_t)__builtin_ctzll(word)];
                    word &= word - 1;
                }
            }
        }
        if (L > 0) {  // emitGossip returns early on an empty list, drawing nothing
            const int64_t r0 = h.row_ptr[v];
            const int deg = (int)(h.row_ptr[v + 1] - r0);
            uint16_t peers[HB_MAX_DEG];
            int np = 0;
            for (int i = 0; i < deg; ++i)
                if (gossip_target(s, h, r0 + i, t)) peers[np++] = (uint16_t)i;
            int target = h.gp.d_lazy;
            const int factor = (int)(h.gp.gossip_factor * (double)np);
            if (factor > target) target = factor;
            const bool shuffle_peers = target <= np;
            if (!shuffle_peers) target = np;
            if (target > 0 && L > (uint32_t)h.gp.max_ihave) {
                h.long_nodes[atomicAdd(h.n_long, 1u)] = v;  // per-target truncation: k_hb_gossip_long
            } else if (target > 0) {
                if (shuffle_peers) {  // an untruncated list is not shuffled (its order is never observable)
                    Rng g = hb_rng(h, v, t, h.rngk[v]);
                    g.shuffle(peers, np);
                }
                for (int p = 0; p < target; ++p) {
                    const size_t x = (size_t)t * h.n_pairs + r0 + peers[p];
                    h.ihave_len[x] = L;
                    h.ihave_hash[x] = dig;
                }
                msgs += (uint64_t)target;
                ids += (uint64_t)target * L;
            }
        }
    }
    flush_count(h.stats, HB_IHAVE_MSGS, msgs);
    flush_count(h.stats, HB_IHAVE_IDS, ids);
}

// ---- lists longer than MaxIHaveLength: one wave per queued node -------------

__device__ __forceinline__ uint32_t wave_prefix(uint32_t x, uint32_t lane) {  // exclusive
    uint32_t incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += y;
    }
    return incl - x;
}

// shuffleStrings of a[0..L) in LDS; g is wave-uniform.  64 Int31s are drawn
// at once (one per lane, Go's rejection rule resolved by a ballot); lane 0
// applies the swaps in order.
__device__ void wave_shuffle(uint32_t* a, uint32_t L, Rng& g, int32_t* jbuf, uint32_t lane) {
    uint32_t i = 0;
    while (i < L) {
        const uint32_t step = i + lane;
        const bool valid = step < L;
        const uint32_t n = step + 1;
        const int32_t x = (int32_t)(h4(g.seed, g.tag, g.vertex, g.base | (g.k + lane)) >> 33);
        const bool pow2 = (n & (n - 1)) == 0;
        const int32_t maxv = pow2 ? 0 : (int32_t)((1u << 31) - 1 - (1u << 31) % n);
        const bool rej = valid && !pow2 && x > maxv;
        const uint64_t rb = __ballot(rej);
        const uint32_t l0 = rb ? (uint32_t)__builtin_ctzll(rb) : 64u;
        const uint32_t nvalid = l0 < L - i ? l0 : L - i;
        if (lane < nvalid) jbuf[lane] = pow2 ? (x & (int32_t)(n - 1)) : (x % (int32_t)n);
        __syncthreads();
        if (lane == 0)
            for (uint32_t k = 0; k < nvalid; ++k) {
                const uint32_t j = (uint32_t)jbuf[k];
                const uint32_t tmp = a[i + k];
                a[i + k] = a[j];
                a[j] = tmp;
            }
        __syncthreads();
        if (l0 < 64) {  // step i + l0 redraws after its rejected draw
            i += l0;
            g.k += l0 + 1;
        } else {
            i += nvalid;
            g.k += nvalid;
        }
    }
}

__global__ __launch_bounds__(64) void k_hb_gossip_long(DevState s, HbState h, uint32_t t,
                                                       const GossipBatch* __restrict__ gb, uint32_t n_gb) {
    extern __shared__ uint32_t mids[];  // message slots, GetGossipIDs order
    __shared__ uint16_t peers[HB_MAX_DEG];
    __shared__ int32_t jbuf[64];
    __shared__ uint32_t kshare;
    const uint32_t lane = threadIdx.x;
    const uint32_t n_long = *h.n_long;
    uint64_t msgs = 0, ids = 0;
    for (uint32_t li = blockIdx.x; li < n_long; li += gridDim.x) {
        const uint32_t v = h.long_nodes[li];
        // GetGossipIDs: windows newest first, batches in Put order, ids ascending
        uint32_t L = 0;
        for (uint32_t b = 0; b < n_gb; ++b) {
            const GossipBatch B = gb[b];
            for (uint32_t w0 = 0; w0 < B.n_words; w0 += 64) {
                const uint32_t w = w0 + lane;
                uint64_t word = w < B.n_words ? B.seen[(size_t)v * B.n_words + w] : 0;
                const uint32_t c = (uint32_t)__popcll(word);
                uint32_t pos = L + wave_prefix(c, lane);
                while (word) {
                    mids[pos++] = B.slot_base + w * 64 + (uint32_t)__builtin_ctzll(word);
                    word &= word - 1;
                }
                L = __shfl(pos, 63, 64);  // lane 63's end = the new total
            }
        }
        __syncthreads();
        Rng g = hb_rng(h, v, t, h.rngk[v]);
        wave_shuffle(mids, L, g, jbuf, lane);
        const int64_t r0 = h.row_ptr[v];
        const int deg = (int)(h.row_ptr[v + 1] - r0);
        int np = 0;
        for (int c0 = 0; c0 < deg; c0 += 64) {
            const int i = c0 + (int)lane;
            const bool ok = i < deg && gossip_target(s, h, r0 + i, t);
            const uint64_t bal = __ballot(ok);
            if (ok) peers[np + __popcll(bal & ((1ull << lane) - 1))] = (uint16_t)i;
            np += __popcll(bal);
        }
        __syncthreads();
        int target = h.gp.d_lazy;
        const int factor = (int)(h.gp.gossip_factor * (double)np);
        if (factor > target) target = factor;
        if (target > np) {
            target = np;
        } else {
            if (lane == 0) {
                g.shuffle(peers, np);
                kshare = g.k;
            }
            __syncthreads();
            g.k = kshare;
        }
        const uint32_t len = (uint32_t)h.gp.max_ihave;  // L > MaxIHaveLength here
        for (int p = 0; p < target; ++p) {
            wave_shuffle(mids, L, g, jbuf, lane);
            uint64_t d = 0;
            for (uint32_t e = lane; e < len; e += 64) d += h.mc_digest[mids[e]];
            d = wave_sum64(d);
            if (lane == 0) {
                const size_t x = (size_t)t * h.n_pairs + r0 + peers[p];
                h.ihave_len[x] = len;
                h.ihave_hash[x] = d;
            }
        }
        if (lane == 0) {
            msgs += (uint64_t)target;
            ids += (uint64_t)target * len;
        }
        __syncthreads();
    }
    flush_count(h.stats, HB_IHAVE_MSGS, msgs);
    flush_count(h.stats, HB_IHAVE_IDS, ids);
}

// ---- (B) receivers -------------------------------------------------------------

// handlePrune at the owner of pair q for topic t (:811-843): the tracer's
// Prune, then the PRUNE's backoff, which travels in whole seconds (:1821).
__device__ __forceinline__ void handle_prune(const DevState& s, const HbState& h, uint64_t q, uint32_t t) {
    ev_prune(s, q, t);
    const int64_t secs = h.gp.prune_backoff_ns / 1000000000LL;
    add_backoff(h, q, t, secs > 0 ? secs * 1000000000LL : h.gp.prune_backoff_ns);
}

__global__ __launch_bounds__(64) void k_hb_recv(DevState s, HbState h) {
    uint64_t accepted = 0, rejected = 0, penalties = 0, handled = 0;
    for (uint32_t u = blockIdx.x * 64u + threadIdx.x; u < h.n_nodes; u += gridDim.x * 64u) {
        const int64_t r0 = h.row_ptr[u], r1 = h.row_ptr[u + 1];
        const DevGossipParams& gp = h.gp;
        for (int64_t q = r0; q < r1; ++q) {  // q = (u -> v), ascending v
            // unsharded, only pairs whose sender marked them carry control;
            // what is read is cleared (the next round starts from zeros)
            if (!h.halo_ctl) {
                if (!h.inbox[q]) continue;
                h.inbox[q] = 0;
            }
            const uint32_t r = h.rev[q];  // r = (v -> u), the sender's pair
            if (r == NO_PAIR) continue;
            uint64_t grafts, prunes;
            if (r & HALO) {  // v on another shard: its control bits came through the exchange
                grafts = h.halo_ctl[2 * (size_t)(r & ~HALO)];
                prunes = h.halo_ctl[2 * (size_t)(r & ~HALO) + 1];
            } else {
                grafts = h.ctl_graft[r];
                prunes = h.ctl_prune[r];
                if (!h.halo_ctl) h.ctl_graft[r] = h.ctl_prune[r] = 0;
            }
            if (!(grafts | prunes)) continue;
            const double score = s.score[q];  // gs.score.Score(p) once per control message
            const uint8_t ef = h.eflags[q];
            // AcceptFrom (gossipsub.go:582-593): a graylisted non-direct sender's RPC is dropped
            if (!(ef & EDGE_DIRECT) && score < h.graylist) continue;
            h.dirty[q] = 1;  // its record may change below: its score is re-evaluated after (B)
            uint64_t resp = 0;
            for (; grafts; grafts &= grafts - 1) {  // handleGraft, :718-809, topics ascending
                const uint32_t t = (uint32_t)__builtin_ctzll(grafts);
                if (hb_in_mesh(s, q, t)) continue;
                if (ef & EDGE_DIRECT) {
                    resp |= 1ull << t;
                    ++rejected;
                    continue;
                }
                const int64_t expire = h.backoff[(size_t)t * h.n_pairs + q];
                if (expire != 0 && h.now < expire) {
                    ev_penalty(s, q, 1);
                    ++penalties;
                    if (h.now < expire + (gp.graft_flood_threshold_ns - gp.prune_backoff_ns)) {
                        ev_penalty(s, q, 1);
                        ++penalties;
                    }
                    add_backoff(h, q, t, gp.prune_backoff_ns);
                    resp |= 1ull << t;
                    ++rejected;
                    continue;
                }
                if (score < 0) {
                    resp |= 1ull << t;
                    add_backoff(h, q, t, gp.prune_backoff_ns);
                    ++rejected;
                    continue;
                }
                int n = 0;
                for (int64_t x = r0; x < r1; ++x) n += hb_in_mesh(s, x, t);
                if (n >= gp.d_hi && !(ef & EDGE_OUTBOUND)) {
                    resp |= 1ull << t;
                    add_backoff(h, q, t, gp.prune_backoff_ns);
                    ++rejected;
                    continue;
                }
                ev_graft(s, q, t, h.now);
                ++accepted;
            }
            h.resp[q] = resp;
            if (resp && !(r & HALO)) h.answer[r] = 1;  // the GRAFT sender has an answer to read in (C)
            for (; prunes; prunes &= prunes - 1) {  // handlePrune
                handle_prune(s, h, q, (uint32_t)__builtin_ctzll(prunes));
                ++handled;
            }
        }
    }
    flush_count(h.stats, HB_ACCEPTED, accepted);
    flush_count(h.stats, HB_REJECTED, rejected);
    flush_count(h.stats, HB_PENALTIES, penalties);
    flush_count(h.stats, HB_PRUNES_HANDLED, handled);
}

// ---- (C) the GRAFT senders handle the PRUNE answers ------------------------------

__global__ __launch_bounds__(256) void k_hb_answer(DevState s, HbState h) {
    uint64_t handled = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x; r < h.n_pairs; r += (uint64_t)gridDim.x * 256u) {  // r = (v -> u)
        if (!h.halo_resp) {  // unsharded: only marked pairs have an answer; what is read is cleared
            if (!h.answer[r]) continue;
            h.answer[r] = 0;
        }
        const uint32_t q = h.rev[r];
        uint64_t resp = q == NO_PAIR ? 0 : (q & HALO) ? h.halo_resp[q & ~HALO] : h.resp[q];
        if (!h.halo_resp && q != NO_PAIR) h.resp[q] = 0;
        // AcceptFrom at v for the answering peer
        if (resp && !(h.eflags[r] & EDGE_DIRECT) && s.score[r] < h.graylist) resp = 0;
        if (resp) h.dirty[r] = 1;
        for (; resp; resp &= resp - 1) {
            handle_prune(s, h, r, (uint32_t)__builtin_ctzll(resp));
            ++handled;
        }
    }
    flush_count(h.stats, HB_PRUNES_HANDLED, handled);
}

// In-mesh (pair, topic) count: one thread per 16 pairs of a tile, reading
// their pair flags and, per topic, the tile's 16 record-flag bytes as uint4.
__global__ __launch_bounds__(256) void k_hb_mesh_links(DevState s, HbState h) {
    static_assert(TILE % 16 == 0 && REC_IN_MESH == 0x01 && PAIR_PRESENT == 0x01, "byte-lane counting below");
    uint64_t c = 0;
    const uint64_t n_chunks = (h.n_pairs + 15) / 16;  // pflags / rflags are padded to whole tiles
    for (uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x; k < n_chunks; k += (uint64_t)gridDim.x * 256u) {
        const uint64_t p0 = k * 16;
        const uint4 pf = *reinterpret_cast<const uint4*>(s.pflags + p0);
        const uint32_t pw[4] = {pf.x & 0x01010101u, pf.y & 0x01010101u, pf.z & 0x01010101u, pf.w & 0x01010101u};
        if (!(pw[0] | pw[1] | pw[2] | pw[3])) continue;
        for (uint32_t t = 0; t < s.n_topics; ++t) {
            const uint4 rf = *reinterpret_cast<const uint4*>(s.rflags + flag_index(p0, t, s.n_topics));
            c += __popc(rf.x & pw[0]) + __popc(rf.y & pw[1]) + __popc(rf.z & pw[2]) + __popc(rf.w & pw[3]);
        }
    }
    flush_count(h.stats, HB_MESH_LINKS, c);
}

// Shard exchange of per-pair control words: send slot j carries the words of
// the local pair send_pair[j] (0 for NO_PAIR), K words per slot.
__global__ __launch_bounds__(256) void k_hb_pack(const uint32_t* __restrict__ send_pair, uint64_t n_send,
                                                 const uint64_t* __restrict__ a, const uint64_t* __restrict__ b,
                                                 uint64_t* __restrict__ out) {
    const int K = b ? 2 : 1;
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < n_send; j += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = send_pair[j];
        out[K * j] = r == NO_PAIR ? 0 : a[r];
        if (b) out[K * j + 1] = r == NO_PAIR ? 0 : b[r];
    }
}

static inline unsigned blocks_for(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }
static inline unsigned grid_cap(uint64_t n, unsigned bs) {
    const unsigned b = blocks_for(n, bs);
    return b < 2048 ? b : 2048;
}
// One-wave blocks, grid-stride over nodes: at most 8192 waves (8 per SIMD),
// so the per-wave counter atomics stay few (same-address atomics serialise).
static inline unsigned wave_grid(uint64_t n) {
    const unsigned b = blocks_for(n, 64);
    return b < 8192 ? b : 8192;
}

hipError_t launch_hb_clear_backoff(const HbState& h, uint32_t n_topics, hipStream_t st) {
    const uint64_t n = (uint64_t)n_topics * h.n_pairs;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_clear_backoff, dim3(grid_cap(n, 256)), dim3(256), 0, st, h, n);
    return hipGetLastError();
}

hipError_t launch_hb_mesh(const DevState& s, const HbState& h, uint32_t t, hipStream_t st) {
    if (h.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_mesh, dim3(wave_grid(h.n_nodes)), dim3(64), 0, st, s, h, t);
    return hipGetLastError();
}

hipError_t launch_hb_gossip(const DevState& s, const HbState& h, uint32_t t, const GossipBatch* gb, uint32_t n_gb,
                            uint32_t max_ids, hipStream_t st) {
    if (h.n_nodes == 0 || n_gb == 0 || max_ids == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(h.n_long, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_hb_gossip, dim3(wave_grid(h.n_nodes)), dim3(64), 0, st, s, h, t, gb, n_gb);
    if (max_ids > (uint32_t)h.gp.max_ihave)  // some node may need the truncating path
        hipLaunchKernelGGL(k_hb_gossip_long, dim3(grid_cap(h.n_nodes, 1)), dim3(64), sizeof(uint32_t) * max_ids, st,
                           s, h, t, gb, n_gb);
    return hipGetLastError();
}

hipError_t launch_hb_recv(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_recv, dim3(wave_grid(h.n_nodes)), dim3(64), 0, st, s, h);
    return hipGetLastError();
}

hipError_t launch_hb_answer(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_answer, dim3(grid_cap(h.n_pairs, 256)), dim3(256), 0, st, s, h);
    return hipGetLastError();
}

hipError_t launch_hb_pack(const uint32_t* send_pair, uint64_t n_send, const uint64_t* a, const uint64_t* b,
                          uint64_t* out, hipStream_t st) {
    if (n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_pack, dim3(grid_cap(n_send, 256)), dim3(256), 0, st, send_pair, n_send, a, b, out);
    return hipGetLastError();
}

hipError_t launch_hb_mesh_links(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_mesh_links, dim3(grid_cap((h.n_pairs + 15) / 16, 256)), dim3(256), 0, st, s, h);
    return hipGetLastError();
}

}  // namespace gsx
