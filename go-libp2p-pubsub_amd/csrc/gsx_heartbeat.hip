// gsx_heartbeat.hip — the GossipSub heartbeat's mesh maintenance and IHAVE
// gossip as one synchronous round over the whole overlay (gsx.h,
// gsx_heartbeat).
//
//  (A) k_hb_scan — one coalesced pass over every wave's 64 nodes' pairs counts
//        each (node, topic) unit's mesh, negative-score and outbound members
//        and lists the units where some step of the maintenance can act
//        (per topic; hub nodes apart).  Then per topic t ascending:
//      k_hb_maintain — one lane per listed unit, its row (scores and
//        mesh / candidate / outbound / backoff bits) and its mesh and candidate
//        lists staged in LDS: the mesh maintenance of (v, t)
//        (gossipsub.go:1344-1510); k_hb_maintain_hub — the same for nodes
//        with more than HB_LANE_DEG peers, one wave each, the row in dynamic
//        LDS.  Everything a unit touches — the records, backoff entries and
//        control bits of v's own pairs for topic t — belongs to it alone.
//      k_hb_gossip — emitGossip (:1669-1723): a coalesced pass over each
//        wave's pairs stages the IHAVE target eligibility in LDS and rewrites
//        the topic's IHAVE slots, then one lane per node.  The IHAVE list is
//        the node's GetGossipIDs set (mcache.go:82-92) read straight from the
//        cached batches' seen words; its order is never observable
//        (handleIHave collects ids into a map, :641-650), so an untruncated
//        list is reported by its length and multiset digest.  Nodes whose
//        list exceeds MaxIHaveLength (per-target reshuffle + truncation,
//        :1708-1716), or whose tile holds a hub row, go to k_hb_gossip_long,
//        one wave per node with the list in LDS.
//  (B) k_hb_recv: one lane per receiving node u (k_hb_recv_hub: one wave per
//      hub), senders in ascending order (the Dhi check reads the mesh size the
//      previous accepts and prunes left, a running count per topic):
//      handleGraft / handlePrune, :718-843, AcceptFrom-gated (:582-593).
//  (C) k_hb_answer: one lane per pair, the GRAFT senders' handlePrune of the
//      PRUNE answers.
// Control messages are per-pair topic bitmasks (bit t of a u64), so a
// receiver reads one word per sender.  Round counters are summed per wave
// before one atomic each; the in-mesh link count is the scan's plus every
// step's change.  Integer/byte work: HBM / latency bound, no MFMA.
#include "gsx_ops.h"

namespace gsx {


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
// time is before every expiry).  The presence bit of a new entry is set too.
__device__ __forceinline__ void add_backoff(const HbState& h, uint64_t r, uint32_t t, int64_t interval) {
    // max(old, expire) with 0 = none: one max (expiries are positive), and the
    // presence bit (set iff the entry is nonzero); no value is read back
    atomicMax(reinterpret_cast<unsigned long long*>(&h.backoff[(size_t)t * h.n_pairs + r]),
              (unsigned long long)(h.now + interval));
    const size_t x = (size_t)(t / 8) * h.n_pairs + r;  // the byte's 32-bit word (the array is 4-B aligned)
    atomicOr(reinterpret_cast<uint32_t*>(h.bo8 + (x & ~(size_t)3)), (1u << (t % 8)) << (8 * (x & 3)));
}
__device__ __forceinline__ bool backoff_present(const HbState& h, uint64_t r, uint32_t t) {
    return (h.bo8[(size_t)(t / 8) * h.n_pairs + r] >> (t % 8)) & 1;
}

// clearBackoff, gossipsub.go:1585-1604: a lane per (pair, 8-topic chunk)
// presence byte; only the set bits' entries are read.
// Marks the IHAVE of topic t that the owner of pair r sends its peer: at the
// receiver's pair (the exchange (D) reads it there), or, when the peer lives
// on another range shard, at r for the shard exchange (gsx_gx_pack_ihave).
__device__ __forceinline__ void ihave_mark(const HbState& h, uint64_t r, uint32_t t) {
    const uint32_t q = h.rev[r];
    if (!h.ihave_bits || q == NO_PAIR) return;
    if (q & HALO) {
        if (h.gxs_out) h.gxs_out[r] |= 1ull << t;
        return;
    }
    h.ihave_bits[q] |= 1ull << t;
}

__global__ __launch_bounds__(256) void k_hb_clear_backoff(HbState h, uint32_t n_topics) {
    uint64_t cleared = 0;
    const uint32_t n_chunks = (n_topics + 7) / 8;
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    // chunk outer, pair inner: no 64-bit division per byte
    for (uint32_t c = 0; c < n_chunks; ++c) {
        const uint8_t* __restrict__ bo = h.bo8 + (size_t)c * h.n_pairs;
        const uint32_t kmax = min(8u, n_topics - 8 * c);
        for (uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x; r < h.n_pairs; r += stride) {
            const uint8_t b = bo[r];
            if (!b) continue;
            // every bit's entry loaded at once: a clear bit loads the first set bit's
            // entry again (a valid address, a cache hit), so no load waits alone;
            // only the chunk's topics (kmax, uniform): one load per lane when T = 1
            const uint32_t k0 = (uint32_t)__builtin_ctz(b);
            int64_t ex[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k)
                if (k < kmax) ex[k] = h.backoff[(size_t)(8 * c + ((b >> k & 1) ? k : k0)) * h.n_pairs + r];
            uint8_t keep = b;
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k)
                if (k < kmax && (b >> k & 1) && ex[k] + 2 * HEARTBEAT_INTERVAL_NS < h.now) {
                    h.backoff[(size_t)(8 * c + k) * h.n_pairs + r] = 0;
                    keep &= (uint8_t)~(1u << k);
                    ++cleared;
                }
            if (keep != b) h.bo8[(size_t)c * h.n_pairs + r] = keep;
        }
    }
    flush_count(h.stats, HB_BACKOFF_CLEARED, cleared);
}

__global__ __launch_bounds__(256) void k_bo_rebuild(const int64_t* __restrict__ backoff, uint8_t* __restrict__ bo8,
                                                    uint64_t n_pairs, uint32_t n_topics) {
    const uint64_t n_bytes = (uint64_t)((n_topics + 7) / 8) * n_pairs;
    for (uint64_t x = (uint64_t)blockIdx.x * 256u + threadIdx.x; x < n_bytes; x += (uint64_t)gridDim.x * 256u) {
        const uint32_t c = (uint32_t)(x / n_pairs);
        const uint64_t r = x % n_pairs;
        uint32_t b = 0;
        for (uint32_t k = 0; k < 8 && 8 * c + k < n_topics; ++k)
            b |= (uint32_t)(backoff[(size_t)(8 * c + k) * n_pairs + r] != 0) << k;
        bo8[x] = (uint8_t)b;
    }
}

// ---- (A) mesh maintenance ---------------------------------------------------------
// The round starts with one scan of every (node, topic) unit (k_hb_scan): a
// coalesced pass over each wave's 64 nodes' pairs counts, per unit, its mesh,
// the negative-score and outbound peers in it; units where no step of
// maintain() can act (a steady mesh: no negative score, Dlo <= |mesh| <= Dhi,
// enough outbound peers, not an opportunistic-graft tick) draw nothing and are
// done.  The others go to the topic's worklist — or to its hub list when the
// node has more than HB_LANE_DEG peers.  Per topic (ascending) k_hb_maintain
// then runs maintain() one lane per unit with the unit's row staged in LDS
// (scores, mesh / candidate / outbound / backoff bits; the mesh and candidate
// lists live in LDS too), and k_hb_maintain_hub one wave per hub unit with
// its row in dynamic LDS.  Only topic t's records, backoff entries and
// control bits of the node's own pairs change, so the scan's decisions for
// later topics stay valid, and every unit is independent of the others.

// Phase timing of k_hb_maintain (build with -DGSX_HB_PROF; development only):
// wave-level s_memrealtime deltas, printed by a few waves per launch.
#ifdef GSX_HB_PROF
#define HBP_DECL uint64_t hbp[10] = {0}; uint64_t hbp_t = wall_clock64();
#define HBP(i)                              \
    do {                                    \
        const uint64_t t_ = wall_clock64(); \
        hbp[i] += t_ - hbp_t;               \
        hbp_t = t_;                         \
    } while (0)
#else
#define HBP(i) \
    do {       \
    } while (0)
#endif

// Staged pair bits (u8, LDS)
constexpr uint8_t ST_MESH = 1;     // present and in the topic's mesh (gs.mesh[topic][p])
constexpr uint8_t ST_CAND = 2;     // present, connected, mesh-capable, not direct: getPeers' base filter
constexpr uint8_t ST_OUT = 4;      // outbound (gs.outbound[p])
constexpr uint8_t ST_BACKOFF = 8;  // gs.backoff[topic][p] present (map presence, :1377)
constexpr uint8_t ST_GRAFT = 16;   // maintain() grafted the pair (effects applied by apply_events)
constexpr uint8_t ST_PRUNE = 32;   // maintain() pruned the pair
constexpr uint8_t ST_ACTIVE = 64;  // the record's mesh-delivery counting is active (REC_ACTIVE)
constexpr uint8_t ST_NOPX = 128;   // pruned for a negative score: its PRUNE carries no PX (:1361-1368)

__device__ __forceinline__ uint8_t stage_pack(uint8_t pf, uint8_t ef, uint8_t rf, bool bo, bool in_t = true) {
    uint8_t f = 0;
    if ((pf & PAIR_PRESENT) && (rf & REC_IN_MESH)) f |= ST_MESH;
    if ((pf & (PAIR_PRESENT | PAIR_CONNECTED)) == (PAIR_PRESENT | PAIR_CONNECTED) && (ef & EDGE_GOSSIPSUB) &&
        !(ef & EDGE_DIRECT) && in_t)
        f |= ST_CAND;
    if (ef & EDGE_OUTBOUND) f |= ST_OUT;
    if (rf & REC_ACTIVE) f |= ST_ACTIVE;
    // only a candidate's backoff is ever tested (a pruned mesh peer gets the bit when pruned)
    if ((f & ST_CAND) && !(f & ST_MESH) && bo) f |= ST_BACKOFF;
    return f;
}
__device__ __forceinline__ uint8_t stage_bits(const DevState& s, const HbState& h, uint64_t r, uint32_t t) {
    // every input loaded unconditionally (no load waits at a divergent join)
    const uint8_t pf = s.pflags[r], ef = h.eflags[r];
    const uint8_t rf = s.rflags[flag_index(r, t, s.n_topics)];
    return stage_pack(pf, ef, rf, backoff_present(h, r, t), topic_peer(h.psub, r, t));
}

// One unit (v, t) over its staged row: sc / fl are the row's scores and bits,
// la / lb two lists of row offsets (deg entries each).  Indices are u16: the
// heartbeat refuses rows longer than HB_HUB_MAX.
struct HbUnit {
    const DevState& s;
    const HbState& h;
    uint32_t t;
    int64_t r0;  // first pair of the row
    int deg;
    const double* sc;
    uint8_t* fl;
    uint16_t* la;
    uint16_t* lb;
    bool scored;  // the topic has score params: Graft / Prune traces set / clear inMesh
    uint64_t grafts = 0, prunes = 0;
    int64_t links = 0;  // in-mesh (pair, topic) delta
#ifdef GSX_HB_PROF
    uint64_t* hbp = nullptr;
    uint64_t* hbp_t = nullptr;
#define HBPU(i)                                 \
    do {                                        \
        const uint64_t t_ = wall_clock64();     \
        hbp[i] += t_ - *hbp_t;                  \
        *hbp_t = t_;                            \
    } while (0)
#else
#define HBPU(i) \
    do {        \
    } while (0)
#endif

    __device__ bool in_mesh(int i) const { return fl[i] & ST_MESH; }
    __device__ int mesh_size() const {
        int n = 0;
        for (int i = 0; i < deg; ++i) n += (fl[i] & ST_MESH) != 0;
        return n;
    }
    __device__ double score(int i) const { return sc[i]; }
    __device__ bool outbound(int i) const { return fl[i] & ST_OUT; }

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
            const uint8_t f = fl[i];
            if ((f & (ST_CAND | ST_MESH | ST_BACKOFF)) != ST_CAND) continue;
            if (outbound_only && !(f & ST_OUT)) continue;
            const double x = sc[i];
            if (score_cmp == 0 && !(x >= ref)) continue;
            if (score_cmp == 1 && !(x > ref)) continue;
            out[n++] = (uint16_t)i;
        }
        g.shuffle(out, n);
        if (count_max > 0 && n > count_max) n = count_max;
        return n;
    }

    // graftPeer (:1353-1359) / prunePeer (:1345-1351) on the staged row only;
    // their memory effects are applied afterwards by apply_events, for the
    // whole stage at once (no dependent global access in the serial part).
    __device__ void graft(int i) {
        fl[i] |= ST_GRAFT;
        if (scored) {  // (a topic without params keeps no inMesh flag)
            fl[i] |= ST_MESH;
            ++links;
        }
        ++grafts;
    }
    __device__ void prune(int i) {  // (only mesh peers are pruned)
        fl[i] |= ST_PRUNE | ST_BACKOFF;
        if (scored) {  // (an unscored topic's imported inMesh flag stays, as in the record)
            fl[i] &= ~ST_MESH;
            --links;
        }
        ++prunes;
    }

    // stable sort by score (desc or asc) — the unstable sort.Slice of
    // :1393 / :1489 after the shuffle, made stable (gsx.h).  Insertion sort for
    // short lists, bottom-up merge sort (through `buf`) for long ones; both
    // keep equal scores in list order, so they agree exactly.
    __device__ bool before(uint16_t a, uint16_t b, bool desc) const {  // a strictly ahead of b
        return desc ? sc[a] > sc[b] : sc[a] < sc[b];
    }
    __device__ void sort_by_score(uint16_t* a, int n, bool desc, uint16_t* buf) const {
        if (n <= 32) {
            for (int i = 1; i < n; ++i) {
                const uint16_t x = a[i];
                int j = i - 1;
                while (j >= 0 && before(x, a[j], desc)) {
                    a[j + 1] = a[j];
                    --j;
                }
                a[j + 1] = x;
            }
            return;
        }
        uint16_t *src = a, *dst = buf;
        for (int w = 1; w < n; w *= 2) {
            for (int lo = 0; lo < n; lo += 2 * w) {
                const int mid = min(lo + w, n), hi = min(lo + 2 * w, n);
                int i = lo, j = mid, k = lo;
                while (i < mid && j < hi) dst[k++] = before(src[j], src[i], desc) ? src[j++] : src[i++];
                while (i < mid) dst[k++] = src[i++];
                while (j < hi) dst[k++] = src[j++];
            }
            uint16_t* x = src;
            src = dst;
            dst = x;
        }
        if (src != a)
            for (int i = 0; i < n; ++i) a[i] = src[i];
    }

    __device__ static void rotate(uint16_t* a, int i) {  // :1411-1418
        const uint16_t p = a[i];
        for (int j = i; j > 0; --j) a[j] = a[j - 1];
        a[0] = p;
    }

    __device__ void maintain(Rng& g) {
        const DevGossipParams& gp = h.gp;
        uint16_t* plst = la;
        uint16_t* tmp = lb;
        // drop all peers with negative score, without PX (:1361-1368)
        int n = mesh_list(plst);
        for (int i = 0; i < n; ++i)
            if (score(plst[i]) < 0) {
                prune(plst[i]);
                fl[plst[i]] |= ST_NOPX;
            }
        HBPU(0);
        // do we have enough peers? (:1370-1385)
        n = mesh_list(plst);
        if (n < gp.d_lo) {
            const int k = get_peers(gp.d - n, false, 0, 0.0, tmp, g);
            for (int i = 0; i < k; ++i) graft(tmp[i]);
        }
        HBPU(1);
        // do we have too many peers? (:1387-1448)
        n = mesh_list(plst);
        if (n > gp.d_hi) {
            g.shuffle(plst, n);
            sort_by_score(plst, n, true, tmp);
            g.shuffle(plst + gp.d_score, n - gp.d_score);
            int outb = 0;
            for (int i = 0; i < gp.d; ++i)
                if (outbound(plst[i])) ++outb;
            if (outb < gp.d_out) {
                if (outb > 0) {
                    int ihave = outb;
                    for (int i = 1; i < gp.d && ihave > 0; ++i)
                        if (outbound(plst[i])) {
                            rotate(plst, i);
                            --ihave;
                        }
                }
                int ineed = gp.d_out - outb;
                for (int i = gp.d; i < n && ineed > 0; ++i)
                    if (outbound(plst[i])) {
                        rotate(plst, i);
                        --ineed;
                    }
            }
            for (int i = gp.d; i < n; ++i) prune(plst[i]);
        }
        HBPU(2);
        // do we have enough outbound peers? (:1450-1476)
        n = mesh_list(plst);
        if (n >= gp.d_lo) {
            int outb = 0;
            for (int i = 0; i < n; ++i)
                if (outbound(plst[i])) ++outb;
            if (outb < gp.d_out) {
                const int k = get_peers(gp.d_out - outb, true, 0, 0.0, tmp, g);
                for (int i = 0; i < k; ++i) graft(tmp[i]);
            }
        }
        HBPU(3);
        // opportunistic grafting (:1478-1510)
        n = mesh_list(plst);
        if (gp.og_ticks && h.tick % gp.og_ticks == 0 && n > 1) {
            sort_by_score(plst, n, false, tmp);
            const double median = score(plst[n / 2]);
            HBPU(4);
            if (median < h.og_threshold) {
                const int k = get_peers(gp.og_peers, false, 1, median, tmp, g);
                for (int i = 0; i < k; ++i) graft(tmp[i]);
            }
        }
        HBPU(5);
    }
};

// The memory effects of maintain()'s grafts and prunes of pair r (staged bits
// f): the score-record events, the backoff entry, the control bits of r, its
// dirty mark and the receiver's inbox mark ((u -> v) of r = (v -> u) has
// control to read in (B)).  A pair is grafted or pruned at most once per unit
// except prune-after-graft, which the graft-then-prune order covers (a pruned
// peer is backed off, so never grafted again in the same round).
__device__ __forceinline__ void apply_events(const DevState& s, const HbState& h, uint64_t r, uint32_t t, uint8_t f,
                                             uint32_t q, bool scored) {
    if (f & ST_GRAFT) {  // ev_graft (a grafted candidate is present)
        if (scored) {
            reinterpret_cast<int64_t*>(s.rec)[rec_index(r, t, s.n_topics, GRAFT)] = h.now;
            s.rflags[flag_index(r, t, s.n_topics)] = REC_IN_MESH | REC_FRESH;
        }
        atomicOr((unsigned long long*)&h.ctl[2 * (size_t)r], 1ull << t);
    }
    if (f & ST_PRUNE) {  // ev_prune (a pruned mesh peer is present)
        if (scored) {
            // after a graft in the same unit the record is fresh (not active)
            const bool active = (f & ST_ACTIVE) && !(f & ST_GRAFT);
            if (active) {
                const size_t b = rec_index(r, t, s.n_topics, FMD);
                const double threshold = s.tp[t].thr3;
                const double mmd = s.rec[b + MMD * TILE];
                if (mmd < threshold) {
                    const double deficit = threshold - mmd;
                    s.rec[b + MFP * TILE] = s.rec[b + MFP * TILE] + deficit * deficit;
                }
            }
            s.rflags[flag_index(r, t, s.n_topics)] = active ? REC_ACTIVE : 0;
        }
        add_backoff(h, r, t, h.gp.prune_backoff_ns);
        atomicOr((unsigned long long*)&h.ctl[2 * (size_t)r + 1], 1ull << t);
        if ((f & ST_NOPX) && h.pxno) h.pxno[r] |= 1;  // noPX[p] ((A) sets only this bit: racing topics agree)
    }
    h.dirty[r] = 1;
    if (q != NO_PAIR && !(q & HALO)) h.inbox[q] = 1;
}

constexpr int APPLY_UNROLL = 4;  // receiver-pair loads per lane in flight

// Draws are keyed by the GLOBAL node id, so a range shard draws what the
// whole-overlay engine draws for the same node.
__device__ __forceinline__ Rng hb_rng(const HbState& h, uint32_t v, uint32_t t, uint32_t k) {
    return Rng{h.seed, TAG_HEARTBEAT, (uint64_t)h.node_lo + v,
               (h.tick << 32) | ((uint64_t)t << 24) | (h.fan_mode ? (1ull << 23) : 0ull), k};
}

// LDS hand-off between the lanes of a one-wave block: a wave's LDS accesses
// are performed in order, so only the compiler must not move them across
// (no s_waitcnt on outstanding global stores, unlike __syncthreads).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_prefix(uint32_t x, uint32_t lane) {  // exclusive
    uint32_t incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += y;
    }
    return incl - x;
}

// Appends the lanes with `want` to list[0 ..) (count in *n): one atomic per wave.
__device__ __forceinline__ void wave_append(bool want, uint32_t value, uint32_t* list, uint32_t* n, uint32_t lane) {
    const uint64_t b = __ballot(want);
    if (!b) return;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(n, (uint32_t)__popcll(b));
    base = __shfl(base, 0, 64);
    if (want) list[base + (uint32_t)__popcll(b & ((1ull << lane) - 1))] = value;
}

constexpr int SCAN_TOPICS = 8;     // topics decided per pass over a wave's pairs
constexpr int SCAN_STAGE = 2048;   // pairs of a tile staged (scan bits, u32) for the per-node counts

// A pair's scan bits for topics t0 .. t0+7 (t0 a multiple of 8): bit k = in
// the mesh of topic t0+k, bit 8 = score < 0, bit 9 = outbound, bit 10 =
// getPeers' base filter with score >= 0 (present, connected, mesh-capable, not
// direct), bit 11 = score below the opportunistic-graft threshold, bit 16+k =
// a getPeers candidate of topic t0+k (base filter, not in that mesh, no
// backoff entry; bo = the pair's presence byte of the chunk).
constexpr uint32_t SC_NEG = 1u << 8, SC_OUT = 1u << 9, SC_CAND = 1u << 10;
constexpr uint32_t SC_OGLOW = 1u << 11;
__device__ __forceinline__ uint32_t scan_pack(uint8_t pf, uint8_t ef, double sc, const uint8_t (&rf)[SCAN_TOPICS],
                                              uint8_t bo, uint32_t nt, double og_threshold, uint32_t in8 = 0xFFu) {
    if (!(pf & PAIR_PRESENT)) return 0;
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < SCAN_TOPICS; ++k)
        if (rf[k] & REC_IN_MESH) m |= 1u << k;
    if ((pf & PAIR_CONNECTED) && (ef & EDGE_GOSSIPSUB) && !(ef & EDGE_DIRECT) && sc >= 0.0)
        m |= (~(m | bo) & ((1u << nt) - 1) & in8) << 16;  // (in8: the peer joined t0 + k)
    if (sc < 0) m |= SC_NEG;
    if (sc < og_threshold) m |= SC_OGLOW;
    if (ef & EDGE_OUTBOUND) m |= SC_OUT;
    if ((pf & PAIR_CONNECTED) && (ef & EDGE_GOSSIPSUB) && !(ef & EDGE_DIRECT) && sc >= 0.0) m |= SC_CAND;
    return m;
}
__device__ __forceinline__ uint32_t scan_bits(const DevState& s, const HbState& h, uint64_t r, uint32_t t0,
                                              uint32_t nt) {
    uint8_t rf[SCAN_TOPICS];
#pragma unroll
    for (int k = 0; k < SCAN_TOPICS; ++k) rf[k] = k < (int)nt ? s.rflags[flag_index(r, t0 + k, s.n_topics)] : 0;
    return scan_pack(s.pflags[r], h.eflags[r], s.score[r], rf, h.bo8[(size_t)(t0 / 8) * h.n_pairs + r], nt,
                     h.og_threshold, h.psub ? (uint32_t)((h.psub[r] >> t0) & 0xFF) : 0xFFu);
}

// (A) scan: every unit of every topic.  A wave takes a tile of 64 consecutive
// nodes: one coalesced pass packs each pair's bits into LDS (four pairs per
// lane in flight), then one lane per node counts its row — mesh size, negative
// and outbound members, members below the opportunistic-graft threshold, and
// which topics have getPeers candidates (any / outbound; the pair's backoff
// presence byte is staged with its bits).
// A unit acts iff some step of maintain() would: a negative member, more than
// Dhi, an opportunistic-graft tick with a mesh of 2+ whose median score is
// below the threshold, or a graft step with a candidate.  The tile's acting units are listed at work[t][tile * 64 ..]
// (count tcnt[t][tile]: no atomics); hub nodes go to the topic's hub list;
// every unit's rngk starts at 0; the in-mesh links before the round are
// counted.  Blocks of four waves over a bounded grid: one counter atomic per
// block (same-address atomics serialise at the memory side).
constexpr int SCAN_WAVES = 4;
__global__ __launch_bounds__(256) void k_hb_scan(DevState s, HbState h) {
    __shared__ int64_t rs_w[SCAN_WAVES][65];
    __shared__ uint32_t st_w[SCAN_WAVES][SCAN_STAGE];
    const DevGossipParams& gp = h.gp;
    const bool og_tick = gp.og_ticks && h.tick % gp.og_ticks == 0;
    const uint32_t lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    int64_t* rs = rs_w[wave];
    uint32_t* st = st_w[wave];
    const uint32_t T = s.n_topics;
    const uint32_t n_tiles = (h.n_nodes + 63) / 64;
    unsigned long long links[1] = {0};
#ifdef GSX_HB_PROF
    HBP_DECL
#endif
    for (uint32_t tb = blockIdx.x * SCAN_WAVES; tb < n_tiles; tb += gridDim.x * SCAN_WAVES) {
        const uint32_t tile = tb + wave;  // (block-uniform loop: every wave reaches every barrier)
        const uint32_t v0 = tile * 64u;
        const uint32_t nv = tile < n_tiles ? min(64u, h.n_nodes - v0) : 0;
        if (nv) {
            rs[lane] = h.row_ptr[v0 + min(lane, nv)];
            if (lane == 0) rs[64] = h.row_ptr[v0 + nv];
        }
        __syncthreads();
        HBP(0);
        const int64_t pa = nv ? rs[0] : 0, pb = nv ? rs[64] : 0;
        const bool staged = pb - pa <= SCAN_STAGE;
        const uint32_t v = v0 + lane;
        const int64_t r0 = lane < nv ? rs[lane] : 0;
        const int deg = lane < nv ? (int)(rs[lane + 1] - r0) : 0;
        for (uint32_t t0 = 0; t0 < T; t0 += SCAN_TOPICS) {
            const uint32_t nt = min((uint32_t)SCAN_TOPICS, T - t0);
            if (staged) {
                for (int64_t rb = pa + lane; rb < pb; rb += 256) {
                    // unconditional loads of clamped (valid) addresses, masked after: a
                    // load under a divergent branch is waited for at the branch's join
                    uint8_t pf[4], ef[4], bo[4], rf[4][SCAN_TOPICS];
                    double sc[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int64_t r = min(rb + 64 * j, pb - 1);
                        pf[j] = s.pflags[r];
                        ef[j] = h.eflags[r];
                        sc[j] = s.score[r];
                        bo[j] = h.bo8[(size_t)(t0 / 8) * h.n_pairs + r];
#pragma unroll
                        for (int k = 0; k < SCAN_TOPICS; ++k) rf[j][k] = s.rflags[flag_index(r, min(t0 + k, T - 1), T)];
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int k = 0; k < SCAN_TOPICS; ++k)
                            if (k >= (int)nt) rf[j][k] = 0;
                    uint32_t in8[4] = {0xFFu, 0xFFu, 0xFFu, 0xFFu};
                    if (h.psub) {  // (uniform) the peers' joined topics
#pragma unroll
                        for (int j = 0; j < 4; ++j) in8[j] = (uint32_t)((h.psub[min(rb + 64 * j, pb - 1)] >> t0) & 0xFF);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int64_t r = rb + 64 * j;
                        if (r < pb) st[r - pa] = scan_pack(pf[j], ef[j], sc[j], rf[j], bo[j], nt, h.og_threshold, in8[j]);
                    }
                }
            }
            __syncthreads();
            HBP(1);
            int n[SCAN_TOPICS], neg[SCAN_TOPICS], outb[SCAN_TOPICS], low[SCAN_TOPICS];
#pragma unroll
            for (int k = 0; k < SCAN_TOPICS; ++k) n[k] = neg[k] = outb[k] = low[k] = 0;
            uint32_t cg = 0, co = 0;  // topics with a getPeers candidate: any / outbound
            for (int i = 0; i < deg; ++i) {
                const uint32_t m = staged ? st[r0 - pa + i] : scan_bits(s, h, r0 + i, t0, nt);
                cg |= m >> 16;
                co |= (m & SC_OUT) ? m >> 16 : 0;
#pragma unroll
                for (int k = 0; k < SCAN_TOPICS; ++k)
                    if (m >> k & 1) {
                        ++n[k];
                        neg[k] += (m & SC_NEG) != 0;
                        outb[k] += (m & SC_OUT) != 0;
                        low[k] += (m & SC_OGLOW) != 0;
                    }
            }
            HBP(2);
            // per topic: a step of maintain() acts (getPeers' steps iff it finds a candidate)
            uint32_t act = 0;
#pragma unroll
            for (int k = 0; k < SCAN_TOPICS; ++k) {
                if (k >= (int)nt || lane >= nv) continue;
                const uint32_t t = t0 + k;
                links[0] += (uint64_t)n[k];
                // opportunistic grafting acts iff the median mesh score (ascending
                // [n/2]) is below the threshold: iff more than n/2 members are
                // (scores are finite; the sort and the draws have no other effect)
                const bool grow = n[k] < gp.d_lo, more_out = !grow && outb[k] < gp.d_out;
                const bool a = joined_node(h.sub, v, t) &&  // gs.mesh holds the joined topics
                               (neg[k] > 0 || n[k] > gp.d_hi || (og_tick && n[k] > 1 && low[k] > n[k] / 2) ||
                                (grow && (cg >> k & 1)) || (more_out && (co >> k & 1)));  // :1370-1385, :1450-1476
                act |= (uint32_t)a << k;
                h.rngk[(size_t)t * h.n_nodes + v] = 0;
                h.mcount[(size_t)t * h.n_nodes + v] = (uint16_t)n[k];  // (A) updates it for acting units
            }
            HBP(3);
            for (uint32_t k = 0; k < nt; ++k) {
                const uint32_t t = t0 + k;
                const bool active = lane < nv && (act >> k & 1);
                if (nv) {
                    const bool lw = active && deg <= HB_LANE_DEG;
                    const uint64_t b = __ballot(lw);
                    if (lw) h.work[(size_t)t * h.n_tiles64 + v0 + (uint32_t)__popcll(b & ((1ull << lane) - 1))] = v;
                    if (lane == 0) h.tcnt[(size_t)t * n_tiles + tile] = (uint8_t)__popcll(b);
                    wave_append(active && deg > HB_LANE_DEG, v, h.hub_work + (size_t)t * h.n_nodes, h.n_hub + t, lane);
                }
            }
            HBP(4);
            __syncthreads();  // st is rewritten by the next topic chunk / tile
            HBP(5);
        }
    }
#ifdef GSX_HB_PROF
    if (threadIdx.x == 0 && blockIdx.x % 512 == 0)
        printf("HBS blk=%u rows=%lu stage=%lu count=%lu decide=%lu out=%lu tail=%lu\n", blockIdx.x, hbp[0], hbp[1],
               hbp[2], hbp[3], hbp[4], hbp[5]);
#endif
    const uint32_t slot[1] = {HB_MESH_LINKS};
    block_count<1>(links, h.stats, slot);
}

constexpr int GOSSIP_STAGE = 1024;  // pairs of a tile k_hb_gossip stages per wave

// (A) per topic: the listed units, one lane each, rows staged in LDS.  A wave
// takes a group of MAINT_GROUP tiles, gathers their listed units (a prefix over the
// per-tile counts: no atomics) 64 at a time, and stages their rows
// cooperatively (every lane loads items of every row, 64 loads per
// instruction); when the rows exceed the stage it runs them in windows of
// whole rows.
constexpr int MAINT_UNROLL = 4;    // staged pairs per lane in flight
constexpr uint32_t MAINT_GROUP = 4;  // tiles per maintenance wave (up to 256 listed units, 64 at a time)
constexpr int HB_STAGE = 1024;       // pairs staged at once (14 KB of LDS per wave)

__global__ __launch_bounds__(64) void k_hb_maintain(DevState s, HbState h, uint32_t t_base) {
    const uint32_t t = t_base + blockIdx.y;  // a run of topics per launch: the units are independent
    __shared__ double sc[HB_STAGE];  // scores; after maintain(): the events' receiver pairs (u32)
    __shared__ uint8_t fl[HB_STAGE];
    __shared__ uint8_t owner[HB_STAGE];  // the lane whose row holds the item
    __shared__ uint16_t la[HB_STAGE], lb[HB_STAGE];
    __shared__ uint32_t offs[65];
    __shared__ int64_t r0s[64];
    __shared__ uint32_t pfx[65];
    uint32_t* qs = reinterpret_cast<uint32_t*>(sc);
    const uint32_t lane = threadIdx.x;
    const uint32_t n_tiles = (h.n_nodes + 63) / 64;
    const uint8_t* tcnt = h.tcnt + (size_t)t * n_tiles;
    const uint32_t* work = h.work + (size_t)t * h.n_tiles64;
    const bool scored = t < s.n_topics && s.tp[t].scored;
    uint64_t grafts = 0, prunes = 0;
    int64_t links = 0;
#ifdef GSX_HB_PROF
    HBP_DECL
#endif
    for (uint32_t g0 = blockIdx.x * MAINT_GROUP; g0 < n_tiles; g0 += gridDim.x * MAINT_GROUP) {
        const uint32_t c = (lane < MAINT_GROUP && g0 + lane < n_tiles) ? tcnt[g0 + lane] : 0;
        const uint32_t p = wave_prefix(c, lane);
        pfx[lane] = p;
        if (lane == 63) pfx[64] = p + c;
        wave_lds_sync();
        const uint32_t total = pfx[64];
        for (uint32_t u0 = 0; u0 < total; u0 += 64) {
            const uint32_t u = u0 + lane;
            const bool valid = u < total;
            uint32_t lo = 0;  // pfx[lo] <= u < pfx[lo + 1]
            for (uint32_t x = 1; x < MAINT_GROUP; ++x) lo += pfx[x] <= u;
            // (clamped in-range address: loaded by every lane, used by the valid ones)
            const uint32_t v = work[(size_t)min(g0 + lo, n_tiles - 1) * 64 + min(u - pfx[lo], 63u)];
            const int64_t ra = h.row_ptr[valid ? v : 0], rb = h.row_ptr[valid ? v + 1 : 0];
            const int64_t r0 = valid ? ra : 0;
            const int deg = valid ? (int)(rb - ra) : 0;
            const uint32_t off = wave_prefix((uint32_t)deg, lane);
            offs[lane] = off;
            r0s[lane] = r0;
            if (lane == 63) offs[64] = off + deg;
            wave_lds_sync();
            HBP(6);
            // windows of whole rows: lanes [l0, l1) whose rows fit [offs[l0], offs[l0] + HB_STAGE)
            uint32_t l0 = 0;
            while (l0 < 64 && offs[l0] < offs[64]) {
                const uint32_t base = offs[l0];
                uint32_t l1 = l0;
                while (l1 < 64 && offs[l1 + 1] - base <= HB_STAGE) ++l1;  // (uniform: every lane computes it)
                const uint32_t end = offs[l1];
                if (lane >= l0 && lane < l1)
                    for (int i = 0; i < deg; ++i) owner[off - base + i] = (uint8_t)lane;
                wave_lds_sync();
                // item k belongs to the row holding it; MAINT_UNROLL items per lane in
                // flight (all loads issued before any result is used)
                for (uint32_t k0 = base + lane; k0 < end; k0 += 64 * MAINT_UNROLL) {
                    uint64_t r[MAINT_UNROLL];
#pragma unroll
                    for (int j = 0; j < MAINT_UNROLL; ++j) {
                        const uint32_t k = min(k0 + 64 * j, end - 1);
                        const uint32_t o = owner[k - base];
                        r[j] = (uint64_t)r0s[o] + (k - offs[o]);
                    }
                    double x[MAINT_UNROLL];
                    uint8_t pf[MAINT_UNROLL], ef[MAINT_UNROLL], rf[MAINT_UNROLL];
                    uint8_t bb[MAINT_UNROLL];
#pragma unroll
                    for (int j = 0; j < MAINT_UNROLL; ++j) {
                        x[j] = s.score[r[j]];
                        pf[j] = s.pflags[r[j]];
                        ef[j] = h.eflags[r[j]];
                        rf[j] = s.rflags[flag_index(r[j], t, s.n_topics)];
                        bb[j] = h.bo8[(size_t)(t / 8) * h.n_pairs + r[j]];
                    }
                    bool in_t[MAINT_UNROLL];
#pragma unroll
                    for (int j = 0; j < MAINT_UNROLL; ++j) in_t[j] = true;
                    if (h.psub) {  // (uniform) the peer joined t
#pragma unroll
                        for (int j = 0; j < MAINT_UNROLL; ++j) in_t[j] = (h.psub[r[j]] >> t) & 1;
                    }
#pragma unroll
                    for (int j = 0; j < MAINT_UNROLL; ++j) {
                        const uint32_t k = k0 + 64 * j;
                        if (k < end) {
                            sc[k - base] = x[j];
                            fl[k - base] = stage_pack(pf[j], ef[j], rf[j], (bb[j] >> (t % 8)) & 1, in_t[j]);
                        }
                    }
                }
                wave_lds_sync();
                HBP(7);
                if (lane >= l0 && lane < l1 && valid) {
                    const uint32_t o = off - base;
                    HbUnit U{s, h, t, r0, deg, sc + o, fl + o, la + o, lb + o, scored};
#ifdef GSX_HB_PROF
                    U.hbp = hbp;
                    U.hbp_t = &hbp_t;
#endif
                    Rng g = hb_rng(h, v, t, 0);
                    U.maintain(g);
                    h.rngk[(size_t)t * h.n_nodes + v] = g.k;  // emitGossip continues this (node, topic) draw stream
                    h.mcount[(size_t)t * h.n_nodes + v] = (uint16_t)U.mesh_size();  // read by (B)'s Dhi check
                    grafts += U.grafts;
                    prunes += U.prunes;
                    links += U.links;
                }
                wave_lds_sync();
                HBP(8);
                // the window's events, the whole wave: first every receiver pair
                // (loads only, APPLY_UNROLL per lane in flight, into the score stage),
                // then the stores and atomics (nothing waits on them)
                for (uint32_t k0 = base + lane; k0 < end; k0 += 64 * APPLY_UNROLL) {
                    uint32_t q[APPLY_UNROLL];
                    bool any = false;
#pragma unroll
                    for (int j = 0; j < APPLY_UNROLL; ++j) {
                        const uint32_t k = min(k0 + 64 * j, end - 1);
                        const uint32_t o = owner[k - base];
                        any |= k0 + 64 * j < end && (fl[k - base] & (ST_GRAFT | ST_PRUNE));
                        q[j] = h.rev[(uint64_t)r0s[o] + (k - offs[o])];
                    }
                    if (!any) continue;
#pragma unroll
                    for (int j = 0; j < APPLY_UNROLL; ++j)
                        if (k0 + 64 * j < end) qs[k0 + 64 * j - base] = q[j];
                }
                wave_lds_sync();
                for (uint32_t k = base + lane; k < end; k += 64) {
                    const uint8_t f = fl[k - base];
                    if (!(f & (ST_GRAFT | ST_PRUNE))) continue;
                    const uint32_t o = owner[k - base];
                    apply_events(s, h, (uint64_t)r0s[o] + (k - offs[o]), t, f, qs[k - base], scored);
                }
                wave_lds_sync();  // the stage is reused by the next window / batch
                HBP(9);
                l0 = l1;
            }
        }
        wave_lds_sync();  // pfx is rewritten by the next group
    }
#ifdef GSX_HB_PROF
    if (lane == 0 && blockIdx.x % 1024 == 0)
        printf("HBP t=%u blk=%u pre=%lu stage=%lu neg=%lu dlo=%lu dhi=%lu out=%lu ogsort=%lu oggraft=%lu post=%lu apply=%lu\n",
               t, blockIdx.x, hbp[6], hbp[7], hbp[0], hbp[1], hbp[2], hbp[3], hbp[4], hbp[5], hbp[8], hbp[9]);
#endif
    flush_count(h.stats, HB_GRAFTS, grafts);
    flush_count(h.stats, HB_PRUNES, prunes);
    flush_count(h.stats, HB_MESH_LINKS, (uint64_t)links);
}

// (A) per topic: hub units (more than HB_LANE_DEG peers), one wave each, the
// row in dynamic LDS (13 B per pair); the wave stages it, lane 0 runs maintain().
__global__ __launch_bounds__(64) void k_hb_maintain_hub(DevState s, HbState h, uint32_t t_base) {
    const uint32_t t = t_base + blockIdx.y;
    extern __shared__ double dyn[];
    const uint32_t lane = threadIdx.x;
    const uint32_t nw = h.n_hub[t];
    const uint32_t* work = h.hub_work + (size_t)t * h.n_nodes;
    const bool scored = t < s.n_topics && s.tp[t].scored;
    uint64_t grafts = 0, prunes = 0;
    int64_t links = 0;
    for (uint32_t w = blockIdx.x; w < nw; w += gridDim.x) {
        const uint32_t v = work[w];
        const int64_t r0 = h.row_ptr[v];
        const int deg = (int)(h.row_ptr[v + 1] - r0);
        double* sc = dyn;
        uint16_t* la = reinterpret_cast<uint16_t*>(sc + deg);
        uint16_t* lb = la + deg;
        uint8_t* fl = reinterpret_cast<uint8_t*>(lb + deg);
        for (int i = lane; i < deg; i += 64) {
            sc[i] = s.score[r0 + i];
            fl[i] = stage_bits(s, h, r0 + i, t);
        }
        __syncthreads();
        if (lane == 0) {
            HbUnit U{s, h, t, r0, deg, sc, fl, la, lb, scored};
            Rng g = hb_rng(h, v, t, 0);
            U.maintain(g);
            h.rngk[(size_t)t * h.n_nodes + v] = g.k;
            h.mcount[(size_t)t * h.n_nodes + v] = (uint16_t)U.mesh_size();
            grafts += U.grafts;
            prunes += U.prunes;
            links += U.links;
        }
        __syncthreads();
        for (int i = lane; i < deg; i += 64) {
            const uint8_t f = fl[i];
            const uint32_t q = h.rev[r0 + i];
            if (f & (ST_GRAFT | ST_PRUNE)) apply_events(s, h, r0 + i, t, f, q, scored);
        }
        __syncthreads();  // the LDS row is restaged by the next unit
    }
    flush_count(h.stats, HB_GRAFTS, grafts);
    flush_count(h.stats, HB_PRUNES, prunes);
    flush_count(h.stats, HB_MESH_LINKS, (uint64_t)links);
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
    // excluded: the mesh, or the fanout for a fanout unit (:1514, :1553)
    const bool excl = h.fan_mode ? ((h.fanout[r] >> t) & 1) != 0 : hb_in_mesh(s, r, t);
    return (s.pflags[r] & (PAIR_PRESENT | PAIR_CONNECTED)) == (PAIR_PRESENT | PAIR_CONNECTED) &&
           topic_peer(h.psub, r, t) && (f & EDGE_GOSSIPSUB) && !(f & EDGE_DIRECT) && !excl &&
           live_score(s, h, r) >= h.gossip_threshold;
}

// A cached batch's per-node summary (count, digest of its ids): once per
// batch.  G lanes per node, each over 4-word chunks of the row, so a wave
// reads whole 128-B rows (G = 4 at 16 words) instead of one word per lane
// at a 128-B stride; the group sums its counts and digests with shuffles.
template <int G>
__global__ __launch_bounds__(256) void k_mc_summary(const uint64_t* __restrict__ seen, uint32_t n_nodes,
                                                    uint32_t n_words, uint32_t n_msgs,
                                                    const uint64_t* __restrict__ msg_dig,
                                                    const uint64_t* __restrict__ word_dig, uint64_t* __restrict__ dig,
                                                    uint32_t* __restrict__ cnt) {
    const uint32_t lc = threadIdx.x % G;
    const uint32_t CWv = G > 1 ? 4 : n_words;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t / G < n_nodes; t += gridDim.x * 256u) {
        const uint32_t v = t / G;
        uint32_t L = 0;
        uint64_t d = 0;
        for (uint32_t w0 = lc * CWv; w0 < n_words; w0 += G * CWv)
            for (uint32_t w = w0; w < w0 + CWv; ++w) {
                uint64_t word = seen[(size_t)v * n_words + w];
                L += (uint32_t)__popcll(word);
                const uint32_t left = n_msgs > w * 64 ? n_msgs - w * 64 : 0;
                const uint64_t full = left >= 64 ? ~0ull : ((1ull << left) - 1);
                if (word && word == full) {  // every message of the word (the common case once a batch has spread)
                    d += word_dig[w];
                    continue;
                }
                uint64_t miss = full & ~word;
                if (word && __popcll(miss) < __popcll(word)) {  // most of the word: its digest less the missing ids
                    d += word_dig[w];
                    for (; miss; miss &= miss - 1) d -= msg_dig[w * 64 + (uint32_t)__builtin_ctzll(miss)];
                    continue;
                }
                for (; word; word &= word - 1) d += msg_dig[w * 64 + (uint32_t)__builtin_ctzll(word)];
            }
#pragma unroll
        for (int o = 1; o < G; o <<= 1) {
            L += __shfl_xor(L, o, G);
            d += __shfl_xor(d, o, G);
        }
        if (lc == 0) {
            dig[v] = d;
            cnt[v] = L;
        }
    }
}

// GetGossipIDs of (v, t): its length and multiset digest, the sum of the
// node's summaries over the batches of the gossip window.
__device__ __forceinline__ uint32_t gossip_ids(const HbState& h, uint32_t v, const GossipBatch* __restrict__ gb,
                                               uint32_t n_gb, uint64_t& dig) {
    uint32_t L = 0;
    dig = 0;
    uint32_t b = 0;
    for (; b + 4 <= n_gb; b += 4) {  // four batches' summaries in flight per round trip
        uint32_t c[4];
        uint64_t d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            c[j] = gb[b + j].cnt[v];
            d[j] = gb[b + j].dig[v];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            L += c[j];
            dig += d[j];
        }
    }
    for (; b < n_gb; ++b) {
        L += gb[b].cnt[v];
        dig += gb[b].dig[v];
    }
    return L;
}

// emitGossip of topic t for every node.  A wave takes a tile of 64
// consecutive nodes: one coalesced pass over their pairs (four per lane in
// flight) rewrites the topic's IHAVE slots of the range (0 = none) and stages
// each pair's target eligibility in LDS; then a lane per node counts its
// GetGossipIDs, lists its eligible peers in LDS, shuffles and writes the
// targets.  A tile whose rows exceed the stage, and every list longer than
// MaxIHaveLength (per-target reshuffle + truncation, :1708-1716), goes to
// k_hb_gossip_long, one wave per node.  Blocks of four waves over a bounded
// grid: one counter atomic per block.
// Per pair, once per round (before any maintenance): GELIG_TARGET = the
// topic-independent part of gossip_target (present, connected, a gossipsub
// peer, not direct: gossipsub.go:1688-1703), GELIG_SCORE = its score as the
// round started >= GossipThreshold; k_hb_gossip reads this byte per topic
// instead of the flags and the score (a pair the round's maintenance touched
// is re-evaluated live there).
__global__ __launch_bounds__(256) void k_hb_gelig(DevState s, HbState h) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x; r < h.n_pairs; r += (uint64_t)gridDim.x * 256u) {
        const uint8_t pf = s.pflags[r], ef = h.eflags[r];
        uint8_t g = 0;
        if ((pf & (PAIR_PRESENT | PAIR_CONNECTED)) == (PAIR_PRESENT | PAIR_CONNECTED) && (ef & EDGE_GOSSIPSUB) &&
            !(ef & EDGE_DIRECT))
            g = GELIG_TARGET | (s.score[r] >= h.gossip_threshold ? GELIG_SCORE : 0);
        h.gelig[r] = g;
    }
}

__global__ __launch_bounds__(256) void k_hb_gossip(DevState s, HbState h, uint32_t t, const GossipBatch* __restrict__ gb,
                                                   uint32_t n_gb) {
    __shared__ int64_t rs_w[SCAN_WAVES][65];
    __shared__ uint8_t el_w[SCAN_WAVES][GOSSIP_STAGE];
    __shared__ uint16_t pl_w[SCAN_WAVES][GOSSIP_STAGE];
    const uint32_t lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    int64_t* rs = rs_w[wave];
    uint8_t* el = el_w[wave];
    uint16_t* pl = pl_w[wave];
    unsigned long long cnt[2] = {0, 0};  // IHAVE messages, ids
    const size_t tslot = (size_t)t * h.n_pairs;
    const uint32_t n_tiles = (h.n_nodes + 63) / 64;
    for (uint32_t tb = blockIdx.x * SCAN_WAVES; tb < n_tiles; tb += gridDim.x * SCAN_WAVES) {
        const uint32_t tile = tb + wave;  // (block-uniform loop: every wave reaches every barrier)
        const uint32_t v0 = tile * 64u;
        const uint32_t nv = tile < n_tiles ? min(64u, h.n_nodes - v0) : 0;
        if (nv) {
            rs[lane] = h.row_ptr[v0 + min(lane, nv)];
            if (lane == 0) rs[64] = h.row_ptr[v0 + nv];
        }
        __syncthreads();
        const int64_t pa = nv ? rs[0] : 0, pb = nv ? rs[64] : 0;
        const bool staged = pb - pa <= GOSSIP_STAGE;
        for (int64_t rb = pa + lane; rb < pb; rb += 256) {
            uint8_t ge[4], rf[4], dt[4];
            bool in_t[4] = {true, true, true, true};
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // unconditional loads of clamped addresses (see k_hb_scan)
                const int64_t r = min(rb + 64 * j, pb - 1);
                ge[j] = h.gelig[r];
                rf[j] = s.rflags[flag_index(r, t, s.n_topics)];
                dt[j] = h.dirty[r];
            }
            if (h.psub) {  // (uniform) the peers' joined topics
#pragma unroll
                for (int j = 0; j < 4; ++j) in_t[j] = (h.psub[min(rb + 64 * j, pb - 1)] >> t) & 1;
            }
            if (h.fan_mode) {  // (uniform) a fanout pass excludes the fanout, not the mesh
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    rf[j] = ((h.fanout[min(rb + 64 * j, pb - 1)] >> t) & 1) ? REC_IN_MESH : 0;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t r = rb + 64 * j;
                if (r >= pb) continue;
                if (!staged) continue;
                // gossip_target from the round's eligibility byte (k_hb_gelig) and the
                // topic's mesh flag; live score: dirty pairs re-evaluated
                bool ok = (ge[j] & GELIG_TARGET) && in_t[j] && !(rf[j] & REC_IN_MESH);
                if (ok) ok = dt[j] ? eval_pair(s, h.pp, r) >= h.gossip_threshold : (ge[j] & GELIG_SCORE) != 0;
                el[r - pa] = ok;
            }
        }
        __syncthreads();
        const bool unit = lane < nv && (h.fan_mode ? ((h.fan_has[v0 + lane] >> t) & 1) != 0
                                                   : joined_node(h.sub, v0 + lane, t));
        if (unit) {
            const uint32_t v = v0 + lane;
            uint64_t dig;
            const uint32_t L = gossip_ids(h, v, gb, n_gb, dig);
            if (L > 0) {  // emitGossip returns early on an empty list, drawing nothing
                if (!staged || L > (uint32_t)h.gp.max_ihave) {
                    h.long_nodes[atomicAdd(h.n_long, 1u)] = v;  // one wave per node: k_hb_gossip_long
                } else {
                    const uint32_t o = (uint32_t)(rs[lane] - pa);
                    const int deg = (int)(rs[lane + 1] - rs[lane]);
                    uint16_t* peers = pl + o;
                    int np = 0;
                    for (int i = 0; i < deg; ++i)
                        if (el[o + i]) peers[np++] = (uint16_t)i;
                    int target = h.gp.d_lazy;
                    const int factor = (int)(h.gp.gossip_factor * (double)np);
                    if (factor > target) target = factor;
                    const bool shuffle_peers = target <= np;
                    if (!shuffle_peers) target = np;
                    if (target > 0) {
                        if (shuffle_peers) {  // an untruncated list is not shuffled (its order is never observable)
                            Rng g = hb_rng(h, v, t, h.rngk[(size_t)t * h.n_nodes + v]);
                            g.shuffle(peers, np);
                        }
                        // the unit's list once (a lane per node: coalesced), a byte per target
                        h.ihave_unit[((size_t)(h.fan_mode ? s.n_topics : 0) + t) * h.n_nodes + v] =
                            IhaveSlot{dig, L, h.ihave_cur};
                        const uint8_t tg = (uint8_t)(h.ihave_cur8 | (h.fan_mode ? IHAVE_FAN : 0));
                        for (int q = 0; q < target; ++q) {
                            h.ihave_tag[tslot + rs[lane] + peers[q]] = tg;
                            ihave_mark(h, (uint64_t)(rs[lane] + peers[q]), t);  // (D) reads it
                        }
                        cnt[0] += (uint64_t)target;
                        cnt[1] += (uint64_t)target * L;
                    }
                }
            }
        }
        __syncthreads();  // rs / el / pl are rewritten by the next tile
    }
    const uint32_t slot[2] = {HB_IHAVE_MSGS, HB_IHAVE_IDS};
    block_count<2>(cnt, h.stats, slot);
}

// ---- lists longer than MaxIHaveLength: one wave per queued node -------------

// The r-th (0-based) set bit of w (r < popcount(w)).
__device__ __forceinline__ uint32_t select64(uint64_t w, uint32_t r) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t sh = 32; sh > 0; sh >>= 1) {
        const uint32_t c = (uint32_t)__popcll(w & ((1ull << sh) - 1));
        if (r >= c) {
            r -= c;
            w >>= sh;
            pos += sh;
        }
    }
    return pos;
}

// Position -> row bit in a node's gossip list: the list is the set bits of
// row[0 .. tw) in order (GetGossipIDs order), pre[w] the bits before word w.
__device__ __forceinline__ uint32_t list_bit(const uint64_t* row, const uint32_t* pre, uint32_t tw, uint32_t pos) {
    uint32_t lo = 0, hi = tw;  // pre[lo] <= pos, and pos < pre[hi] (pre[tw] = L, never read)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (pre[mid] <= pos) lo = mid;
        else hi = mid;
    }
    return lo * 64 + select64(row[lo], pos - pre[lo]);
}

// Floyd's sampling of kk of the list's L positions (gsx.h, truncated IHAVE
// lists): for j = L - kk .. L - 1, x = Int31n(j + 1) (Go's rejection rule),
// take x unless already taken, then j.  The chosen positions' row bits are
// set in sel (zeroed first).  64 steps at a time: one draw per lane (a
// ballot resolves rejections, as in Go a rejected draw is redrawn with the
// next counter); then in step order each step's outcome is final and is
// broadcast to the later lanes, whose x it may take.
__device__ void wave_floyd(uint64_t* sel, const uint64_t* row, const uint32_t* pre, uint32_t tw, uint32_t L,
                           uint32_t kk, Rng g, uint32_t lane) {
    for (uint32_t w = lane; w < tw; w += 64) sel[w] = 0;
    wave_lds_sync();
    uint32_t i = 0;
    while (i < kk) {
        const uint32_t step = i + lane;
        const bool valid = step < kk;
        const uint32_t j = L - kk + step;
        const uint32_t n = j + 1;
        const int32_t x = (int32_t)(h4(g.seed, g.tag, g.vertex, g.base | (g.k + lane)) >> 33);
        const bool pow2 = (n & (n - 1)) == 0;
        const int32_t maxv = pow2 ? 0 : (int32_t)((1u << 31) - 1 - (1u << 31) % n);
        const bool rej = valid && !pow2 && x > maxv;
        const uint64_t rb = __ballot(rej);
        const uint32_t l0 = rb ? (uint32_t)__builtin_ctzll(rb) : 64u;
        const uint32_t nvalid = l0 < kk - i ? l0 : kk - i;
        const bool act = lane < nvalid;
        uint32_t bx = 0xFFFFFFFFu, bj = 0xFFFFFFFEu;
        bool hit = false;
        if (act) {
            const uint32_t xv = pow2 ? ((uint32_t)x & (n - 1)) : ((uint32_t)x % n);
            bx = list_bit(row, pre, tw, xv);
            bj = list_bit(row, pre, tw, j);
            hit = (sel[bx / 64] >> (bx % 64)) & 1;
        }
        for (uint32_t q = 0; q < nvalid; ++q) {
            const uint32_t y = __shfl(hit ? bj : bx, (int)q, 64);
            if (lane > q && y == bx) hit = true;
        }
        if (act) {
            const uint32_t y = hit ? bj : bx;
            atomicOr(reinterpret_cast<unsigned long long*>(&sel[y / 64]), 1ull << (y % 64));
        }
        wave_lds_sync();
        if (l0 < 64) {  // step i + l0 redraws after its rejected draw
            i += l0;
            g.k += l0 + 1;
        } else {
            i += nvalid;
            g.k += nvalid;
        }
    }
}

// One wave per queued node: lists longer than MaxIHaveLength, and nodes of
// tiles whose rows did not fit the stage.  Dynamic LDS: the node's gossip
// row (tw u64: its cache bits of the topic's batches at their row_off), the
// Floyd marks (tw u64), the row's prefix counts (tw u32), then the eligible
// peers (max_deg u16).  Each target of a truncated list gets the subset of
// Floyd's sampling over its own draw stream h(seed, 13, node << 32 | peer,
// tick << 32 | topic << 24 | fan << 23 | k): the marked positions when
// min(MaxIHaveLength, L - MaxIHaveLength) == MaxIHaveLength, else the
// unmarked ones; with the exchange on, its row goes to the topic's GxSub.
__global__ __launch_bounds__(64) void k_hb_gossip_long(DevState s, HbState h, uint32_t t,
                                                       const GossipBatch* __restrict__ gb, uint32_t n_gb,
                                                       uint32_t tw) {
    extern __shared__ uint64_t lds_long[];
    uint64_t* row = lds_long;
    uint64_t* sel = row + tw;
    uint32_t* pre = reinterpret_cast<uint32_t*>(sel + tw);
    uint16_t* peers = reinterpret_cast<uint16_t*>(pre + tw + (tw & 1));
    __shared__ uint32_t kshare;
    const uint32_t lane = threadIdx.x;
    const uint32_t n_long = *h.n_long;
    const size_t tslot = (size_t)t * h.n_pairs;
    const uint32_t slot0 = gb[0].slot_base;
    const uint32_t maxl = (uint32_t)h.gp.max_ihave;
    uint64_t msgs = 0, ids = 0;
    for (uint32_t li = blockIdx.x; li < n_long; li += gridDim.x) {
        const uint32_t v = h.long_nodes[li];
        uint64_t dall;
        const uint32_t L = gossip_ids(h, v, gb, n_gb, dall);  // GetGossipIDs: length and digest (k_mc_summary)
        Rng g = hb_rng(h, v, t, h.rngk[(size_t)t * h.n_nodes + v]);
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
        wave_lds_sync();
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
            wave_lds_sync();
            g.k = kshare;
        }
        if (L <= maxl) {  // the whole list to every target
            for (int p = lane; p < target; p += 64) {
                const int64_t r = r0 + peers[p];
                h.ihave_slot[tslot + r] = IhaveSlot{dall, L, h.ihave_cur};
                h.ihave_tag[tslot + r] = (uint8_t)(h.ihave_cur8 | IHAVE_OWN);
                ihave_mark(h, (uint64_t)r, t);  // (D) reads it
            }
            msgs += (uint64_t)target;
            ids += (uint64_t)target * L;
        } else if (target > 0) {
            // the node's gossip row and its prefix counts
            for (uint32_t b = 0; b < n_gb; ++b) {
                const GossipBatch B = gb[b];
                for (uint32_t w = lane; w < B.n_words; w += 64) row[B.row_off + w] = B.seen[(size_t)v * B.n_words + w];
            }
            wave_lds_sync();
            uint32_t carry = 0;
            for (uint32_t w0 = 0; w0 < tw; w0 += 64) {
                const uint32_t w = w0 + lane;
                const uint32_t c = w < tw ? (uint32_t)__popcll(row[w]) : 0u;
                const uint32_t p = wave_prefix(c, lane);
                if (w < tw) pre[w] = carry + p;
                carry += __shfl(p + c, 63, 64);
            }
            wave_lds_sync();
            const uint32_t kk = maxl < L - maxl ? maxl : L - maxl;
            const bool take = kk == maxl;  // the marked positions are the list, else the unmarked ones
            for (int p = 0; p < target; ++p) {
                const int64_t r = r0 + peers[p];
                const Rng gs{h.seed, TAG_IHAVE_SUB, ((uint64_t)(h.node_lo + v) << 32) | (uint32_t)h.col[r],
                             (h.tick << 32) | ((uint64_t)t << 24) | (h.fan_mode ? (1ull << 23) : 0ull), 0};
                wave_floyd(sel, row, pre, tw, L, kk, gs, lane);
                uint64_t d = 0;
                for (uint32_t w = lane; w < tw; w += 64)
                    for (uint64_t m = sel[w]; m; m &= m - 1) d += h.mc_digest[slot0 + w * 64 + (uint32_t)__builtin_ctzll(m)];
                d = wave_sum64(d);
                const uint32_t q = h.ihave_bits ? h.rev[r] : NO_PAIR;
                if (lane == 0) {
                    h.ihave_slot[tslot + r] = IhaveSlot{take ? d : dall - d, maxl, h.ihave_cur};
                    h.ihave_tag[tslot + r] = (uint8_t)(h.ihave_cur8 | IHAVE_OWN);
                    ihave_mark(h, (uint64_t)r, t);
                }
                // the subset the receiver's handleIHave reads (D): marked at the
                // receiver's pair, or for a receiver on another range shard at the
                // sender's pair, whose cache rows travel masked with it (k_gxs_rows)
                if (q != NO_PAIR && h.gsub.pool && (!(q & HALO) || h.gxs_tro)) {
                    uint32_t x = 0;
                    if (lane == 0) {
                        x = atomicAdd(h.gsub.cnt, 1u);
                        if (x < h.gsub.cap) {
                            h.gsub.idx[r] = x;
                            if (q & HALO)
                                h.gxs_tro[r] |= 1ull << t;
                            else
                                h.ihave_tr[q] |= 1ull << t;
                        } else {
                            h.gx_err[0] = 1;  // (the host bounds the targets: never)
                        }
                    }
                    x = __shfl(x, 0, 64);
                    if (x < h.gsub.cap) {
                        uint64_t* dst = h.gsub.pool + (size_t)x * h.gsub.tw;
                        for (uint32_t w = lane; w < tw; w += 64) dst[w] = take ? sel[w] : (row[w] & ~sel[w]);
                    }
                }
                wave_lds_sync();  // sel is redrawn for the next target
            }
            msgs += (uint64_t)target;
            ids += (uint64_t)target * maxl;
        }
        wave_lds_sync();
    }
    if (lane == 0) {
        if (msgs) atomicAdd(&h.stats[HB_IHAVE_MSGS], (unsigned long long)msgs);
        if (ids) atomicAdd(&h.stats[HB_IHAVE_IDS], (unsigned long long)ids);
    }
}

// ---- (B) receivers -------------------------------------------------------------

// handlePrune at the owner of pair q for topic t (:811-843): the tracer's
// Prune, then the PRUNE's backoff, which travels in whole seconds (:1821).
// Returns whether it removed a mesh link.
__device__ __forceinline__ bool handle_prune(const DevState& s, const HbState& h, uint64_t q, uint32_t t) {
    const bool was = hb_in_mesh(s, q, t) && scored_topic(s, q, t);
    ev_prune(s, q, t);
    if (h.tr_hp) h.tr_hp[q] |= 1ull << t;  // tracer.Prune, :822
    const int64_t secs = h.gp.prune_backoff_ns / 1000000000LL;
    add_backoff(h, q, t, secs > 0 ? secs * 1000000000LL : h.gp.prune_backoff_ns);
    return was;
}

// The control a receiver u reads from the sender of its pair q (unsharded:
// only marked pairs carry any, and what is read is cleared, so the next round
// starts from zeros).  Returns false when there is nothing to handle.
__device__ __forceinline__ bool recv_control(const HbState& h, uint64_t q, bool write, uint32_t& r, uint64_t& grafts,
                                             uint64_t& prunes) {
    r = h.rev[q];  // r = (v -> u), the sender's pair
    if (r == NO_PAIR) return false;
    if (r & HALO) {  // v on another shard: its control bits came through the exchange
        grafts = h.halo_ctl[2 * (size_t)(r & ~HALO)];
        prunes = h.halo_ctl[2 * (size_t)(r & ~HALO) + 1];
    } else {
        const ulonglong2 c = reinterpret_cast<const ulonglong2*>(h.ctl)[r];
        grafts = c.x;
        prunes = c.y;
        if (write && !h.halo_ctl && !h.keep_ctl && (grafts | prunes))
            reinterpret_cast<ulonglong2*>(h.ctl)[r] = make_ulonglong2(0, 0);
    }
    return (grafts | prunes) != 0;
}


// Per-lane counters of (B).
struct RecvCounts {
    uint64_t accepted = 0, rejected = 0, penalties = 0, handled = 0;
    int64_t links = 0;
    __device__ void flush(const HbState& h) const {
        flush_count(h.stats, HB_ACCEPTED, accepted);
        flush_count(h.stats, HB_REJECTED, rejected);
        flush_count(h.stats, HB_PENALTIES, penalties);
        flush_count(h.stats, HB_PRUNES_HANDLED, handled);
        flush_count(h.stats, HB_MESH_LINKS, (uint64_t)links);
    }
};

// handleGraft then handlePrune (:718-843) of the control the peer of pair q
// (u -> v) sent u, AcceptFrom-gated (:582-593).  The caller walks u's senders
// in ascending order: the Dhi check reads the running mesh count.
__device__ __forceinline__ void recv_pair(const DevState& s, const HbState& h, uint32_t u, uint64_t q, bool write,
                                          RecvCounts& c) {
    uint32_t r;
    uint64_t grafts, prunes;
    if (!recv_control(h, q, write, r, grafts, prunes)) return;
    // doPX = false for this RPC's PRUNE answers (:721-781): a GRAFT of a topic u
    // has not joined, from a direct peer, inside the backoff or of a negative score
    bool nopx = h.sub && (grafts & ~h.sub[u]);
    if (h.sub) {  // GRAFT / PRUNE of a topic u has not joined: ignored (:727-733, :816-819)
        grafts &= h.sub[u];
        prunes &= h.sub[u];
        if (!(grafts | prunes)) return;
    }
    // gs.score.Score(p) once per control message (the cache holds the round's
    // state for every pair read here: the subset re-score of dirty && inbox after (A))
    const double score = s.score[q];
    const uint8_t ef = h.eflags[q];
    if (!(ef & EDGE_DIRECT) && score < h.graylist) return;
    h.dirty[q] = 1;  // its record may change below: re-scored before (C) reads it and at the end
    const DevGossipParams& gp = h.gp;
    uint64_t resp = 0;
    for (; grafts; grafts &= grafts - 1) {  // handleGraft, :718-809, topics ascending
        const uint32_t t = (uint32_t)__builtin_ctzll(grafts);
        if (hb_in_mesh(s, q, t)) continue;
        if (ef & EDGE_DIRECT) {
            resp |= 1ull << t;
            ++c.rejected;
            nopx = true;
            continue;
        }
        const int64_t expire = h.backoff[(size_t)t * h.n_pairs + q];
        if (expire != 0 && h.now < expire) {
            nopx = true;
            ev_penalty(s, q, 1);
            ++c.penalties;
            if (h.now < expire + (gp.graft_flood_threshold_ns - gp.prune_backoff_ns)) {
                ev_penalty(s, q, 1);
                ++c.penalties;
            }
            add_backoff(h, q, t, gp.prune_backoff_ns);
            resp |= 1ull << t;
            ++c.rejected;
            continue;
        }
        if (score < 0) {
            resp |= 1ull << t;
            add_backoff(h, q, t, gp.prune_backoff_ns);
            ++c.rejected;
            nopx = true;
            continue;
        }
        // the mesh size (A) left, kept current by this receiver's accepts and prunes
        uint16_t* mc = h.mcount + (size_t)t * h.n_nodes + u;
        if (*mc >= gp.d_hi && !(ef & EDGE_OUTBOUND)) {
            resp |= 1ull << t;
            add_backoff(h, q, t, gp.prune_backoff_ns);
            ++c.rejected;
            continue;
        }
        ev_graft(s, q, t, h.now);
        if (h.tr_acc) h.tr_acc[q] |= 1ull << t;  // tracer.Graft, :795
        ++c.accepted;
        if (scored_topic(s, q, t)) {
            ++c.links;
            *mc = (uint16_t)(*mc + 1);
        }
    }
    h.resp[q] = resp;
    if (resp && !(r & HALO)) h.answer[r] = 1;  // the GRAFT sender has an answer to read in (C)
    if (h.pxno && nopx) h.pxno[q] |= 2;
    for (; prunes; prunes &= prunes - 1) {  // handlePrune
        const uint32_t t = (uint32_t)__builtin_ctzll(prunes);
        if (handle_prune(s, h, q, t)) {
            --c.links;
            h.mcount[(size_t)t * h.n_nodes + u] -= 1;
        }
        ++c.handled;
    }
}

// (B) one lane per receiving node u (up to HB_LANE_DEG peers; hubs run in
// k_hb_recv_hub), senders in ascending order: handleGraft then handlePrune
// per sender (:718-843), AcceptFrom-gated (:582-593).  The Dhi check reads
// the mesh size the previous accepts and prunes of this round left: a
// running count per topic, taken from the row on first use.
__global__ __launch_bounds__(64) void k_hb_recv(DevState s, HbState h) {
    const uint32_t lane = threadIdx.x;
    const bool clear = !hb_bulk_round(h.stats[HB_GRAFTS], h.stats[HB_PRUNES], h.n_pairs);
    RecvCounts c;
    for (uint32_t u = blockIdx.x * 64u + lane; u < h.n_nodes; u += gridDim.x * 64u) {
        const int64_t r0 = h.row_ptr[u], r1 = h.row_ptr[u + 1];
        if (r1 - r0 > HB_LANE_DEG) continue;  // k_hb_recv_hub
        for (int64_t c0 = r0; c0 < r1; c0 += 8) {
          // the row's marks eight at a time, loaded unconditionally (clamped)
          uint8_t ib[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) ib[j] = h.inbox[min(c0 + j, r1 - 1)];
          for (int j = 0; j < 8 && c0 + j < r1; ++j) {
            const int64_t q = c0 + j;  // q = (u -> v), ascending v
            if (!h.halo_ctl) {
                if (!ib[j]) continue;
                h.inbox[q] = 0;
            }
            recv_pair(s, h, u, (uint64_t)q, clear, c);
          }
        }
    }
    c.flush(h);
}

// (B) pair-parallel: RG lanes per receiving node u (up to HB_LANE_DEG peers),
// one lane per sender pair, the row RG pairs at a time.  Everything handleGraft
// / handlePrune (:718-843) does to one pair — its control words, AcceptFrom,
// the direct / backoff / negative-score rejections with their penalties and
// backoffs, the tracer bits, the records — belongs to that pair alone, so the
// lanes do it side by side with coalesced per-pair loads.  The one thing the
// senders share is the Dhi check (:786-795): a non-outbound GRAFT is refused
// once the mesh holds Dhi peers, and the mesh size is what the earlier senders'
// accepts and prunes left.  The group resolves that recurrence per topic over
// its lanes in ascending pair order, on a 5-bit code per lane (candidate,
// outbound, scored, PRUNE, in the mesh before) moved by shuffles, then every
// lane applies its own outcome.  Bit-identical to the sequential walk.
constexpr int RG = 16;
enum : uint32_t { RC_CAND = 1, RC_OUT = 2, RC_SC = 4, RC_PR = 8, RC_INM = 16 };

__global__ __launch_bounds__(256) void k_hb_recv_grp(DevState s, HbState h) {
    const uint32_t lane = threadIdx.x % 64;
    const uint32_t gl = lane % RG;         // the lane's place in its node's group
    const uint32_t gbase = lane & ~(RG - 1);  // the group's first lane in the wave
    const uint32_t grp = lane / RG;
    const DevGossipParams& gp = h.gp;
    RecvCounts c;
    const uint32_t wave = blockIdx.x * 4u + threadIdx.x / 64u, n_waves = gridDim.x * 4u;
    // (a bulk round's control words are cleared at the next round's start)
    const bool clear = !hb_bulk_round(h.stats[HB_GRAFTS], h.stats[HB_PRUNES], h.n_pairs);
    for (uint32_t tile = wave * 64u; tile < h.n_nodes; tile += n_waves * 64u) {
      // which of the tile's 64 nodes received control: a lane scans each row's
      // marks (eight at a time, clamped); hubs run in k_hb_recv_hub
      bool act = false;
      {
        const uint32_t un = tile + lane;
        if (un < h.n_nodes) {
            const int64_t a0 = h.row_ptr[un], a1 = h.row_ptr[un + 1];
            if (a1 > a0 && a1 - a0 <= HB_LANE_DEG) {
                if (h.halo_ctl) {
                    act = true;
                } else {
                    for (int64_t c0 = a0; c0 < a1 && !act; c0 += 8) {
                        uint8_t ib[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) ib[j] = h.inbox[min(c0 + j, a1 - 1)];
#pragma unroll
                        for (int j = 0; j < 8; ++j) act |= ib[j] != 0;
                    }
                }
            }
        }
      }
      // the active nodes, 64 / RG at a time: group g takes the g-th
      for (uint64_t mask = __ballot(act); mask;) {  // (wave-uniform)
        uint64_t mm = mask;
        for (uint32_t i = 0; i < grp; ++i) mm &= mm - 1;
#pragma unroll
        for (uint32_t i = 0; i < 64u / RG; ++i) mask &= mask - 1;
        if (!mm) continue;  // (group-uniform)
        const uint32_t u = tile + (uint32_t)__builtin_ctzll(mm);
        const int64_t r0 = h.row_ptr[u], r1 = h.row_ptr[u + 1];
        for (int64_t c0 = r0; c0 < r1; c0 += RG) {  // group-uniform
            const int64_t q = c0 + gl;  // q = (u -> v), ascending v
            bool live = false, nopx = false, outb = false;
            uint32_t r = NO_PAIR;
            uint64_t cand = 0, prn = 0, inm = 0, scd = 0, resp = 0;
            // unsharded, only marked pairs carry control: a chunk without one is done
            const bool act = q < r1 && (h.halo_ctl || h.inbox[q] != 0);
            if (!((__ballot(act) >> gbase) & ((1ull << RG) - 1))) continue;  // (group-uniform)
            if (act) {
                if (!h.halo_ctl) h.inbox[q] = 0;
                uint64_t grafts = 0, prunes = 0;
                if (act && recv_control(h, (uint64_t)q, clear, r, grafts, prunes)) {
                    nopx = h.sub && (grafts & ~h.sub[u]);  // doPX = false (:721-781)
                    if (h.sub) {  // topics u has not joined: ignored (:727-733, :816-819)
                        grafts &= h.sub[u];
                        prunes &= h.sub[u];
                    }
                    const double score = (grafts | prunes) ? s.score[q] : 0.0;
                    const uint8_t ef = (grafts | prunes) ? h.eflags[q] : 0;
                    if ((grafts | prunes) && ((ef & EDGE_DIRECT) || !(score < h.graylist))) {
                        live = true;
                        h.dirty[q] = 1;
                        outb = ef & EDGE_OUTBOUND;
                        for (; grafts; grafts &= grafts - 1) {  // handleGraft up to the Dhi check
                            const uint32_t t = (uint32_t)__builtin_ctzll(grafts);
                            if (hb_in_mesh(s, q, t)) continue;
                            if (ef & EDGE_DIRECT) {
                                resp |= 1ull << t;
                                ++c.rejected;
                                nopx = true;
                                continue;
                            }
                            const int64_t expire = h.backoff[(size_t)t * h.n_pairs + q];
                            if (expire != 0 && h.now < expire) {
                                nopx = true;
                                ev_penalty(s, q, 1);
                                ++c.penalties;
                                if (h.now < expire + (gp.graft_flood_threshold_ns - gp.prune_backoff_ns)) {
                                    ev_penalty(s, q, 1);
                                    ++c.penalties;
                                }
                                add_backoff(h, q, t, gp.prune_backoff_ns);
                                resp |= 1ull << t;
                                ++c.rejected;
                                continue;
                            }
                            if (score < 0) {
                                resp |= 1ull << t;
                                add_backoff(h, q, t, gp.prune_backoff_ns);
                                ++c.rejected;
                                nopx = true;
                                continue;
                            }
                            cand |= 1ull << t;
                        }
                        prn = prunes;
                        for (uint64_t m = cand | prn; m; m &= m - 1) {
                            const uint32_t t = (uint32_t)__builtin_ctzll(m);
                            if (scored_topic(s, q, t)) scd |= 1ull << t;
                            if ((prn >> t & 1) && hb_in_mesh(s, q, t)) inm |= 1ull << t;
                        }
                    }
                }
            }
            // the Dhi recurrence, per topic any lane of the group has an event for
            uint64_t any = cand | prn;
#pragma unroll
            for (int off = RG / 2; off > 0; off >>= 1) any |= __shfl_xor(any, off, RG);
            uint64_t acc = 0;
            for (; any; any &= any - 1) {  // group-uniform
                const uint32_t t = (uint32_t)__builtin_ctzll(any);
                const uint32_t code = (uint32_t)(cand >> t & 1) * RC_CAND | (outb ? RC_OUT : 0u) |
                                      (uint32_t)(scd >> t & 1) * RC_SC | (uint32_t)(prn >> t & 1) * RC_PR |
                                      (uint32_t)(inm >> t & 1) * RC_INM;
                const bool ev = code & (RC_CAND | RC_PR);
                uint32_t lanes = (uint32_t)((__ballot(ev) >> gbase) & ((1ull << RG) - 1));
                uint16_t* mcp = h.mcount + (size_t)t * h.n_nodes + u;
                const int n0 = *mcp;
                int n = n0;
                for (; lanes; lanes &= lanes - 1) {
                    const uint32_t j = (uint32_t)__builtin_ctz(lanes);
                    const uint32_t cj = (uint32_t)__shfl((int)code, (int)j, RG);
                    const bool a = (cj & RC_CAND) && ((cj & RC_OUT) || n < gp.d_hi);
                    if (a && (cj & RC_SC)) ++n;
                    if ((cj & RC_PR) && (cj & RC_SC) && ((cj & RC_INM) || a)) --n;
                    if (gl == j && a) acc |= 1ull << t;
                }
                if (gl == 0 && n != n0) *mcp = (uint16_t)n;
            }
            __threadfence_block();  // the next chunk's lanes read the counts written here
            if (!live) continue;
            for (uint64_t m = cand; m; m &= m - 1) {
                const uint32_t t = (uint32_t)__builtin_ctzll(m);
                if (acc >> t & 1) {
                    ev_graft(s, q, t, h.now);
                    if (h.tr_acc) h.tr_acc[q] |= 1ull << t;  // tracer.Graft, :795
                    ++c.accepted;
                    if (scd >> t & 1) ++c.links;
                } else {  // the mesh is full (Dhi)
                    resp |= 1ull << t;
                    add_backoff(h, q, t, gp.prune_backoff_ns);
                    ++c.rejected;
                }
            }
            h.resp[q] = resp;
            if (resp && !(r & HALO)) h.answer[r] = 1;  // the GRAFT sender has an answer to read in (C)
            if (h.pxno && nopx) h.pxno[q] |= 2;
            for (uint64_t m = prn; m; m &= m - 1) {  // handlePrune
                if (handle_prune(s, h, q, (uint32_t)__builtin_ctzll(m))) --c.links;
                ++c.handled;
            }
        }
      }
    }
    c.flush(h);
}

// (B) for hub receivers (more than HB_LANE_DEG peers): one wave per node.
// The wave finds the marked pairs 64 at a time (ballot); every lane then runs
// the same sequential handling of each sender in ascending order (its values
// are uniform across the wave), lane 0 writing, and mesh sizes are counted by
// the whole wave.
__global__ __launch_bounds__(64) void k_hb_recv_hub(DevState s, HbState h) {
    const uint32_t lane = threadIdx.x;
    const bool bulk = hb_bulk_round(h.stats[HB_GRAFTS], h.stats[HB_PRUNES], h.n_pairs);
    const bool w0 = lane == 0;
    uint64_t accepted = 0, rejected = 0, penalties = 0, handled = 0;
    int64_t links = 0;
    const DevGossipParams& gp = h.gp;
    for (uint32_t k = blockIdx.x; k < h.n_hubs; k += gridDim.x) {
        const uint32_t u = h.hubs[k];
        const int64_t r0 = h.row_ptr[u], r1 = h.row_ptr[u + 1];
        for (int64_t c0 = r0; c0 < r1; c0 += 64) {
            const int64_t ql = c0 + lane;
            bool mine = ql < r1;
            if (mine && !h.halo_ctl) mine = h.inbox[ql] != 0;
            uint64_t mask = __ballot(mine);
            __syncthreads();  // every lane has read its inbox byte before lane 0 clears any
            for (; mask; mask &= mask - 1) {
                const uint64_t q = (uint64_t)c0 + (uint32_t)__builtin_ctzll(mask);
                if (!h.halo_ctl && w0) h.inbox[q] = 0;
                uint32_t r;
                uint64_t grafts, prunes;
                if (!recv_control(h, q, false, r, grafts, prunes)) continue;
                __syncthreads();  // every lane has the words before lane 0 clears them
                if (w0 && !(r & HALO) && !h.halo_ctl && !h.keep_ctl && !bulk)
                    reinterpret_cast<ulonglong2*>(h.ctl)[r] = make_ulonglong2(0, 0);
                bool nopx = h.sub && (grafts & ~h.sub[u]);  // doPX = false (:721-781)
                if (h.sub) {  // topics u has not joined: ignored (:727-733, :816-819)
                    grafts &= h.sub[u];
                    prunes &= h.sub[u];
                    if (!(grafts | prunes)) continue;
                }
                const double score = s.score[q];
                const uint8_t ef = h.eflags[q];
                if (!(ef & EDGE_DIRECT) && score < h.graylist) continue;
                if (w0) h.dirty[q] = 1;
                uint64_t resp = 0;
                for (; grafts; grafts &= grafts - 1) {
                    const uint32_t t = (uint32_t)__builtin_ctzll(grafts);
                    if (hb_in_mesh(s, q, t)) continue;
                    if (ef & EDGE_DIRECT) {
                        resp |= 1ull << t;
                        rejected += w0;
                        nopx = true;
                        continue;
                    }
                    const int64_t expire = h.backoff[(size_t)t * h.n_pairs + q];
                    if (expire != 0 && h.now < expire) {
                        nopx = true;
                        const bool twice = h.now < expire + (gp.graft_flood_threshold_ns - gp.prune_backoff_ns);
                        if (w0) {
                            ev_penalty(s, q, 1);
                            if (twice) ev_penalty(s, q, 1);
                            add_backoff(h, q, t, gp.prune_backoff_ns);
                        }
                        penalties += w0 ? (twice ? 2 : 1) : 0;
                        resp |= 1ull << t;
                        rejected += w0;
                        __syncthreads();
                        continue;
                    }
                    if (score < 0) {
                        resp |= 1ull << t;
                        if (w0) add_backoff(h, q, t, gp.prune_backoff_ns);
                        rejected += w0;
                        nopx = true;
                        __syncthreads();
                        continue;
                    }
                    uint16_t* mcp = h.mcount + (size_t)t * h.n_nodes + u;
                    const int n = *mcp;
                    __syncthreads();  // every lane has read the count before lane 0 updates it
                    if (n >= gp.d_hi && !(ef & EDGE_OUTBOUND)) {
                        resp |= 1ull << t;
                        if (w0) add_backoff(h, q, t, gp.prune_backoff_ns);
                        rejected += w0;
                        __syncthreads();
                        continue;
                    }
                    const bool sc_t = scored_topic(s, q, t);
                    __syncthreads();  // every lane has read the flags before lane 0 grafts
                    if (w0) {
                        ev_graft(s, q, t, h.now);
                        if (h.tr_acc) h.tr_acc[q] |= 1ull << t;  // tracer.Graft, :795
                        if (sc_t) *mcp = (uint16_t)(n + 1);
                    }
                    accepted += w0;
                    if (sc_t) links += w0;
                    __syncthreads();
                }
                if (w0) {
                    h.resp[q] = resp;
                    if (resp && !(r & HALO)) h.answer[r] = 1;
                    if (h.pxno && nopx) h.pxno[q] |= 2;
                }
                for (; prunes; prunes &= prunes - 1) {
                    const uint32_t t = (uint32_t)__builtin_ctzll(prunes);
                    const bool was = hb_in_mesh(s, q, t) && scored_topic(s, q, t);
                    __syncthreads();
                    if (w0) {
                        handle_prune(s, h, q, t);
                        if (was) h.mcount[(size_t)t * h.n_nodes + u] -= 1;
                    }
                    if (was) links -= w0;
                    handled += w0;
                    __syncthreads();
                }
            }
        }
    }
    flush_count(h.stats, HB_ACCEPTED, accepted);
    flush_count(h.stats, HB_REJECTED, rejected);
    flush_count(h.stats, HB_PENALTIES, penalties);
    flush_count(h.stats, HB_PRUNES_HANDLED, handled);
    flush_count(h.stats, HB_MESH_LINKS, (uint64_t)links);
}

// ---- (C) the GRAFT senders handle the PRUNE answers ------------------------------

__global__ __launch_bounds__(256) void k_hb_answer(DevState s, HbState h) {
    uint64_t handled = 0;
    int64_t links = 0;
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
        if (resp && h.sub) resp &= h.sub[h.pair_obs[r]];  // (a PRUNE of a topic v left: ignored)
        if (resp) h.dirty[r] = 1;
        for (; resp; resp &= resp - 1) {
            if (handle_prune(s, h, r, (uint32_t)__builtin_ctzll(resp))) --links;
            ++handled;
        }
    }
    flush_count(h.stats, HB_PRUNES_HANDLED, handled);
    flush_count(h.stats, HB_MESH_LINKS, (uint64_t)links);
}

// Shard exchange of per-pair control words: send slot j carries the words of
// the local pair send_pair[j] (0 for NO_PAIR), K words per slot.
__global__ __launch_bounds__(256) void k_hb_pack(const uint32_t* __restrict__ send_pair, uint64_t n_send,
                                                 uint32_t stride, const uint64_t* __restrict__ a,
                                                 const uint64_t* __restrict__ b, uint64_t* __restrict__ out) {
    const int K = b ? 2 : 1;
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < n_send; j += (uint64_t)gridDim.x * 256u) {
        const uint32_t r = send_pair[j];
        out[K * j] = r == NO_PAIR ? 0 : a[(size_t)stride * r];
        if (b) out[K * j + 1] = r == NO_PAIR ? 0 : b[(size_t)stride * r];
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

// Every span: the bytes before the first 16-B boundary, 16-B stores, the tail.
__global__ __launch_bounds__(256) void k_zero_spans(ZeroSpans z) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256u + threadIdx.x, stride = (uint64_t)gridDim.x * 256u;
    for (uint32_t j = 0; j < z.k; ++j) {
        uint8_t* p = z.p[j];
        const uint64_t n = z.n[j];
        uint64_t head = (16u - ((uintptr_t)p & 15u)) & 15u;
        head = head < n ? head : n;
        if (tid < head) p[tid] = 0;
        uint4* v = reinterpret_cast<uint4*>(p + head);
        const uint64_t nv = (n - head) / 16;
        for (uint64_t i = tid; i < nv; i += stride) v[i] = make_uint4(0u, 0u, 0u, 0u);
        const uint64_t done = head + 16 * nv;
        if (tid < n - done) p[done + tid] = 0;
    }
}
hipError_t launch_zero_spans(const ZeroSpans& z, hipStream_t st) {
    uint64_t most = 0;
    for (uint32_t j = 0; j < z.k; ++j) most = z.n[j] > most ? z.n[j] : most;
    if (most == 0) return hipSuccess;
    uint64_t b = (most / 16 + 1023) / 1024;  // ~4 stores per lane on the largest span
    b = b < 1 ? 1 : b > 8192 ? 8192 : b;
    hipLaunchKernelGGL(k_zero_spans, dim3((unsigned)b), dim3(256), 0, st, z);
    return hipGetLastError();
}

hipError_t launch_hb_clear_backoff(const HbState& h, uint32_t n_topics, hipStream_t st) {
    const uint64_t n = (uint64_t)((n_topics + 7) / 8) * h.n_pairs;  // a lane per presence byte
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_clear_backoff, dim3(grid_cap(n, 256)), dim3(256), 0, st, h, n_topics);
    return hipGetLastError();
}

hipError_t launch_bo_rebuild(const int64_t* backoff, uint8_t* bo8, uint64_t n_pairs, uint32_t n_topics,
                             hipStream_t st) {
    const uint64_t n = (uint64_t)((n_topics + 7) / 8) * n_pairs;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_bo_rebuild, dim3(grid_cap(n, 256)), dim3(256), 0, st, backoff, bo8, n_pairs, n_topics);
    return hipGetLastError();
}

hipError_t launch_hb_scan(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_nodes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_scan, dim3(grid_cap(h.n_nodes, 256)), dim3(256), 0, st, s, h);  // a tile per wave
    return hipGetLastError();
}

hipError_t launch_hb_maintain(const DevState& s, const HbState& h, uint32_t t_base, uint32_t n_t, int64_t max_deg,
                              hipStream_t st) {
    if (h.n_nodes == 0 || n_t == 0) return hipSuccess;
    // a wave per group of MAINT_GROUP tiles (the per-tile lists of k_hb_scan), blockIdx.y the topic
    const uint64_t groups = ((uint64_t)h.n_nodes + 64 * MAINT_GROUP - 1) / (64 * MAINT_GROUP);
    // (≈ 8192 waves over the run: one resident round; a wave loops over groups)
    hipLaunchKernelGGL(k_hb_maintain, dim3((unsigned)std::min<uint64_t>(groups, std::max(8192u / n_t, 256u)), n_t),
                       dim3(64), 0, st, s, h, t_base);
    if (max_deg > HB_LANE_DEG) {
        const size_t lds = (size_t)max_deg * (sizeof(double) + 2 * sizeof(uint16_t) + 1);
        static bool attr = false;
        if (!attr) {
            hipError_t e = hipFuncSetAttribute((const void*)k_hb_maintain_hub, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)(HB_HUB_MAX * (sizeof(double) + 2 * sizeof(uint16_t) + 1)));
            if (e != hipSuccess) return e;
            attr = true;
        }
        hipLaunchKernelGGL(k_hb_maintain_hub, dim3(1024, n_t), dim3(64), lds, st, s, h, t_base);
    }
    return hipGetLastError();
}

hipError_t launch_hb_gelig(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_gelig, dim3((unsigned)std::min<uint64_t>((h.n_pairs + 255) / 256, 8192)), dim3(256), 0, st,
                       s, h);
    return hipGetLastError();
}
hipError_t launch_hb_gossip(const DevState& s, const HbState& h, uint32_t t, const GossipBatch* gb, uint32_t n_gb,
                            uint32_t tw, int64_t max_deg, hipStream_t st) {
    if (h.n_nodes == 0 || n_gb == 0 || tw == 0) return hipSuccess;
    hipError_t e = hipSuccess;  // (h.n_long: the topic's counter, cleared at the round's start)
    hipLaunchKernelGGL(k_hb_gossip, dim3(grid_cap(h.n_nodes, 256)), dim3(256), 0, st, s, h, t, gb, n_gb);
    // queued nodes (long lists, tiles with hub rows): the kernel returns at once without any
    const size_t lds = (size_t)tw * 20 + 4 + sizeof(uint16_t) * (size_t)std::max<int64_t>(max_deg, 1);
    static size_t attr = 0;
    if (lds > 65536 && lds > attr) {
        e = hipFuncSetAttribute((const void*)k_hb_gossip_long, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = lds;
    }
    hipLaunchKernelGGL(k_hb_gossip_long, dim3(grid_cap(h.n_nodes, 1)), dim3(64), lds, st, s, h, t, gb, n_gb, tw);
    return hipGetLastError();
}

hipError_t launch_hb_recv(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_nodes == 0) return hipSuccess;
    // GSX_HB_RECV_LANE=1 selects the lane-per-receiver kernel (A/B measurement)
    static const bool lane_per_node = getenv("GSX_HB_RECV_LANE") != nullptr;
    if (lane_per_node)
        hipLaunchKernelGGL(k_hb_recv, dim3(wave_grid(h.n_nodes)), dim3(64), 0, st, s, h);
    else
        hipLaunchKernelGGL(k_hb_recv_grp, dim3(grid_cap((uint64_t)h.n_nodes * RG, 256)), dim3(256), 0, st, s, h);
    if (h.n_hubs) hipLaunchKernelGGL(k_hb_recv_hub, dim3(std::min<uint32_t>(h.n_hubs, 4096)), dim3(64), 0, st, s, h);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_mask_and(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                  uint8_t* __restrict__ out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
        out[i] = a[i] && b[i];
}
hipError_t launch_mask_and(const uint8_t* a, const uint8_t* b, uint8_t* out, uint64_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mask_and, dim3(grid_cap(n, 256)), dim3(256), 0, st, a, b, out, n);
    return hipGetLastError();
}

hipError_t launch_mc_summary(const uint64_t* seen, uint32_t n_nodes, uint32_t n_words, uint32_t n_msgs,
                             const uint64_t* msg_dig, const uint64_t* word_dig, uint64_t* dig, uint32_t* cnt,
                             hipStream_t st) {
    if (n_nodes == 0) return hipSuccess;
    const uint64_t nn = n_nodes;
    if (n_words % 16 == 0)
        hipLaunchKernelGGL(k_mc_summary<4>, dim3(grid_cap(4 * nn, 256)), dim3(256), 0, st, seen, n_nodes, n_words,
                           n_msgs, msg_dig, word_dig, dig, cnt);
    else if (n_words % 8 == 0)
        hipLaunchKernelGGL(k_mc_summary<2>, dim3(grid_cap(2 * nn, 256)), dim3(256), 0, st, seen, n_nodes, n_words,
                           n_msgs, msg_dig, word_dig, dig, cnt);
    else
        hipLaunchKernelGGL(k_mc_summary<1>, dim3(grid_cap(nn, 256)), dim3(256), 0, st, seen, n_nodes, n_words, n_msgs,
                           msg_dig, word_dig, dig, cnt);
    return hipGetLastError();
}

// The seen rows of a whole batch from its message blocks (message-parallel
// replicas, gsx_mcache_put): word w of node v holds the batch's messages
// [64w, 64w + 64); each block overlapping them contributes its bits, shifted
// from the block's own numbering.  A lane per (node, word), coalesced writes.
__global__ __launch_bounds__(256) void k_mc_merge(const McPart* __restrict__ parts, uint32_t n_parts,
                                                  uint64_t* __restrict__ dst, uint32_t n_nodes, uint32_t W) {
    const uint64_t n = (uint64_t)n_nodes * W;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const uint32_t v = (uint32_t)(i / W), w = (uint32_t)(i % W);
        const uint32_t g0 = 64u * w, g1 = g0 + 64u;
        uint64_t x = 0;
        for (uint32_t p = 0; p < n_parts; ++p) {
            const McPart P = parts[p];
            const uint32_t lo = max(g0, P.off), hi = min(g1, P.off + P.n);
            if (lo >= hi) continue;
            const uint32_t b0 = lo - P.off, wa = b0 / 64u, sa = b0 % 64u, len = hi - lo;
            const uint64_t* row = P.rows + (size_t)v * P.words;
            uint64_t bits = row[wa] >> sa;
            if (sa && wa + 1 < P.words) bits |= row[wa + 1] << (64u - sa);
            if (len < 64u) bits &= (1ull << len) - 1;
            x |= bits << (lo - g0);
        }
        dst[i] = x;
    }
}

hipError_t launch_mc_merge(const McPart* parts, uint32_t n_parts, uint64_t* dst, uint32_t n_nodes, uint32_t n_words,
                           hipStream_t st) {
    const uint64_t n = (uint64_t)n_nodes * n_words;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mc_merge, dim3(grid_cap(n, 256)), dim3(256), 0, st, parts, n_parts, dst, n_nodes, n_words);
    return hipGetLastError();
}

// ---- peer exchange on PRUNE (gossipsub.go:811-843, 861-910, 1814-1850) ----------

// One lane per pruning node u (kind 0: the (A) PRUNEs in ctl_prune, before
// (B) reads them; kind 1: the (B) answers in resp, before (C) reads them).
// makePrune's getPeers(topic, PrunePeers, xp != p && score(xp) >= 0): per
// pruned topic t of u, the candidates of u's row (ascending peer) are staged
// once in pxbase over u's own row range; every PRUNE of t copies them without
// its own peer into mscratch, shuffles with the draws of gsx.h and truncates.
// Then the receiver p's side: AcceptFrom, the joined-topic check of
// handlePrune, AcceptPXThreshold on its score of u, and pxConnect's "not
// connected" filter (p's row is sorted by peer: a binary search).  The scores
// are the cache as the receiving step reads it (gsx.h).  PX is off by
// default and this kernel runs only with do_px: candidates are logged with
// one L2 atomic each.
// pxConnect's candidates of one PX list at the receiver p (local node) of the
// pruner ug (global id): AcceptPXThreshold on its score of the pruner (pair q),
// then the peers p is not connected to (p's row is sorted by peer: a binary
// search; ids global on a shard).  Logs (p, candidate, pruner, topic | kind).
__device__ __forceinline__ void px_connect(const DevState& s, const HbState& h, uint32_t p, uint32_t ug, double rs,
                                           const uint32_t* ids, int n, uint32_t t, uint32_t kind, uint64_t& ignored,
                                           uint64_t& connect) {
    if (rs < h.accept_px) {  // :833-838
        ++ignored;
        return;
    }
    const int64_t p0 = h.row_ptr[p], p1 = h.row_ptr[p + 1];
    for (int i = 0; i < n; ++i) {  // pxConnect (:861-910): the peers p is not connected to
        const int32_t xp = (int32_t)ids[i];
        int64_t lo = p0, hi = p1;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (h.col[mid] < xp) lo = mid + 1;
            else hi = mid;
        }
        if (lo < p1 && h.col[lo] == xp && (s.pflags[lo] & PAIR_CONNECTED)) continue;
        if (h.px_log) {
            const unsigned long long k = atomicAdd(&h.stats[HB_PX_CONNECT], 1ull);
            if (k < h.px_cap) {
                uint32_t* o = h.px_log + 4 * k;
                o[0] = h.node_lo + p;
                o[1] = (uint32_t)xp;
                o[2] = ug;
                o[3] = t | (kind << 8);
            }
        } else {
            ++connect;
        }
    }
}

// Count pass of the shard exchange: the PX PRUNEs of cross-shard pairs whose
// peer tracks the pruner, per destination rank (one entry each).
__global__ __launch_bounds__(256) void k_hb_px_count(HbState h, uint32_t kind) {
    const uint8_t nobit = kind ? 2 : 1;
    for (uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x; r < h.n_pairs; r += (uint64_t)gridDim.x * 256u) {
        const uint64_t bits = kind ? h.resp[r] : h.ctl[2 * (size_t)r + 1];
        if (!bits || (h.pxno[r] & nobit) || (h.eflags[r] & EDGE_NO_PX)) continue;
        const uint32_t q = h.rev[r];
        if (q == NO_PAIR || !(q & HALO)) continue;
        const uint32_t j = h.send_slot[r];
        if (j == NO_PAIR) continue;
        atomicAdd(&h.pxs_cnt[h.send_dest[j]], (unsigned long long)__popcll(bits));
    }
}

// The receivers' side of the PX lists other ranks sent (one lane per entry).
__global__ __launch_bounds__(256) void k_hb_px_recv(DevState s, HbState h, const uint32_t* __restrict__ ent,
                                                    uint64_t n_ent) {
    uint64_t ignored = 0, connect = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n_ent; i += (uint64_t)gridDim.x * 256u) {
        const uint32_t* o = ent + i * h.pxs_w;
        const int n = (int)o[2];
        if (n <= 0) continue;
        const uint32_t t = o[1] & 0xFFu, kind = o[1] >> 8;
        const uint32_t q = h.halo_pair[o[0]];  // (p -> u): the receiver's pair
        const uint32_t p = h.pair_obs[q];
        const double rs = s.score[q];
        if (!(h.eflags[q] & EDGE_DIRECT) && rs < h.graylist) continue;  // AcceptFrom drops the RPC
        if (!joined_node(h.sub, p, t)) continue;                         // handlePrune never reads it (:816-819)
        px_connect(s, h, p, (uint32_t)h.col[q], rs, o + 3, n, t, kind, ignored, connect);
    }
    flush_count(h.stats, HB_PX_IGNORED, ignored);
    flush_count(h.stats, HB_PX_CONNECT, connect);
}

__global__ __launch_bounds__(64) void k_hb_px(DevState s, HbState h, uint32_t kind) {
    uint64_t lists = 0, listed = 0, ignored = 0, connect = 0;
    const uint8_t nobit = kind ? 2 : 1;
    for (uint32_t u = blockIdx.x * 64u + threadIdx.x; u < h.n_nodes; u += gridDim.x * 64u) {
        const int64_t r0 = h.row_ptr[u], r1 = h.row_ptr[u + 1];
        uint64_t any = 0;  // the topics some PRUNE of u carries a list for
        for (int64_t r = r0; r < r1; ++r) {
            const uint64_t bits = kind ? h.resp[r] : h.ctl[2 * (size_t)r + 1];
            if (!bits || (h.pxno[r] & nobit) || (h.eflags[r] & EDGE_NO_PX)) continue;
            any |= bits;
        }
        for (; any; any &= any - 1) {
            const uint32_t t = (uint32_t)__builtin_ctzll(any);
            int nb = 0;
            for (int64_t x = r0; x < r1; ++x) {  // getPeers' candidates of t, ascending peer
                if ((s.pflags[x] & (PAIR_PRESENT | PAIR_CONNECTED)) != (PAIR_PRESENT | PAIR_CONNECTED)) continue;
                if (!topic_peer(h.psub, (uint64_t)x, t) || !(h.eflags[x] & EDGE_GOSSIPSUB)) continue;
                if (!(s.score[x] >= 0.0)) continue;
                h.pxbase[r0 + nb++] = (uint32_t)(x - r0);
            }
            for (int64_t r = r0; r < r1; ++r) {  // r = (u -> p), a PRUNE of t with PX
                const uint64_t bits = kind ? h.resp[r] : h.ctl[2 * (size_t)r + 1];
                if (!((bits >> t) & 1) || (h.pxno[r] & nobit) || (h.eflags[r] & EDGE_NO_PX)) continue;
                const uint32_t q = h.rev[r];  // (p -> u): the receiver's pair (HALO: p on another shard)
                const uint32_t pg = (uint32_t)h.col[r];  // p's global id (= the local one unsharded)
                int n = 0;
                const uint32_t self = (uint32_t)(r - r0);
                for (int i = 0; i < nb; ++i) {
                    const uint32_t x = h.pxbase[r0 + i];
                    if (x != self) h.mscratch[r0 + n++] = x;  // xp != p
                }
                Rng g{h.seed, TAG_PX, ((uint64_t)(h.node_lo + u) << 32) | (uint64_t)pg,
                      (h.tick << 32) | ((uint64_t)t << 24) | ((uint64_t)kind << 23), 0};
                g.shuffle(h.mscratch + r0, n);
                if (n > h.gp.prune_peers) n = h.gp.prune_peers;
                if (q != NO_PAIR && (q & HALO)) {  // the list travels to p's rank (k_hb_px_recv there)
                    const uint32_t j = h.send_slot[r];
                    if (j != NO_PAIR) {  // (else p does not track u: nobody reads it)
                        const uint32_t d = h.send_dest[j];
                        const unsigned long long k = atomicAdd(&h.pxs_cnt[d], 1ull);
                        uint32_t* o = h.pxs_out + (size_t)(h.pxs_off[d] + k) * h.pxs_w;
                        o[0] = (uint32_t)(h.dest_halo_base[d] + (j - h.send_base[d]));
                        o[1] = t | (kind << 8);
                        o[2] = n > 0 ? (uint32_t)n : 0u;
                        for (int i = 0; i < n; ++i) o[3 + i] = (uint32_t)h.col[r0 + h.mscratch[r0 + i]];
                    }
                    if (n > 0) {
                        ++lists;
                        listed += (uint64_t)n;
                    }
                    continue;
                }
                if (n <= 0) continue;
                ++lists;
                listed += (uint64_t)n;
                if (q == NO_PAIR) continue;  // p does not track u
                const uint32_t p = pg - h.node_lo;
                const double rs = s.score[q];
                if (!(h.eflags[q] & EDGE_DIRECT) && rs < h.graylist) continue;  // AcceptFrom drops the RPC
                if (!joined_node(h.sub, p, t)) continue;  // handlePrune never reads it (:816-819)
                for (int i = 0; i < n; ++i) h.mscratch[r0 + i] = (uint32_t)h.col[r0 + h.mscratch[r0 + i]];
                px_connect(s, h, p, h.node_lo + u, rs, h.mscratch + r0, n, t, kind, ignored, connect);
            }
        }
        // (B) never reads nor clears the words of a pair its receiver does not
        // track: cleared here, so each round's (A) bits start from zeros
        if (!kind && !h.keep_ctl)
            for (int64_t r = r0; r < r1; ++r)
                if (h.rev[r] == NO_PAIR && h.ctl[2 * (size_t)r + 1])
                    reinterpret_cast<ulonglong2*>(h.ctl)[r] = make_ulonglong2(0, 0);
    }
    flush_count(h.stats, HB_PX_PRUNES, lists);
    flush_count(h.stats, HB_PX_PEERS, listed);
    flush_count(h.stats, HB_PX_IGNORED, ignored);
    flush_count(h.stats, HB_PX_CONNECT, connect);
}

hipError_t launch_hb_answer(const DevState& s, const HbState& h, hipStream_t st) {
    if (h.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_answer, dim3(grid_cap(h.n_pairs, 256)), dim3(256), 0, st, s, h);
    return hipGetLastError();
}

hipError_t launch_hb_px(const DevState& s, const HbState& h, uint32_t kind, hipStream_t st) {
    if (h.n_nodes == 0 || !h.pxno) return hipSuccess;
    hipLaunchKernelGGL(k_hb_px, dim3(grid_cap(h.n_nodes, 64)), dim3(64), 0, st, s, h, kind);
    return hipGetLastError();
}

hipError_t launch_hb_px_count(const HbState& h, uint32_t kind, hipStream_t st) {
    if (h.n_pairs == 0 || !h.pxno) return hipSuccess;
    hipLaunchKernelGGL(k_hb_px_count, dim3(grid_cap(h.n_pairs, 256)), dim3(256), 0, st, h, kind);
    return hipGetLastError();
}

hipError_t launch_hb_px_recv(const DevState& s, const HbState& h, const uint32_t* entries, uint64_t n,
                             hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_px_recv, dim3(grid_cap(n, 256)), dim3(256), 0, st, s, h, entries, n);
    return hipGetLastError();
}

hipError_t launch_hb_pack(const uint32_t* send_pair, uint64_t n_send, uint32_t stride, const uint64_t* a, const uint64_t* b,
                          uint64_t* out, hipStream_t st) {
    if (n_send == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hb_pack, dim3(grid_cap(n_send, 256)), dim3(256), 0, st, send_pair, n_send, stride, a, b, out);
    return hipGetLastError();
}

}  // namespace gsx
