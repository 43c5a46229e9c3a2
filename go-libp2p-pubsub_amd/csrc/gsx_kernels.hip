// gsx_kernels.hip — CDNA4 (gfx950) kernels of the GossipSub scoring engine.
//
// Hot path: k_refresh_score, one streaming pass that fuses refreshScores()
// (score.go:497-558) with score() (score.go:258-335) for every
// (observer, peer) pair.  HBM-bound FP64/integer byte work: no MFMA, no LDS.
// Lane l of a wave owns pair 64*w + l; the records of a wave's 64 pairs form
// one contiguous tile (gsx_device.h), so every load and store instruction moves
// one contiguous 512-B span and a wave streams a single HBM block.  Topic
// parameters are read from the kernel-argument segment (scalar loads).
//
// Build with -ffp-contract=off: each expression is evaluated with the
// reference's roundings (Go on amd64 does not fuse multiply-add), which is what
// makes the results bit-identical to the CPU oracle.
#include "gsx_ops.h"

namespace gsx {

// ---- hot path: fused refresh + score ---------------------------------------

template <int TT, bool REFRESH>
__global__ __launch_bounds__(256) void k_refresh_score(DevState s, KernParams kp, int64_t now,
                                                       const uint8_t* __restrict__ only,
                                                       const uint8_t* __restrict__ only2,
                                                       const unsigned long long* __restrict__ gate) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= s.n_pairs) return;
    // a masked pass whose marks all come from counted events (gate: their
    // counters) has nothing to re-score when they sum to zero
    if (!REFRESH && gate && gate[0] + gate[1] == 0) return;
    // score-only pass over a subset (the pairs a heartbeat step touched, and
    // with only2 also marked there): the others keep their cached score, a
    // wave without one returns at once
    if (!REFRESH && only && (!only[p] || (only2 && !only2[p]))) return;
    const uint8_t st = s.pflags[p];
    if (!(st & PAIR_PRESENT)) {  // no peerStats: Score() returns 0 (:259-262)
        s.score[p] = 0.0;
        return;
    }
    const DevPeerParams& pp = kp.pp;
    // Disconnected (retained) peers are not decayed (:503-516).
    const bool conn = REFRESH && (st & PAIR_CONNECTED);
    const int T = TT > 0 ? TT : (int)s.n_topics;
    const uint64_t lane = p % TILE;
    double* const tile = s.rec + (p / TILE) * (uint64_t)T * (NFIELD * TILE) + lane;
    uint8_t* const ftile = s.rflags + (p / TILE) * (uint64_t)T * TILE + lane;
    double score = 0.0;
    // One topic's refresh (decay, write-back of changed counters, meshTime /
    // activation) and score term, from its already-loaded record.
    auto topic_step = [&](int t, const DevTopicParams& tp, double fmd, double mmd, double mfp, double imd,
                          int64_t graft, uint8_t fl) {
        double* const r = tile + (uint64_t)t * (NFIELD * TILE);
        int64_t mt = 0;
        if (conn) {
            // a counter that decays stays written back only if it changed: a
            // zero counter (most peers never send an invalid message, most
            // meshes never fail) decays to itself, and a wave whose 64 lanes
            // all hold zero skips the 512-B store entirely
            const double fmd0 = fmd, mmd0 = mmd, mfp0 = mfp, imd0 = imd;
            fmd = decay(fmd, tp.d2, pp.decay_to_zero);
            mmd = decay(mmd, tp.d3, pp.decay_to_zero);
            mfp = decay(mfp, tp.d3b, pp.decay_to_zero);
            imd = decay(imd, tp.d4, pp.decay_to_zero);
            if (__double_as_longlong(fmd) != __double_as_longlong(fmd0)) __builtin_nontemporal_store(fmd, r + FMD * TILE);
            if (__double_as_longlong(mmd) != __double_as_longlong(mmd0)) __builtin_nontemporal_store(mmd, r + MMD * TILE);
            if (__double_as_longlong(mfp) != __double_as_longlong(mfp0)) __builtin_nontemporal_store(mfp, r + MFP * TILE);
            if (__double_as_longlong(imd) != __double_as_longlong(imd0)) __builtin_nontemporal_store(imd, r + IMD * TILE);
            uint8_t nf = fl & ~REC_FRESH;
            if (fl & REC_IN_MESH) {  // :544-549
                mt = now - graft;
                if (mt > tp.act3) nf |= REC_ACTIVE;
            }
            if (nf != fl) ftile[t * TILE] = nf;  // rare once the mesh is steady
            fl = nf;
        } else if ((fl & REC_IN_MESH) && !(fl & REC_FRESH)) {
            mt = s.last_refresh - graft;
        }
        score += topic_score(tp, fl, mt, fmd, mmd, mfp, imd);
    };
    // streamed once per pass: non-temporal loads/stores (measured +4 %, tools/microbench)
    if constexpr (TT > 0) {
        // Every scored topic's record is loaded before any is used, so a wave
        // has all T x 5 loads (T x 2.5 KB) in flight at once instead of one
        // topic's at a time.  graftTime is loaded whether or not the record
        // is in the mesh (T > 1): some lane of the wave nearly always is, so
        // its line is fetched anyway, and the load no longer waits on the flag.
        double fmd[TT], mmd[TT], mfp[TT], imd[TT];
        int64_t gr[TT];
        uint8_t fl[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            if (!kp.tp[t].scored) continue;
            const double* const r = tile + (uint64_t)t * (NFIELD * TILE);
            fmd[t] = __builtin_nontemporal_load(r + FMD * TILE);
            mmd[t] = __builtin_nontemporal_load(r + MMD * TILE);
            mfp[t] = __builtin_nontemporal_load(r + MFP * TILE);
            imd[t] = __builtin_nontemporal_load(r + IMD * TILE);
            fl[t] = ftile[t * TILE];
            // with one topic there is nothing to overlap the flag load with,
            // and skipping graftTime outside the mesh saves its line (cfg5)
            gr[t] = (TT > 1 || (fl[t] & REC_IN_MESH))
                        ? __builtin_nontemporal_load(reinterpret_cast<const int64_t*>(r) + GRAFT * TILE)
                        : 0;
        }
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            if (!kp.tp[t].scored) continue;
            topic_step(t, kp.tp[t], fmd[t], mmd[t], mfp[t], imd[t], gr[t], fl[t]);
        }
    } else {
        for (int t = 0; t < T; ++t) {
            const DevTopicParams& tp = s.tp[t];
            if (!tp.scored) continue;
            const double* const r = tile + (uint64_t)t * (NFIELD * TILE);
            const uint8_t fl = ftile[t * TILE];
            const int64_t graft = (fl & REC_IN_MESH) ? reinterpret_cast<const int64_t*>(r)[GRAFT * TILE] : 0;
            topic_step(t, tp, __builtin_nontemporal_load(r + FMD * TILE), __builtin_nontemporal_load(r + MMD * TILE),
                       __builtin_nontemporal_load(r + MFP * TILE), __builtin_nontemporal_load(r + IMD * TILE), graft, fl);
        }
    }
    double bp = s.bp[p];
    if (conn) {
        bp = decay(bp, pp.d7, pp.decay_to_zero);
        s.bp[p] = bp;
    }
    s.score[p] = score_tail(s, pp, p, score, bp);
}

// refreshScores' purge of expired retained peers (score.go:503-515).  Runs
// before k_refresh_score so that the P6 counts it reads are post-purge.
__global__ __launch_bounds__(256) void k_purge(DevState s, int64_t now) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= s.n_pairs) return;
    const uint8_t st = s.pflags[p];
    if ((st & (PAIR_PRESENT | PAIR_CONNECTED)) != PAIR_PRESENT) return;
    if (!(now > s.expire[p])) return;  // now.After(pstats.expire)
    s.pflags[p] = 0;                   // delete(ps.peerStats, p)
    const uint2 g = reinterpret_cast<const uint2*>(s.ipg)[p];
    if (g.x != IPG_NONE) atomicSub(&s.ipcount[g.x & ~IPG_WL], 1u);  // removeIPs
    if (g.y != IPG_NONE && g.y != g.x) atomicSub(&s.ipcount[g.y & ~IPG_WL], 1u);
}

// ---- tracer events (score.go:588-974), one thread per observer ------------

// Events are grouped by observer (all state an event touches belongs to its
// observer, so groups are independent); within a group they run in the order
// the caller issued them.
__device__ __forceinline__ void apply_event(const DevState& s, const DevPeerParams& pp, const DevEvent& e) {
    switch (e.kind) {
    case 1: ev_add_peer(s, e.pair); break;
    case 2: ev_remove_peer(s, pp, e.pair, e.now_ns); break;
    case 3: ev_graft(s, e.pair, e.topic, e.now_ns); break;
    case 4: ev_prune(s, e.pair, e.topic); break;
    case 5: ev_first(s, e.pair, e.topic); break;
    case 6: ev_mesh(s, e.pair, e.topic); break;
    case 7: ev_invalid(s, e.pair, e.topic); break;
    case 8: ev_penalty(s, e.pair, e.arg); break;
    case 9: s.app[e.pair] = __longlong_as_double((long long)e.arg); break;  // AppSpecificScore(p), :320
    default: break;
    }
}

__global__ __launch_bounds__(64) void k_apply_events(DevState s, DevPeerParams pp, const DevEvent* __restrict__ ev,
                                                     const uint32_t* __restrict__ group_off, uint32_t n_groups) {
    const uint32_t g = blockIdx.x * 64u + threadIdx.x;
    if (g >= n_groups) return;
    for (uint32_t i = group_off[g]; i < group_off[g + 1]; ++i) apply_event(s, pp, ev[i]);
}

// The drop-in scorer's round trip in one launch (gsx_score / gsx_score_many
// on an engine small enough to keep a host copy of its scores, when that copy
// was current before the queued tracer events): one workgroup applies the
// events (read from host-mapped memory, grouped by observer), then score()s
// what they changed (eval_pair: the same operations as the score pass) into
// the device vector and the host copy (host-mapped): the event pairs
// themselves (a delivery, Graft / Prune, penalty or application score changes
// only its own pair's score), and the whole row of an observer with an
// AddPeer / RemovePeer (the IP colocation counts every pair of its IP groups
// reads); then stores `tag` to a host-mapped flag at system scope, which the
// host polls instead of synchronising the stream.  The work is the events',
// not the router's peer count.
__global__ __launch_bounds__(1024) void k_dropin(DevState s, DevPeerParams pp, const DevEvent* ev,
                                                 const uint32_t* goff, uint32_t n_groups, const uint32_t* obs,
                                                 uint32_t n_obs, const uint64_t* prs, uint32_t n_prs,
                                                 const int64_t* __restrict__ row_ptr, double* hscore, uint32_t* flag,
                                                 uint32_t tag) {
    for (uint32_t g = threadIdx.x; g < n_groups; g += blockDim.x)
        for (uint32_t i = goff[g]; i < goff[g + 1]; ++i) apply_event(s, pp, ev[i]);
    __threadfence();
    __syncthreads();
    for (uint32_t k = 0; k < n_obs; ++k) {
        const int64_t a = row_ptr[obs[k]], b = row_ptr[obs[k] + 1];
        for (int64_t p = a + threadIdx.x; p < b; p += blockDim.x) {
            const double v = eval_pair(s, pp, (uint64_t)p);
            s.score[p] = v;
            hscore[p] = v;
        }
    }
    for (uint32_t i = threadIdx.x; i < n_prs; i += blockDim.x) {
        const uint64_t p = prs[i];
        const double v = eval_pair(s, pp, p);
        s.score[p] = v;
        hscore[p] = v;
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// out[i] = score[pairs[i]] (gsx_score_many on a large engine)
__global__ __launch_bounds__(256) void k_gather_scores(const double* __restrict__ score, const uint64_t* __restrict__ pairs,
                                                       uint64_t n, double* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
        out[i] = score[pairs[i]];
}

// SetTopicScoreParams recap (score.go:217-231)
__global__ __launch_bounds__(256) void k_recap(DevState s, uint32_t topic, double cap2, double cap3) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= s.n_pairs || !(s.pflags[p] & PAIR_PRESENT)) return;
    const size_t b = rec_index(p, topic, s.n_topics, FMD);
    if (s.rec[b + FMD * TILE] > cap2) s.rec[b + FMD * TILE] = cap2;
    if (s.rec[b + MMD * TILE] > cap3) s.rec[b + MMD * TILE] = cap3;
}

__global__ __launch_bounds__(256) void k_rebuild_ipcount(DevState s) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= s.n_pairs || !(s.pflags[p] & PAIR_PRESENT)) return;
    const uint2 g = reinterpret_cast<const uint2*>(s.ipg)[p];
    if (g.x != IPG_NONE) atomicAdd(&s.ipcount[g.x & ~IPG_WL], 1u);
    if (g.y != IPG_NONE && g.y != g.x) atomicAdd(&s.ipcount[g.y & ~IPG_WL], 1u);
}

// ---- import / export permutations ------------------------------------------

__global__ __launch_bounds__(256) void k_tile_field(DevState s, int field, const void* __restrict__ src) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint32_t t = blockIdx.y;
    if (p >= s.n_pairs) return;
    const size_t i = (size_t)t * s.n_pairs + p;
    if (field < NFIELD)
        s.rec[rec_index(p, t, s.n_topics, field)] = static_cast<const double*>(src)[i];
    else
        s.rflags[flag_index(p, t, s.n_topics)] = static_cast<const uint8_t*>(src)[i] & (REC_IN_MESH | REC_ACTIVE);
}

__global__ __launch_bounds__(256) void k_untile_field(DevState s, int field, void* __restrict__ dst) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint32_t t = blockIdx.y;
    if (p >= s.n_pairs) return;
    const size_t i = (size_t)t * s.n_pairs + p;
    const bool present = s.pflags[p] & PAIR_PRESENT;  // no peerStats: no topicStats either (export zeros)
    if (field < NFIELD)
        static_cast<double*>(dst)[i] = present ? s.rec[rec_index(p, t, s.n_topics, field)] : 0.0;
    else
        static_cast<uint8_t*>(dst)[i] =
            present ? (s.rflags[flag_index(p, t, s.n_topics)] & (REC_IN_MESH | REC_ACTIVE)) : 0;
}

__global__ __launch_bounds__(256) void k_mesh_time_export(DevState s, int64_t* __restrict__ dst) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint32_t t = blockIdx.y;
    if (p >= s.n_pairs) return;
    const uint8_t fl = s.rflags[flag_index(p, t, s.n_topics)];
    dst[(size_t)t * s.n_pairs + p] = (s.pflags[p] & PAIR_PRESENT) ? mesh_time_of(s, fl, p, t) : 0;
}

__global__ __launch_bounds__(256) void k_mesh_time_import(DevState s, const int64_t* __restrict__ src,
                                                          uint32_t* n_bad) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint32_t t = blockIdx.y;
    if (p >= s.n_pairs) return;
    const size_t fi = flag_index(p, t, s.n_topics);
    const uint8_t fl = s.rflags[fi];
    if (!(fl & REC_IN_MESH)) return;
    const int64_t mt = src[(size_t)t * s.n_pairs + p];
    const int64_t graft = reinterpret_cast<const int64_t*>(s.rec)[rec_index(p, t, s.n_topics, GRAFT)];
    if (mt == 0) s.rflags[fi] = fl | REC_FRESH;
    else if (mt != s.last_refresh - graft) atomicAdd(n_bad, 1u);
}

// ---- seeded synthetic state (gsx/synth.py restated on the device) ------------

__device__ __forceinline__ double unif(uint64_t seed, uint64_t tag, uint64_t a, uint64_t b) {
    return (double)(h4(seed, tag, a, b) >> 11) * (1.0 / 9007199254740992.0);
}

constexpr uint64_t TAG_STATE = 4;

__global__ __launch_bounds__(256) void k_synth_records(DevState s, const int32_t* __restrict__ col, DevSynthSpec sp) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint32_t t = blockIdx.y;
    if (p >= s.n_pairs) return;
    const uint64_t a = (uint64_t)t * s.n_pairs + p;
    const size_t b = rec_index(p, t, s.n_topics, FMD);
    s.rec[b + FMD * TILE] = unif(sp.seed, TAG_STATE, a, 1) * sp.fmd_max;
    s.rec[b + MMD * TILE] = unif(sp.seed, TAG_STATE, a, 2) * sp.mmd_max;
    s.rec[b + MFP * TILE] = unif(sp.seed, TAG_STATE, a, 3) * sp.mfp_max;
    const double u4 = unif(sp.seed, TAG_STATE, a, 4) * sp.imd_max;
    s.rec[b + IMD * TILE] = ((uint32_t)col[p] >= sp.sybil_first) ? u4 : 0.0;
    const bool in_mesh = unif(sp.seed, TAG_STATE, a, 5) < sp.p_in_mesh;
    const int64_t graft = sp.now - (int64_t)(unif(sp.seed, TAG_STATE, a, 6) * (double)sp.graft_window);
    reinterpret_cast<int64_t*>(s.rec)[b + GRAFT * TILE] = graft;
    s.rflags[flag_index(p, t, s.n_topics)] = in_mesh ? REC_IN_MESH : 0;  // meshTime = now - graft
}

__global__ __launch_bounds__(256) void k_synth_pairs(DevState s, DevSynthSpec sp) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= s.n_pairs) return;
    uint8_t pf = PAIR_PRESENT | PAIR_CONNECTED;
    if (sp.p_disc > 0 && unif(sp.seed, TAG_STATE, p, 7) < sp.p_disc) pf = PAIR_PRESENT;
    if (sp.p_abs > 0 && unif(sp.seed, TAG_STATE, p, 8) < sp.p_abs) pf = 0;
    s.pflags[p] = pf;
    s.expire[p] = sp.now + (int64_t)((unif(sp.seed, TAG_STATE, p, 9) - 0.5) * (double)sp.expire_jitter);
    s.bp[p] = unif(sp.seed, TAG_STATE, p, 10) * sp.bp_max;
}

// ---- launchers -------------------------------------------------------------

static inline unsigned blocks_for(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_purge(const DevState& s, int64_t now, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_purge, dim3(blocks_for(s.n_pairs, 256)), dim3(256), 0, st, s, now);
    return hipGetLastError();
}

template <bool R>
static hipError_t launch_rs(const DevState& s, const KernParams& kp, int64_t now, const uint8_t* only,
                            const uint8_t* only2, hipStream_t st, const unsigned long long* gate = nullptr) {
    const dim3 grid(blocks_for(s.n_pairs, 256)), block(256);
    switch (s.n_topics) {
    case 1: hipLaunchKernelGGL((k_refresh_score<1, R>), grid, block, 0, st, s, kp, now, only, only2, gate); break;
    case 2: hipLaunchKernelGGL((k_refresh_score<2, R>), grid, block, 0, st, s, kp, now, only, only2, gate); break;
    case 4: hipLaunchKernelGGL((k_refresh_score<4, R>), grid, block, 0, st, s, kp, now, only, only2, gate); break;
    case 8: hipLaunchKernelGGL((k_refresh_score<8, R>), grid, block, 0, st, s, kp, now, only, only2, gate); break;
    default: hipLaunchKernelGGL((k_refresh_score<0, R>), grid, block, 0, st, s, kp, now, only, only2, gate); break;
    }
    return hipGetLastError();
}

hipError_t launch_refresh_score(const DevState& s, const KernParams& kp, int64_t now, bool refresh, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    return refresh ? launch_rs<true>(s, kp, now, nullptr, nullptr, st) : launch_rs<false>(s, kp, now, nullptr, nullptr, st);
}

hipError_t launch_score_subset(const DevState& s, const KernParams& kp, const uint8_t* only, hipStream_t st,
                              const uint8_t* only2, const unsigned long long* gate) {
    if (s.n_pairs == 0) return hipSuccess;
    return launch_rs<false>(s, kp, 0, only, only2, st, gate);
}

// setIPs (score.go:1021-1059) for pairs whose peer's IP list changed
// (refreshIPs, score.go:560-586; AddPeer of a peer seen on new addresses):
// a present peer leaves the sets of its old IPs and joins those of its new
// ones; an absent one only records the list (AddPeer counts it).  One thread
// per observer, its moves in the order given (the counts are the observer's).
__global__ __launch_bounds__(64) void k_set_ips(DevState s, const DevIpMove* __restrict__ mv,
                                                const uint32_t* __restrict__ group_off, uint32_t n_groups) {
    const uint32_t g = blockIdx.x * 64u + threadIdx.x;
    if (g >= n_groups) return;
    for (uint32_t i = group_off[g]; i < group_off[g + 1]; ++i) {
        const uint64_t p = mv[i].pair;
        const bool present = s.pflags[p] & PAIR_PRESENT;
        if (present) ipcount_add(s, p, -1);
        reinterpret_cast<uint2*>(const_cast<uint32_t*>(s.ipg))[p] = make_uint2(mv[i].g0, mv[i].g1);
        if (present) ipcount_add(s, p, +1);
    }
}
hipError_t launch_set_ips(const DevState& s, const DevIpMove* mv, const uint32_t* group_off, uint32_t n_groups,
                          hipStream_t st) {
    if (n_groups == 0) return hipSuccess;
    hipLaunchKernelGGL(k_set_ips, dim3(blocks_for(n_groups, 64)), dim3(64), 0, st, s, mv, group_off, n_groups);
    return hipGetLastError();
}

// ipColocationFactor (score.go:337-381) of every pair, unweighted: the
// PeerScoreSnapshot's IPColocationFactor (score.go:487); 0 without peerStats.
__global__ __launch_bounds__(256) void k_ip_colocation_export(DevState s, DevPeerParams pp, double* __restrict__ out) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= s.n_pairs) return;
    out[p] = (s.pflags[p] & PAIR_PRESENT) ? ip_colocation(s, pp, p) : 0.0;
}
hipError_t launch_ip_colocation_export(const DevState& s, const DevPeerParams& pp, double* out, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ip_colocation_export, dim3(blocks_for(s.n_pairs, 256)), dim3(256), 0, st, s, pp, out);
    return hipGetLastError();
}

// Sets mask[p] = val for every pair of the listed observers (incremental
// re-scoring after events, gsx_score).
__global__ __launch_bounds__(256) void k_mark_rows(const int64_t* __restrict__ row_ptr, const uint32_t* __restrict__ obs,
                                                   uint32_t n, uint8_t* __restrict__ mask, uint8_t val) {
    // one wave per observer, its lanes over the row
    const uint32_t lane = threadIdx.x % 64;
    for (uint32_t i = blockIdx.x * 4u + threadIdx.x / 64; i < n; i += gridDim.x * 4u) {
        const uint32_t o = obs[i];
        for (int64_t p = row_ptr[o] + lane; p < row_ptr[o + 1]; p += 64) mask[p] = val;
    }
}
hipError_t launch_mark_rows(const int64_t* row_ptr, const uint32_t* obs, uint32_t n, uint8_t* mask, uint8_t val,
                            hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mark_rows, dim3(std::min<uint32_t>((n + 3) / 4, 4096)), dim3(256), 0, st, row_ptr, obs, n, mask,
                       val);
    return hipGetLastError();
}

hipError_t launch_apply_events(const DevState& s, const DevPeerParams& pp, const DevEvent* ev,
                               const uint32_t* group_off, uint32_t n_groups, hipStream_t st) {
    if (n_groups == 0) return hipSuccess;
    hipLaunchKernelGGL(k_apply_events, dim3(blocks_for(n_groups, 64)), dim3(64), 0, st, s, pp, ev, group_off,
                       n_groups);
    return hipGetLastError();
}

hipError_t launch_dropin(const DevState& s, const DevPeerParams& pp, const DevEvent* ev, const uint32_t* goff,
                         uint32_t n_groups, const uint32_t* obs, uint32_t n_obs, const uint64_t* prs, uint32_t n_prs,
                         const int64_t* row_ptr, double* hscore, uint32_t* flag, uint32_t tag, hipStream_t st) {
    hipLaunchKernelGGL(k_dropin, dim3(1), dim3(n_obs ? 1024 : 256), 0, st, s, pp, ev, goff, n_groups, obs, n_obs, prs,
                       n_prs, row_ptr, hscore, flag, tag);
    return hipGetLastError();
}

hipError_t launch_gather_scores(const double* score, const uint64_t* pairs, uint64_t n, double* out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t b = (n + 255) / 256;
    hipLaunchKernelGGL(k_gather_scores, dim3((unsigned)(b < 4096 ? b : 4096)), dim3(256), 0, st, score, pairs, n, out);
    return hipGetLastError();
}

hipError_t launch_recap(const DevState& s, uint32_t topic, double cap2, double cap3, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_recap, dim3(blocks_for(s.n_pairs, 256)), dim3(256), 0, st, s, topic, cap2, cap3);
    return hipGetLastError();
}

hipError_t launch_rebuild_ipcount(const DevState& s, uint32_t n_groups_ip, hipStream_t st) {
    hipError_t e = hipMemsetAsync(s.ipcount, 0, sizeof(uint32_t) * (n_groups_ip ? n_groups_ip : 1), st);
    if (e != hipSuccess || s.n_pairs == 0) return e;
    hipLaunchKernelGGL(k_rebuild_ipcount, dim3(blocks_for(s.n_pairs, 256)), dim3(256), 0, st, s);
    return hipGetLastError();
}

hipError_t launch_synthesize(const DevState& s, const int32_t* col, const DevSynthSpec& spec, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    const unsigned nb = blocks_for(s.n_pairs, 256);
    hipLaunchKernelGGL(k_synth_records, dim3(nb, s.n_topics), dim3(256), 0, st, s, col, spec);
    hipLaunchKernelGGL(k_synth_pairs, dim3(nb), dim3(256), 0, st, s, spec);
    return hipGetLastError();
}

hipError_t launch_tile_field(const DevState& s, int field, const void* src, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_tile_field, dim3(blocks_for(s.n_pairs, 256), s.n_topics), dim3(256), 0, st, s, field, src);
    return hipGetLastError();
}

hipError_t launch_untile_field(const DevState& s, int field, void* dst, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_untile_field, dim3(blocks_for(s.n_pairs, 256), s.n_topics), dim3(256), 0, st, s, field, dst);
    return hipGetLastError();
}

hipError_t launch_mesh_time_export(const DevState& s, int64_t* dst, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mesh_time_export, dim3(blocks_for(s.n_pairs, 256), s.n_topics), dim3(256), 0, st, s, dst);
    return hipGetLastError();
}

hipError_t launch_mesh_time_import(const DevState& s, const int64_t* src, uint32_t* n_bad, hipStream_t st) {
    if (s.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mesh_time_import, dim3(blocks_for(s.n_pairs, 256), s.n_topics), dim3(256), 0, st, s, src,
                       n_bad);
    return hipGetLastError();
}

}  // namespace gsx
