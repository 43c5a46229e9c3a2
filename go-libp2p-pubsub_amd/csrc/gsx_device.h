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

// Topic parameters travel in the kernel argument segment for up to
// KARG_TOPICS topics, so every read is a scalar (s_load) from the kernarg
// buffer; larger engines read them through a read-only global pointer.
constexpr int KARG_TOPICS = 8;
struct KernParams {
    DevPeerParams pp;
    DevTopicParams tp[KARG_TOPICS];
};

// ---- HBM layout of the per-record state ------------------------------------
// Records (one per observer, peer, topic: the reference's topicStats,
// score.go:37-62) are tiled by 64 pairs — one wavefront's lanes:
//   rec   [p/64][t][field][64]  8-byte fields, field = FMD, MMD, MFP, IMD, GRAFT
//   rflag [p/64][t][64]         u8: IN_MESH | ACTIVE | FRESH
// so the lanes of a wave read each field of a topic as one contiguous 512-B
// span and a wave's whole working set (T x 2.6 KB) is one contiguous block
// of HBM.  meshTime is not stored: for an in-mesh record it is
// FRESH ? 0 : (last refresh time - graftTime), which is exactly what
// refreshScores() would have written (score.go:544-546; Graft zeroes it,
// score.go:658).
constexpr int TILE = 64;
constexpr int NFIELD = 5;
enum Field { FMD = 0, MMD = 1, MFP = 2, IMD = 3, GRAFT = 4 };

__host__ __device__ __forceinline__ size_t rec_index(uint64_t p, uint32_t t, uint32_t n_topics, int field) {
    return (((p / TILE) * n_topics + t) * NFIELD + field) * TILE + (p % TILE);
}
__host__ __device__ __forceinline__ size_t flag_index(uint64_t p, uint32_t t, uint32_t n_topics) {
    return ((p / TILE) * n_topics + t) * TILE + (p % TILE);
}

struct DevState {
    double* rec;          // tiled records (GRAFT slot holds int64 bits)
    uint8_t* rflags;      // tiled record flags
    uint8_t* pflags;      // per pair: PRESENT | CONNECTED
    int64_t* expire;      // per pair: retention expiry
    double* bp;           // per pair: behaviourPenalty
    double* app;          // per pair: AppSpecificScore snapshot (GSX_EV_APP_SCORE updates one)
    const uint32_t* ipg;  // 2 per pair: (observer, ip) group id | WL bit, or NONE
    uint32_t* ipcount;    // per group: number of present pairs carrying it
    double* score;        // per pair: output
    const DevTopicParams* tp;  // all topics (used when n_topics > KARG_TOPICS)
    uint64_t n_pairs;
    uint32_t n_topics;
    int64_t last_refresh;  // time of the last refreshScores() (derives meshTime)
};

constexpr uint8_t REC_IN_MESH = 0x01;
constexpr uint8_t REC_ACTIVE = 0x02;
constexpr uint8_t REC_FRESH = 0x04;  // grafted since the last refresh that covered it: meshTime == 0
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

// ---- propagation (gsx_propagate.hip) -------------------------------------------
constexpr uint8_t EDGE_OUTBOUND = 0x01, EDGE_DIRECT = 0x02, EDGE_GOSSIPSUB = 0x04, EDGE_FLOODSUB = 0x08,
                  EDGE_NO_PX = 0x10;
constexpr uint32_t ROUTER_FLOODSUB = 0, ROUTER_GOSSIPSUB = 1, ROUTER_RANDOMSUB = 2;
constexpr uint32_t NO_PAIR = 0xFFFFFFFFu;
constexpr uint8_t FWD_FORWARD = 0x01;    // v sends messages it received to u
constexpr uint8_t FWD_PUBLISH = 0x02;    // v sends messages it published to u
constexpr uint8_t FWD_RSUB_CAND = 0x04;  // u is one of v's RandomSub peers (drawn per message)
constexpr uint8_t FWD_SEND = 0x07;       // any of the above: v sends something to u
// Not about sending: the pair's observer drops every RPC from the pair's
// neighbour (gossipsub AcceptFrom: score < GraylistThreshold and not a direct
// peer, gossipsub.go:583-594, pubsub.go:1014-1017), this call.
constexpr uint8_t FWD_GIN = 0x08;
constexpr int RANDOMSUB_D = 6;           // randomsub.go:16-18
constexpr int MAX_HOPS = 64;
// Propagation counters: duplicates, first receipts per hop, and the
// push-minimal traffic terms of SURVEY.md §8d (summed over hops and 64-message
// words): eligible (edge, word) sends and (vertex, word) pairs gaining bits.
// STAT_BACKSENDS: receipts counted as duplicates that the `from` exclusion removes.
enum {
    STAT_DUPS = 0,
    STAT_HOP0 = 1,
    STAT_EDGE_SENDS = STAT_HOP0 + MAX_HOPS + 1,
    STAT_NEW_WORDS,
    STAT_BACKSENDS,
    STAT_REJECTED,  // receipts of REJECT messages
    STAT_IGNORED,   // receipts of IGNORE / THROTTLE messages
    STAT_GRAY,      // copies the receiver's AcceptFrom dropped (graylisted sender), counted apart from STAT_DUPS
    // range shards, compacted exchange: [hop] entries scattered into the halo
    // for that hop (k_halo_scatter), so a hop with no local frontier and no
    // remote row returns at once
    STAT_HALO0,
    STAT_WORDS = STAT_HALO0 + MAX_HOPS + 1
};
// rev[q] of a pair whose neighbour lives on another shard: HALO | receive slot.
constexpr uint32_t HALO = 0x80000000u;
constexpr uint32_t HALO_GRAY = 0x40000000u;  // pin of a remote pair whose copies u's AcceptFrom drops
constexpr uint32_t HALO_SLOT = 0x3FFFFFFFu;  // receive slots < 2^30
constexpr int PIN_FWD_SHIFT = 29;
constexpr uint32_t MAX_RANKS = 64;  // ranks of a shard plan (one node: 8)
// pin of a local pair: bit 28 = v drops what u sends it (graylisted u), so the
// back-sends the `from` exclusion removes were never counted as duplicates
constexpr uint32_t PIN_RDROP = 1u << 28;
constexpr uint32_t PIN_NODE_MASK = PIN_RDROP - 1;  // nodes per shard < 2^28

struct DevMsg {
    uint32_t source;      // global node id
    uint32_t validation;  // GSX_VALIDATION_*
    uint64_t msg_id;
};

// Node-major bitsets: a node's (or pair's) n_words message words are
// contiguous, so one gather brings every word of a neighbour.
struct PropState {
    const int64_t* row_ptr;
    const int32_t* col;        // global node ids
    const uint32_t* rev;       // pair (u -> v) -> pair (v -> u); NO_PAIR; HALO | slot if v is remote
    const uint32_t* pair_obs;  // per pair: local observer index
    const uint8_t* eflags;
    uint8_t* fwd;              // per pair r = (v -> u), this call: FWD_* (v sends to u)
    uint32_t* pin;             // per pair q = (u -> v), this call: NO_PAIR | HALO[|HALO_GRAY]|slot | fwd<<29 [| RDROP] | v_local
    uint32_t* corr;            // per pair (u -> v), this call: in-window back-sends v will not make
    const DevMsg* msgs;
    uint64_t* seen;            // [node][word]
    uint64_t* origin;          // [node][word] messages the node published
    uint64_t* from_mask;       // [pair (u -> v)][word] messages u first received from v (null: not tracked)
    uint32_t* fcnt;            // per pair (u -> v), this call: first receipts from v
    uint64_t* flast;           // per pair: hop << 32 | first receipts of the last hop that had any
    uint64_t* hfrom;           // [pair q = (u -> v), v remote][word]: u's first receipts from v at its latest such hop
    // compacted exchange: halo rows are [slot][tag | W words], a row empty unless its tag
    // is halo_tag | hop (k_halo_scatter); 0: the dense exchange's untagged [slot][W] rows
    uint64_t halo_tag;
    const uint32_t* send_slot;  // per pair: its send slot (NO_PAIR: no remote receiver asked for it)
    // Range shards, replicated frontier (rep != 0; the lean calls: late duplicate
    // accounting, no RandomSub draws, no first-deliverer rows).  Every rank keeps
    // the frontier rows of ALL n_total nodes, two hops deep: front_g
    // [parity][n_total][W] and occ_g [parity][(n_total + 63) / 64 + 1] (a row is valid
    // only under its bit); pins hold global node ids, so the hop gathers a remote
    // sender's row exactly as a local one.  Per hop each rank contributes its
    // new frontier rows (k_rep_pack) and scatters the others' (k_rep_scatter).
    uint32_t mark_div;          // very sparse hops (k_prop_mark) below n / mark_div receipts (GSX_MARK_DIV: A/B)
    uint32_t occ_div;           // lean hops gather a sender's row after its occupancy bit below n / occ_div
                                // receipts last hop (GSX_OCC_DIV: A/B; dense hops gather beside it)
    // One-word lean calls on one engine: STAT_EDGE_SENDS is counted at the call's end
    // (k_prop_dups, from each sender's forwarding hops), so k_prop_hop_fast1 can skip a
    // receiver whose seen word holds every message of the call (full1)
    uint32_t edge_late;
    uint64_t full1;
    uint32_t rep, n_total;
    // rep_rows: the hop's rows move as every rank's dense slice of front_g (one
    // all-gather) and its occupancy bits as a summed row, chunks of hops with no
    // host read; no very sparse marking (remote rows would not mark)
    uint32_t rep_rows;
    uint64_t* front_g;
    uint64_t* occ_g;
    uint64_t rep_in;            // remote frontier rows scattered for this hop (host-known)
    const uint32_t* rmark_v;    // [n_recv] remote senders' global ids, ascending (their local receivers: rmark_u)
    const uint32_t* rmark_u;
    uint64_t n_rmark;
    const uint64_t* src_bits;   // [(n_total + 63) / 64 + 1] bit per global node: published in this call
    const uint32_t* src_ids;    // [n_src] the sources' global ids, ascending, and their
    const uint64_t* src_rows;   // [n_src][W] origin rows (every message each published)
    uint32_t n_src;
    uint64_t* touch;           // [2][node / 64] bit per node, buffer h & 1: some sender's row is non-empty (very sparse hops)
    const uint32_t* halo_node; // per receive slot: the local node whose pair it feeds
    uint64_t* sel;             // [pair][word] RandomSub draws (null for other routers)
    uint32_t* rcand;           // [pair] RandomSub candidate lists, each node's staged over its own pair range
    const uint64_t* hist;      // [hop][node][word]: messages first received at that hop (row 0: published)
    uint32_t n_rows;           // valid history rows (hops run + 1)
    uint32_t win_hops;         // P3 window in hops: floor(window / latency)
    uint32_t* dupcnt;          // per pair: duplicates inside the P3 window
    uint32_t* firstcnt;        // per pair: first receipts (deferred credits), or null
    unsigned long long* stats; // STAT_*
    const uint64_t* halo;      // [receive slot][word]: filtered sends of remote neighbours
    const uint32_t* send_pair; // per send slot: the local pair (v -> u) it carries, NO_PAIR = none
    const uint8_t* send_dest;  // per send slot: destination rank
    const uint64_t* send_base; // per rank: first send slot of its segment
    const uint64_t* dest_halo_base;  // per rank: the halo slot its segment starts at, on that rank
    uint64_t n_send;
    uint32_t n_ranks;
    uint64_t n_pairs;
    uint32_t n_nodes, n_words, n_msgs, node_lo;
    uint32_t router, topic, flood_publish, credit, all_dups_in_window, rsub_sqrt, sharded;
    uint32_t max_hops, back_in_window;  // back_in_window: 2 * latency <= P3 window
    uint32_t late;                      // duplicates of local pairs by k_prop_dups at the end of the call
    uint32_t pending;                   // the pending credit counts may be non-zero (else they are not read)
    const uint64_t* drop;               // [word]: messages not accepted (seen, not delivered, not forwarded); null: none
    const uint64_t* reject;             // [word]: REJECT messages (P4 to the sender)
    uint32_t* invcnt;                   // per pair: pending invalid deliveries (markInvalidMessageDelivery)
    uint64_t* dseen;                    // [node][word]: hop-1 receipts of dropped messages (after the call)
    uint64_t* occ;                      // [hop][node / 64] bit per node: frontier row non-empty
    double publish_threshold;
    double graylist_threshold;          // AcceptFrom's gate (gossipsub only: ps.gate)
    // topic membership (null: every node joined every topic, no fanout)
    const uint64_t* psub;               // [pair]: topics the peer has joined (gs.p.topics)
    const uint64_t* sub;                // [node]: topics the node has joined (gs.mesh)
    const uint64_t* fanout;             // [pair]: topics whose fanout holds the peer
    uint32_t gate;                      // gossipsub: receivers drop copies from graylisted senders (FWD_GIN)
    unsigned long long* gray_pairs;     // pairs with FWD_GIN (counted by k_prop_fwd, kept with fwd)
    int64_t hop_latency, window;
    uint64_t seed;
    uint32_t* hop_flag;  // host-mapped, [hop]: k_prop_mark(h) stores (hop_seq << 1) | (hop h-1 delivered); null: off
    uint32_t hop_seq;
    // Compacted senders for k_prop_hop_fast: node u's pairs whose pin is not
    // NO_PAIR, packed at the front of its own pair range (row_ptr[u] ..
    // cend[u]) as (pin, pair).  Kept current with pin: rebuilt for the nodes
    // whose pins a changed fwd byte touched (k_prop_fwd's change list).
    uint2* cent;
    uint32_t* cend;
    uint8_t* rfwd;       // [pair q]: fwd of the reverse pair (k_prop_pin), so k_prop_dups reads it coalesced
    uint32_t* chg;       // [chg_cap] pairs whose fwd byte changed this call (k_prop_fwd)
    uint32_t* nchg;      // their count (> chg_cap: rebuild every pin)
    uint64_t* ndirty;    // [node / 64] nodes whose compacted row must be rebuilt
    uint32_t chg_cap;
    uint32_t inc;        // fwd / pin / cent hold the previous call's values: update them incrementally
    uint32_t flast_every;  // k_prop_hop_fast keeps flast at every hop (stepped calls), else at max_hops only
    uint32_t flast_live;   // this call's hops wrote flast (else it is all zero: k_prop_dups skips its load)
    // Topic-term cache of the re-scoring fold (k_prop_count<true, true>):
    // tterm[q * n_topics + t] = topic_score() of record (q, t) (times its
    // weight), valid for pair q while tgen[q] == tepoch.  The host moves tepoch
    // whenever anything but this fold may have changed a record, so a fold
    // recomputes only its own topic's term and re-sums the cached ones in
    // ascending topic order (bit-identical to eval_pair).  null: off.
    double* tterm;
    uint32_t* tgen;
    uint32_t tepoch;
    // Lazy re-scoring of the fold (k_prop_count<true, true>; null: off).  The
    // credits of P2 / P3 only raise a score when every scored topic has
    // TopicWeight >= 0, FirstMessageDeliveriesWeight >= 0 and
    // MeshMessageDeliveriesWeight <= 0 (the signs score_params.go:207-260
    // validates), so a pair whose stored score is >= lazy_thr (the largest
    // threshold a fwd byte tests) keeps its fwd byte: its re-score is left to
    // the next score reader (the host settles stale[] pairs, gsx_engine.cpp
    // ensure_scores), and stale[q] = 1 marks it.  P4 credits lower a score:
    // such pairs are always re-scored.
    uint8_t* stale;
    double lazy_thr;
    // Deferred folds (gsx_engine.cpp prop_end / fold_deferred; null: off): the
    // credits of pairs that keep their stored score (>= lazy_thr, no P4 this
    // call) are not folded per call but summed over calls — acc_s[r] the
    // copies the sender pair r sent (k_prop_dups), acc_f[q] the first
    // receipts of the receiver pair q — and folded once, before anything
    // reads the records or scores: q's P2 / P3 steps are acc_f[q] first
    // receipts and acc_s[rev q] - acc_f[q] duplicates.  Every step is the same
    // capped +1 of an unchanged mesh flag, so the sums fold to the
    // one-call-at-a-time result.
    uint32_t* acc_s;
    uint32_t* acc_f;
};

// pins_only: the fwd bytes stand (a RESCORE count kept them), update the
// pins / compacted senders of the listed changes only
hipError_t launch_prop_fwd(const PropState& ps, const DevState& s, hipStream_t st, bool pins_only = false,
                           bool compact = true);
hipError_t launch_prop_compact(const PropState& ps, hipStream_t st);  // compacted senders from the pins
hipError_t launch_prop_init(const PropState& ps, uint64_t* front, hipStream_t st);
hipError_t launch_prop_clear(const PropState& ps, bool clear_flast, bool clear_corr, hipStream_t st);
hipError_t launch_rsub_select(const PropState& ps, const uint64_t* front, const uint64_t* front_occ, hipStream_t st);
hipError_t launch_prop_pack(const PropState& ps, const uint64_t* front, const uint64_t* front_occ, uint64_t* send,
                            hipStream_t st);
hipError_t launch_prop_pack_compact(const PropState& ps, const uint64_t* front, const uint64_t* front_occ,
                                    uint64_t* out, unsigned long long* dcount, uint32_t* tab, hipStream_t st);
uint32_t pack_table_words(uint32_t n_nodes, uint32_t n_ranks);  // u32 words of its per-(block, rank) table
hipError_t launch_pack_counts(const unsigned long long* dcount, const unsigned long long* hop_new, uint32_t world,
                              int64_t* out, hipStream_t st);
hipError_t launch_halo_scatter(const PropState& ps, uint64_t* halo, const uint64_t* ent, uint64_t n, uint32_t h,
                               hipStream_t st);
hipError_t launch_prop_mark(const PropState& ps, uint32_t h, const uint64_t* front_occ, hipStream_t st);
hipError_t launch_prop_hop(const PropState& ps, uint32_t h, const uint64_t* front, uint64_t* nxt, hipStream_t st);
bool hop_lean(const PropState& ps);  // the call's hops take k_prop_hop_fast[1] (no RandomSub, no from rows, late)
// range shards, replicated frontier (PropState::rep)
hipError_t launch_rep_init(const PropState& ps, hipStream_t st);
hipError_t launch_rep_pack(const PropState& ps, uint32_t h, uint64_t* out, unsigned long long* cnt, hipStream_t st);
struct RepParts {  // the other ranks' entries of a hop (k_rep_scatter: one launch for all of them)
    const uint64_t* p[MAX_RANKS];
    uint64_t off[MAX_RANKS + 1];  // entry offsets; off[n] = total
    uint32_t n;
};
hipError_t launch_rep_scatter(const PropState& ps, uint32_t h, const RepParts& parts, hipStream_t st);
hipError_t launch_rep_fwd_pack(const PropState& ps, uint8_t* out, hipStream_t st);
hipError_t launch_rep_fwd_recv(const PropState& ps, const uint8_t* in, hipStream_t st);
hipError_t launch_rep_sends(const PropState& ps, uint32_t h_run, uint64_t* vcnt, uint64_t* out, hipStream_t st);
hipError_t launch_rep_sends_recv(const PropState& ps, const uint64_t* in, hipStream_t st);
hipError_t launch_prop_count(const PropState& ps, const DevState& s, bool fold, bool rescore, const DevPeerParams& pp,
                             hipStream_t st);
// gray_only: count the sends on pairs whose receiver graylists the sender
// (STAT_GRAY) and nothing else (per-hop accounting); else the late accounting.
hipError_t launch_prop_dups(const PropState& ps, uint32_t h_run, uint64_t* vcnt, bool gray_only, hipStream_t st);
// The deferred-fold call's per-pair pass (instead of k_prop_count): the pairs
// that must fold now (score below lazy_thr, or a P4 credit) fold their sums
// and are re-scored with their fwd bytes; the rest keep accumulating.
hipError_t launch_prop_defer(const PropState& ps, const DevState& s, const DevPeerParams& pp, hipStream_t st);
// Folds every deferred sum (acc_s / acc_f of topic ps.topic) into the records
// and marks the folded pairs stale (re-scored by the caller); the sums are
// cleared by the caller.
hipError_t launch_prop_fold_acc(const PropState& ps, const DevState& s, hipStream_t st);
hipError_t launch_prop_fold(const PropState& ps, const DevState& s, uint32_t* first, uint32_t* dup,
                            hipStream_t st);
hipError_t launch_prop_from(const PropState& ps, int32_t* first_from, hipStream_t st);
hipError_t launch_prop_hops_export(const PropState& ps, uint8_t* hop_mn, hipStream_t st);
// The call's arrival hops as the validation-code planes of its message set
// (VcRef: [plane][node][word], n_planes <= 8; hist rows 1 .. n_rows - 1).
hipError_t launch_prop_vcodes(const PropState& ps, uint64_t* vc, uint32_t n_planes, hipStream_t st);
hipError_t launch_prop_dup_rows(const PropState& ps, uint64_t* out, hipStream_t st);
hipError_t launch_prop_uncache(const PropState& ps, bool mask_cache, hipStream_t st);

// ---- heartbeat (gsx_heartbeat.hip) -------------------------------------------
// A round whose (A) sent more control messages than pairs / 32 leaves the
// control words for one bulk clear at the next round's start: (B) does not
// clear them one by one (a scattered line write per message).
__host__ __device__ __forceinline__ bool hb_bulk_round(unsigned long long grafts, unsigned long long prunes,
                                                       uint64_t n_pairs) {
    return grafts + prunes > n_pairs / 32;
}
constexpr int HB_LANE_DEG = 64;     // units up to this degree: one lane each, row staged in LDS
constexpr int HB_HUB_MAX = 12000;   // hub rows (one wave each) live in dynamic LDS: 13 B per pair
constexpr int64_t HEARTBEAT_INTERVAL_NS = 1000000000LL;  // GossipSubHeartbeatInterval (clearBackoff slack)
constexpr uint8_t HB_GRAFT = 1, HB_PRUNE = 2;            // control bytes [topic][pair]
enum {
    HB_GRAFTS = 0,
    HB_PRUNES,
    HB_ACCEPTED,
    HB_REJECTED,
    HB_PRUNES_HANDLED,
    HB_PENALTIES,
    HB_BACKOFF_CLEARED,
    HB_MESH_LINKS,
    HB_IHAVE_MSGS,
    HB_IHAVE_IDS,
    HB_BROKEN_PROMISES,
    HB_IHAVE_IGNORED,
    HB_IWANT_MSGS,
    HB_IWANT_IDS,
    HB_IWANT_SERVED,
    HB_GOSSIP_DELIVERED,
    HB_GOSSIP_REJECTED,
    HB_GOSSIP_DUPLICATES,
    HB_PX_PRUNES,
    HB_PX_PEERS,
    HB_PX_IGNORED,
    HB_PX_CONNECT,
    HB_FWD_DELIVERED,
    HB_FWD_DUPLICATES,
    HB_FWD_GRAYLISTED,
    HB_STAT_WORDS
};  // the order of gsx_heartbeat_out

struct DevGossipParams {
    int32_t d, d_lo, d_hi, d_score, d_out, og_peers;
    uint64_t og_ticks;
    int64_t prune_backoff_ns, graft_flood_threshold_ns;
    int32_t d_lazy, max_ihave;
    double gossip_factor;
    int32_t max_ihave_msgs, retransmission;  // MaxIHaveMessages, GossipRetransmission
    int64_t followup_ns;                      // IWantFollowupTime
    int64_t fanout_ttl;                       // FanoutTTL
    int32_t do_px, prune_peers;               // WithPeerExchange, PrunePeers
};

// When each node's copy of a message set's messages finished validating
// (score.go:944-974 keeps drec.validated per (observer, message); gsx.h (D)):
// a code per (node, message) as bit planes [plane][node][word] (plane b holds
// bit b of the codes of the node's word), codes indexing the set's validation
// times on the host (the call's copies: code = arrival hop, validated at t0 +
// hop * (hop_latency + validation_delay); every exchange round that recovered
// copies of the set appends the code of its `now`).  `vin` bit c: a copy with
// code c is inside this round's P3 window.
constexpr uint32_t VC_MAX_PLANES = 16;
struct VcRef {
    const uint64_t* vc;   // null: every code 0
    const uint64_t* vin;  // [codes / 64] (mixed sets; else null)
    uint64_t plane;       // words per plane (nodes x n_words)
    uint32_t n_planes, pad;
};
// The bits of `bits` (old copies in word idx = node * n_words + w) whose code
// is inside.  Bit by bit with the plane words re-read (cached) rather than held:
// the mixed-window path is rare, and registers it held would count against
// every caller's occupancy (the forwarding pull's).
__device__ __forceinline__ uint64_t vc_inside(const VcRef& V, size_t idx, uint64_t bits) {
    uint64_t in = 0;
    for (uint64_t m = bits; m; m &= m - 1) {
        const uint32_t i = (uint32_t)__builtin_ctzll(m);
        uint32_t c = 0;
        for (uint32_t b = 0; b < V.n_planes; ++b) c |= (uint32_t)((V.vc[b * V.plane + idx] >> i) & 1) << b;
        if ((V.vin[c >> 6] >> (c & 63)) & 1) in |= 1ull << i;
    }
    return in;
}
// old_in: 0 no old copy of the set is inside the window, 1 every one, 2 by code (V)
__device__ __forceinline__ uint64_t old_inside(uint32_t old_in, const VcRef& V, size_t idx, uint64_t bits) {
    return old_in == 1 ? bits : old_in == 2 ? vc_inside(V, idx, bits) : 0ull;
}

// One advertised batch of the gossip exchange (heartbeat step (D)): the
// batch's cache rows, and its message set's seen rows (exchange start),
// receipts of this exchange, validation outcomes and serial (promise handles
// are serial << 32 | message index).
// One (topic, pair) IHAVE slot, written whole by one 16-B store (emitGossip's
// observable output: gsx_gossip_results): ids advertised, their multiset
// digest, the round that wrote it (an older tag reads as no IHAVE).
struct alignas(16) IhaveSlot {
    uint64_t hash;
    uint32_t len, tag;
};
constexpr uint8_t IHAVE_OWN = 0x80;     // ihave_tag: the pair's own slot holds the list
constexpr uint8_t IHAVE_FAN = 0x40;     // ihave_tag: sent by the fanout pass (its units' half of ihave_unit)
constexpr uint32_t IHAVE_TAG_MAX = 0x3F;  // byte tags cycle 1..63 (the array is cleared at the wrap)
struct GxBatch {
    const uint64_t* mem;  // [node][word]: in the node's cache
    const uint64_t* all;  // [node][word]: seen by the node
    uint64_t* x;          // [node][word]: received in this exchange
    const uint32_t* val;  // [message]: GSX_VALIDATION_*
    uint8_t* got;         // set to 1 when some node delivers a message of the set
    const uint8_t* full;  // [node]: the node has seen every message of the set (nothing to ask)
    uint32_t n_words, serial, topic, avail;  // avail: still cached after this heartbeat's Shift
    uint32_t row_off;     // word offset of the batch in its topic's gossip rows (GxSub)
    uint32_t woff;        // word offset of the batch in the flat word list of all advertised batches
    uint32_t n_msgs;      // messages of the set (bits of the last word past it are never set)
    const uint64_t* common;  // [n_words]: the set's messages every node had seen as the exchange began (k_gx_setprep)
    uint32_t nxt;         // the next advertised batch of the same set, cache order (GX_END: none)
    uint32_t dense;       // a first-hand batch (most rows hold uncommon messages): k_gx_rhm sets its bit unread
    const uint64_t* src;  // [n_msgs] the set's origins (node << 32 | index, ascending): the forwarding's back counts
    uint32_t old_in;      // a copy of the set's messages validated before this round is inside the P3 window (old_inside)
    uint32_t grp;         // the set's group: up to 64 sets of one topic (the forwarding's hop-1 back counts)
    VcRef vc;             // the set's validation codes (old_in 2)
    const uint32_t* cnt;  // [node]: messages the node holds in this batch (k_mc_summary / k_gx_merge_sets)
    uint32_t vin_off;     // (range shards, old_in 2) word offset of the inside rows in a gxs_rows entry: 1 + fw + woff
    // (one engine) [n_words]: the set's messages every node missing at most GX_POOR of them had seen
    // (k_gx_setprep, after `common`); null on range shards
    const uint64_t* common2;
};
// A node missing more than GX_POOR messages of a set is "poor" in it: the
// common2 words leave it out, and k_gx_ask walks its pairs' rows of that set
// unfiltered (every other node's missing messages lie outside common2).
constexpr uint32_t GX_POOR = 16;
// The truncated IHAVE lists of one topic this round (emitGossip, gsx.h): the
// list the sender of pair r sent is row idx[r] of `pool` (tw words; bit
// row_off * 64 + k = message k of the batch at row_off), valid where the
// receiver's ihave_tr bit of the topic is set; rows are handed out by an
// atomic counter below cap (a bound on the round's targets).
struct GxSub {
    uint64_t* pool;
    uint32_t* idx;  // [pair (sender's side)]
    uint32_t* cnt;  // rows handed out
    uint32_t tw, cap;
};
// gs.p.topics[t] holds the peer of pair r / node v has joined t (null: all)
__device__ __forceinline__ bool topic_peer(const uint64_t* psub, uint64_t r, uint32_t t) {
    return !psub || ((psub[r] >> t) & 1);
}
__device__ __forceinline__ bool joined_node(const uint64_t* sub, uint32_t v, uint32_t t) {
    return !sub || ((sub[v] >> t) & 1);
}
constexpr uint64_t TAG_HEARTBEAT = 8, TAG_FANOUT = 10, TAG_JOIN = 11, TAG_PX = 12;  // draw tags (gsx.h)
constexpr uint32_t GX_PROMISE_SLOTS0 = 4;  // initial promise slots per pair (gossip_tracer.go:24-27; grown on demand)
constexpr uint64_t TAG_IWANT = 9, TAG_IHAVE_SUB = 13;

// One cached gossipsub batch (a gsx_propagate call) of an mcache window:
// node v has message k iff bit k % 64 of seen[v * n_words + k / 64].
struct GossipBatch {
    const uint64_t* seen;
    const uint64_t* dig;  // [node]: multiset digest of the node's ids in this batch (k_mc_summary)
    const uint32_t* cnt;  // [node]: how many ids the node holds in this batch
    uint32_t n_words;
    uint32_t slot_base;  // slot of message 0 in HbState::mc_digest (64 x the batch's first word of all topics)
    uint32_t wdig_base;  // HbState::mc_digest[wdig_base + w]: digest sum of all of word w's messages
    uint32_t n_msgs;
    uint32_t row_off;    // word offset of the batch in its topic's gossip rows (slot_base / 64 - the topic's first)
};

struct HbState {
    const int64_t* row_ptr;
    const uint32_t* rev;
    const uint8_t* eflags;
    int64_t* backoff;     // [topic][pair] expiry, 0 = no entry
    uint8_t* bo8;         // [topic / 8][pair]: bit topic % 8, backoff entry present (kept with `backoff`; 4-B aligned)
    uint64_t* ctl;        // [pair][2] (v -> u): bit t of [0] = v sent GRAFT(t) this round, of [1] PRUNE(t)
                          // (one 16-B load per control message: (B) reads both)
    uint64_t* resp;       // per pair (u -> v): bit t = u answers v's GRAFT(t) with PRUNE
    const uint64_t* halo_ctl;   // [receive slot][2]: GRAFT / PRUNE bits of remote senders (shards)
    const uint64_t* halo_resp;  // [receive slot]: PRUNE answers of remote receivers (shards)
    uint8_t* dirty;       // per pair: grafted / pruned by its owner's maintenance this round
    uint8_t* inbox;       // per pair (u -> v): v sent GRAFT / PRUNE bits on (v -> u) this round (unsharded reads)
    uint8_t* answer;      // per pair (v -> u): u answered with PRUNE bits on (u -> v) this round
    unsigned long long* stats;
    uint32_t* rngk;        // [topic][node]: draw counter after the unit's maintenance (emitGossip continues it)
    uint16_t* mcount;      // [topic][node]: mesh size, as the scan found it / (A) left it / (B) keeps it
    uint64_t* tr_acc;      // [pair]: topics whose GRAFT the owner accepted (tracing; else null)
    uint64_t* tr_hp;       // [pair]: topics whose PRUNE the owner handled (tracing; else null)
    bool keep_ctl;         // (B) leaves the control words it reads (tracing: gsx_hb_trace_words)
    uint32_t* work;        // [topic][tile * 64 + i]: units the scan found acting, per 64-node tile
    uint8_t* tcnt;         // [topic][tile]: how many (lane-per-unit maintenance)
    uint64_t n_tiles64;    // 64 * tiles: the per-topic stride of `work`
    uint32_t* hub_work;    // [topic][node]: acting units of nodes with more than HB_LANE_DEG peers
    uint32_t* n_hub;       // [topic]
    const uint32_t* hubs;  // nodes with more than HB_LANE_DEG peers (k_hb_recv_hub)
    uint32_t n_hubs;
    // emitGossip's observable output (gsx_gossip_results), per (topic, pair): a
    // one-byte mark of this round's targets (ihave_tag: IHAVE_TAG(cur8) = the
    // sending unit's list, in ihave_unit [topic][node], written once per unit;
    // | IHAVE_OWN = a truncated list's subset, in the pair's own ihave_slot)
    IhaveSlot* ihave_slot;  // [topic][pair] a truncated list's subset (valid under tag == ihave_cur)
    IhaveSlot* ihave_unit;  // [pass][topic][node] the unit's whole list (hash, len) of this round (pass 1: fanout)
    uint8_t* ihave_tag;     // [topic][pair] cur8 (| IHAVE_OWN) on this round's targets
    uint32_t ihave_cur;    // this round's tag
    uint32_t ihave_cur8;   // this round's byte tag (1..IHAVE_TAG_MAX)
    uint8_t* gelig;        // [pair] GELIG_TARGET | GELIG_SCORE as the round started (k_hb_gelig)
    // the gossip exchange (step (D)); null when it is off
    uint64_t* ihave_bits;  // [pair (u -> v), the receiver's]: topics v sent u an IHAVE for this round
    uint64_t* ihave_tr;    // [pair (u -> v)]: topics whose IHAVE from v was truncated (a GxSub row)
    GxSub gsub;            // k_hb_gossip of one topic: its truncated-list rows (pool null: none kept)
    const GxSub* gsubs;    // [topic]: the exchange's view of every topic's rows
    uint32_t* gx_err;      // [8]: 0 = a GxSub bound broken (an internal error), 6 = nodes listed in gx_nodes
    uint32_t* gx_nodes;    // [node]: the nodes with an asked pair (k_gx_ask -> k_gx_receive)
    uint64_t* gx_touch;    // [node bit]: the nodes whose receipt rows this round may hold a bit (listed by
                           // k_gx_ask, or a forwarding receiver): k_gx_merge_sets reads only their rows
    uint8_t* gx_mark;      // [pair]: answered pairs (their records took the receipts' credits; re-scored after)
    const uint64_t* gx_rhm;  // [node]: bit g = its row of advertised batch g holds a not-everywhere message
                             // (one engine: outside the batch's common2 words, gx_poor)
    uint32_t gx_poor;        // gx_rhm is over common2: k_gx_ask adds the batches its node is poor in (GX_POOR)
    const int32_t* col;    // [pair]: the peer (local node id; global on a shard)
    const GxBatch* gx;     // advertised batches, per topic gx_off[t] .. gx_off[t + 1]
    const uint32_t* gx_off;
    // every set's words in canonical order (topic, the set by its first batch
    // in cache order, word): (first batch, word, topic, 0); gx_nsw of them
    const uint4* gx_sw;
    uint32_t gx_nsw;
    // the flat word list of the advertised batches (GxBatch::woff): gx_fw
    // words, gx_wb[f] the batch of word f
    uint32_t gx_fw;
    const uint32_t* gx_wb;
    // the exchange on a range shard (null unsharded): the IHAVEs this rank's
    // nodes sent over cross-shard pairs (sender side, [pair]: topic bits), and
    // per cross-shard pair (u -> v), receiver side: v answers u's IWANT
    // (v's score of u >= GossipThreshold), and the index of v's cache rows in
    // the rows v's rank sent (gxs_rows: entries of 1 + gxs_fw words, the flat
    // word list of the advertised batches; NO_PAIR: v holds only common messages)
    uint64_t* gxs_out;
    uint64_t* gxs_tro;  // [pair (sender side)]: topics whose IHAVE over the cross-shard pair was
                        // truncated (its subset is row gsub.idx[pair]; k_gxs_rows masks the rows with it)
    uint8_t* gxs_rans;
    uint32_t* gxs_hidx;
    const uint64_t* gxs_rows;
    uint32_t gxs_fw;
    uint32_t gx_mixed;  // some set of the round has old_in 2 (per-copy validation codes)
    uint32_t gxs_vin;   // entries carry, after the rows, the sender's inside rows of the mixed sets (old_in 2):
                        // the bits of its row whose copy at the sender is inside the P3 window (hop-1 back-sends)
    // the IWANT first receipts per (topic, pair) of this round (the forwarding's
    // hop-1 back-sends, GxFwd); null when nothing is forwarded
    uint32_t* gxb_st0;     // [pair] stamp: the pair's counts were written this round
    uint32_t* gxb_cnt0;    // [group][pair]: sets whose old copies are inside the P3 window | the others << 16
    uint32_t gxb_ngrp;     // set groups this round (GxBatch::grp)
    uint32_t gxb_stamp;
    uint32_t* gx_req;      // [pair]: ids asked in this exchange (0 = none), GX_REQ_ALL: every candidate
    uint64_t* prom_h;      // [pair][prom_slots]: promised message handle
    int64_t* prom_e;       // [pair][prom_slots]: its expiry (0 = free slot)
    uint32_t prom_slots;   // slots per pair (grown by the host while every pair keeps one free)
    uint8_t* prom_any;     // [pair]: some slot may be in use (set on every add, recomputed by k_gx_promises)
    uint32_t* prom_occ;    // max over pairs of the slots in use after the exchange
    // topic membership (null: every node joined every topic, no fanout)
    const uint64_t* psub;  // [pair]: topics the peer has joined (gs.p.topics)
    const uint64_t* sub;   // [node]: topics the node has joined (gs.mesh)
    uint64_t* fanout;      // [pair]: topics whose fanout holds the peer (gs.fanout)
    uint64_t* fan_has;     // [node]: topics with a fanout entry
    int64_t* lastpub;      // [node][topic] (gs.lastpub; 0 = none)
    uint32_t fan_mode;     // k_hb_gossip: 0 the joined units' mesh gossip, 1 the fanout units' (:1553)
    uint32_t* mscratch;    // [pair]: candidate lists of the membership kernels (each row one lane's)
    uint32_t* pxbase;      // [pair]: k_hb_px's per-topic candidate list over each pruning node's row
    const uint32_t* pair_obs;  // [pair]: its owner (local node; set with sub)
    // peer exchange on PRUNE (do_px; null otherwise)
    uint8_t* pxno;         // [pair]: bit 0 = (A) pruned it without PX, bit 1 = its (B) answers go without PX
    uint32_t* px_log;      // [px_cap][4]: connection candidates (receiver, candidate, pruner, topic | kind << 8)
    uint64_t px_cap;
    // peer exchange across range shards: a PRUNE of a cross-shard pair carries
    // its PX list to the receiver's rank as an entry (receive slot there,
    // topic | kind << 8, n, ids[PrunePeers]: pxs_w u32), grouped per destination
    const uint32_t* send_slot;        // [pair]: the pair's send slot (NO_PAIR: the peer does not track it)
    const uint8_t* send_dest;         // [send slot]: destination rank
    const uint64_t* send_base;        // [rank + 1]: first send slot of each destination
    const uint64_t* dest_halo_base;   // [rank]: the destination's receive slot of this rank's first
    uint32_t* pxs_out;                // entries (null: the count pass)
    const uint64_t* pxs_off;          // [rank]: first entry of each destination
    unsigned long long* pxs_cnt;      // [rank]: entries counted / written
    uint32_t pxs_w;
    const uint32_t* halo_pair;        // [receive slot]: the local pair (u -> v) whose peer v is remote
    double accept_px;      // AcceptPXThreshold
    double publish_threshold;
    const uint64_t* mc_digest;  // per cache slot: mix64(id + golden)
    uint32_t* long_nodes;  // nodes whose gossip list needs per-target truncation
    uint32_t* n_long;
    DevPeerParams pp;  // live scores of emitGossip
    double gossip_threshold;
    uint64_t n_pairs;
    uint32_t n_nodes;
    uint32_t node_lo;  // global id of local node 0 (range shards)
    uint64_t tick;
    int64_t now;
    uint64_t seed;
    double og_threshold, graylist;  // PeerScoreThresholds (score_params.go:12-32)
    DevGossipParams gp;
};

hipError_t launch_hb_clear_backoff(const HbState& h, uint32_t n_topics, hipStream_t st);
// Byte ranges cleared in one launch (a round's per-round clears: one dispatch
// instead of one fill each, every fill costing ~5 us of the stream however small).
constexpr uint32_t ZERO_SPANS = 12;
struct ZeroSpans {
    uint8_t* p[ZERO_SPANS];
    uint64_t n[ZERO_SPANS];
    uint32_t k;
};
hipError_t launch_zero_spans(const ZeroSpans& z, hipStream_t st);
// Rebuilds the backoff presence bits from the expiry array (gsx_import_backoff).
hipError_t launch_bo_rebuild(const int64_t* backoff, uint8_t* bo8, uint64_t n_pairs, uint32_t n_topics,
                             hipStream_t st);
hipError_t launch_hb_scan(const DevState& s, const HbState& h, hipStream_t st);
// The gossip exchange: broken promises at the heartbeat start (P7); step (D) below.
hipError_t launch_gx_promises(const DevState& s, const HbState& h, hipStream_t st);
// Topic membership (gossipsub.go:943-1083, 1517-1554): psub from sub; the
// fanout of unjoined publishers (one lane per source); the heartbeat's fanout
// expiry + maintenance of topic t; Join / Leave of (node, topic) entries.
hipError_t launch_psub(const int32_t* col, const uint64_t* sub, uint64_t* psub, uint64_t n_pairs, hipStream_t st);
hipError_t launch_fanout_pick(const DevState& s, const HbState& h, const uint32_t* sources, uint32_t n_src,
                              uint32_t topic, int64_t now, uint64_t seed, double publish_threshold, hipStream_t st);
hipError_t launch_hb_fanout(const DevState& s, const HbState& h, uint32_t t, hipStream_t st);
hipError_t launch_join(const DevState& s, const HbState& h, const uint32_t* nodes, const uint32_t* topics,
                       uint32_t n, uint32_t leave, hipStream_t st);
hipError_t launch_gx_exchange(const DevState& s, const HbState& h, hipStream_t st);
// Per node, the advertised batches whose cache row holds a message outside
// its set's common words (gx_rhm: only there can the node hold a message some
// receiver lacks).
hipError_t launch_gx_rhm(const GxBatch* gx, uint32_t n_gx, uint32_t n_nodes, uint64_t* rhm, hipStream_t st);
// One pass over the seen rows of the message sets of an exchange that need
// it (blockIdx.y = entry): the receipt rows zeroed (x non-null), `full`
// recomputed (non-null) and the common words ANDed (non-null; preset to ~0 by
// the caller); the seen rows are read only for the last two.
struct GxSetPrep {
    const uint64_t* all;
    uint64_t* x;
    uint8_t* full;
    uint64_t* common;
    uint32_t n_words, n_msgs;
    uint64_t* common2;  // (one engine) AND over the nodes missing at most GX_POOR messages (GxBatch::common2)
};
hipError_t launch_gx_setprep(const GxSetPrep* sets, uint32_t n_sets, uint32_t n_nodes, hipStream_t st);
// After the exchange, every set in one pass (blockIdx.y = set): seen |= the
// receipts, the receipt rows keep the accepted messages only (the recovered
// copies' cache rows) and their k_mc_summary (count, digest per node) is
// written beside them, so the copies are Put without another pass.
struct GxSetMerge {
    uint64_t* all;
    uint64_t* x;
    const uint64_t* acc;       // [W] accepted messages
    const uint64_t* msg_dig;   // [W * 64] id digests, then [W] word digests
    uint64_t* dig;             // [node] summary digest of the recovered rows
    uint32_t* cnt;             // [node] their message count
    uint32_t n_words, n_msgs;
    uint64_t* vc;              // the set's code planes: the recovered copies take `code` (null: none)
    uint64_t plane;
    uint32_t n_planes, code;
    uint8_t* chg;              // set to 1 when some receipt changes the set's seen rows
    const uint64_t* touch;     // [node bit]: nodes whose rows may hold a receipt (null: every node); the
                               // others' receipt rows, counts and digests are zero already (k_gx_setprep)
    uint8_t* full;             // the set's full bytes, kept exact at the touched nodes (null: recomputed later)
};
hipError_t launch_gx_merge_sets(const GxSetMerge* sets, uint32_t n_sets, uint32_t n_nodes, hipStream_t st);
// The forwarding of the recovered messages (gsx.h (D): a delivered message is
// published on at once, gossipsub.go:943-1013), in synchronous hops inside the
// round.  One run covers up to 64 message sets of up to GXF_SLOTS topics (the
// node-level frontier and receiver masks are one bit per set); runs are
// independent (their messages are disjoint).
constexpr uint32_t GXF_SLOTS = 8;
constexpr uint32_t GXF_MAX_HOPS = 4096;  // hops of one run (the count arrays)
struct GxFwdSet {
    const uint64_t* all;  // [node][W] seen as the exchange began
    uint64_t* x;          // [node][W] this round's receipts (the forwarded first receipts are added)
    const uint64_t* acc;  // [W] accepted messages
    const uint64_t* src;  // [n_msgs] origin node << 32 | message index, ascending
    uint64_t* fr[2];      // [node][W] frontier rows by hop parity (valid under the node's fmask bit)
    uint32_t n_words, n_msgs, topic, slot, serial;
    uint32_t woff;        // word offset of the set's rows in a cross-shard frontier entry (range shards)
    uint8_t* got;         // set to 1 when a node delivers a message of the set (its recovered batch is Put)
    uint32_t old_in;      // a copy of a message the receiver had before the round is inside the P3 window (old_inside)
    VcRef vc;             // the set's validation codes (old_in 2)
};
struct GxFwd {
    const GxFwdSet* sets;
    uint32_t n_sets, n_slots;
    uint32_t slot_topic[GXF_SLOTS];
    uint32_t slot_grp[GXF_SLOTS];  // the slot's set group (hop-1 back counts)
    uint64_t slot_sets[GXF_SLOTS];  // per topic slot: its sets
    uint64_t* fmask[2];  // [node] the sets of the node's frontier, by hop parity
    uint32_t* flist[2];  // frontier nodes, by hop parity
    uint32_t* fcnt;      // [hop] frontier sizes (hop 0: the recovering nodes)
    uint64_t* rmask;     // [node] this hop: the sets some frontier neighbour may send (cleared by the pull)
    uint32_t* rlist;     // this hop's receivers
    uint32_t* rcnt;      // [hop]
    uint64_t* srcm;      // [node] the sets holding a message the node published
    // back-sends (the `from` exclusion): first receipts of pair (x -> v) per topic,
    // hop 0 (the IWANT answers, [topic][pair] u16 under stamp0) and later hops
    // ([parity][pair][slot] u16 under stamps seq + hop)
    const uint32_t* bst0;
    const uint32_t* bcnt0;  // [topic][pair]: (sets with old_in) | (the others) << 16
    uint32_t stamp0;
    uint32_t* bst[2];
    uint16_t* bcnt[2];
    uint32_t seq;
    // per pair, this run: fout[r] = the slots whose topic the pair's owner
    // forwards over r (k_gxf_init); fin[q] = fout[rev q] | GXF_GRAY (the
    // receiver's AcceptFrom drops the peer of q), a pass of its own on range
    // shards only (remote senders' slots arrive there); null on one engine:
    // the pull gathers fout[rev q] for the senders in the frontier alone
    uint8_t* fout;
    uint16_t* fin;
    // per receiver x, this run: its pairs whose sender forwards a run topic to
    // it (fin & 0xFF), ascending, as (q, rev q, peer's local index, fin) at
    // fent[row_ptr[x] .. fend[x]) (k_gxf_compact, before hop 1): the pull walks
    // x's mesh senders instead of every pair of its row (null: every pair)
    uint4* fent;
    uint32_t* fend;
    uint64_t all_sets;
    uint64_t* fbit[2];  // [node / 64] bit per node: in the frontier (the pull's filter: L2-resident)
    // range shards: the frontier of remote senders, per hop, as entries of
    // GXF_HDR + rw words (receive slot, set mask, back-send counts per slot and
    // their in-window part as 8 x u16 each, then the rows of every run set at
    // its woff); per cross-shard pair (x -> v): the entry of v this hop
    // (hstamp == seq + hop) and its index
    uint32_t* hstamp;
    uint32_t* hidx;
    const uint64_t* hent;
    uint32_t rw;
    uint32_t dense_div;  // a hop is dense when its last frontier exceeds n_nodes / dense_div
    // one engine with the eligible-sender lists: fout is computed once a hop's
    // frontier holds more than fout_lazy nodes (k_gxf_fout_pre; before the
    // first dense hop's lists) and not at the run's start; a smaller
    // frontier's hop evaluates its senders' slots itself (0: fout computed at
    // the start)
    uint32_t fout_lazy;
    uint32_t mixed;      // some set's old copies are split by the P3 window (old_in 2)
};
constexpr uint32_t GXF_HDR = 6;
constexpr uint32_t GXF_DENSE = 16;
constexpr uint32_t GXF_FOUT_DIV = 64;     // GxFwd::fout_lazy = min(n / GXF_FOUT_DIV, GXF_FOUT_MAX)
constexpr uint32_t GXF_FOUT_MAX = 16384;  // (GSX_GXF_FOUT_DIV / GSX_GXF_FOUT_MAX: A/B)
constexpr uint16_t GXF_GRAY = 0x100;
hipError_t launch_gxf_init(const DevState& s, const HbState& h, const GxFwd& f, uint32_t n_src_total,
                           hipStream_t st);
hipError_t launch_gxf_hop(const DevState& s, const HbState& h, const GxFwd& f, uint32_t hop, hipStream_t st);
// The exchange across range shards (gsx.h, gsx_gx_*): per send slot, the
// IHAVE topic bits and the answer bit of its pair ([n_send][2]); their
// receipt per receive slot; the entries of the senders' cache rows (a count
// pass per destination with out null, then the pack into out at off[dest]);
// their receipt; the forwarding's per-pair topic slots (fout) per send slot
// and their receipt; a hop's frontier entries (count / pack) and their receipt.
struct GxsPlan {  // the shard plan's send side (gsx_shard_send_plan)
    const uint32_t* send_pair;       // [send slot]: the local pair (v -> u) it carries, NO_PAIR = none
    const uint8_t* send_dest;        // [send slot]: destination rank
    const uint64_t* send_base;       // [rank + 1]: first send slot of each destination
    const uint64_t* dest_halo_base;  // [rank]: the destination's receive slot of this rank's first
    const uint32_t* pair_obs;        // [pair]: its local owner
    uint64_t n_send;
};
hipError_t launch_gxs_pack_ihave(const DevState& s, const HbState& h, const GxsPlan& P, uint64_t* out, hipStream_t st);
hipError_t launch_gxs_recv_ihave(const HbState& h, const uint64_t* in, const uint32_t* halo_pair, uint64_t n_recv,
                                 hipStream_t st);
hipError_t launch_gxs_rows(const HbState& h, const GxsPlan& P, const GxBatch* gx, uint32_t n_gx,
                           unsigned long long* cnt, const uint64_t* off, uint64_t* out, hipStream_t st);
hipError_t launch_gxs_rows_recv(const HbState& h, const uint64_t* in, uint64_t n, const uint32_t* halo_pair,
                                hipStream_t st);
hipError_t launch_gxf_pack_fout(const GxFwd& f, const GxsPlan& P, uint64_t* out, hipStream_t st);
hipError_t launch_gxf_recv_fout(const GxFwd& f, const uint64_t* in, const uint32_t* halo_pair, uint64_t n_recv,
                                hipStream_t st);
hipError_t launch_gxf_halo(const HbState& h, const GxFwd& f, const GxsPlan& P, uint32_t hop, unsigned long long* cnt,
                           const uint64_t* off, uint64_t* out, hipStream_t st);
hipError_t launch_gxf_pack_counts(const unsigned long long* cnt, const uint32_t* front, uint32_t world, int64_t* out,
                                  hipStream_t st);
hipError_t launch_gxf_halo_recv(const HbState& h, const GxFwd& f, uint32_t hop, const uint64_t* in, uint64_t n,
                                const uint32_t* halo_pair, const uint32_t* halo_node, hipStream_t st);
// Promise slots [pair][from] -> [pair][to] (to > from; new slots free).
hipError_t launch_gx_prom_grow(const uint64_t* h_in, const int64_t* e_in, uint32_t from, uint64_t* h_out,
                               int64_t* e_out, uint32_t to, uint64_t n_pairs, hipStream_t st);
// GetBrokenPromises without the penalty (gsx_promise_broken): counts per pair, frees them.
hipError_t launch_gx_broken(const HbState& h, uint32_t* counts, hipStream_t st);
// The promises outstanding (gsx_promise_count): summed into *n (zeroed by the caller).
hipError_t launch_gx_count(const HbState& h, unsigned long long* n, hipStream_t st);
hipError_t launch_hb_maintain(const DevState& s, const HbState& h, uint32_t t_base, uint32_t n_t, int64_t max_deg,
                              hipStream_t st);  // topics t_base .. t_base + n_t - 1
// tw: the topic's gossip row words (sum of its batches' n_words)
constexpr uint8_t GELIG_TARGET = 1, GELIG_SCORE = 2;
hipError_t launch_hb_gelig(const DevState& s, const HbState& h, hipStream_t st);
hipError_t launch_hb_gossip(const DevState& s, const HbState& h, uint32_t t, const GossipBatch* gb, uint32_t n_gb,
                            uint32_t tw, int64_t max_deg, hipStream_t st);
constexpr uint32_t HB_GOSSIP_MAX_WORDS = 4096;  // a topic's gossip rows: 262,144 ids (the long path's LDS rows)
hipError_t launch_hb_recv(const DevState& s, const HbState& h, hipStream_t st);
// out[i] = a[i] && b[i] (the pairs a heartbeat step re-scores before the next reads them)
hipError_t launch_mask_and(const uint8_t* a, const uint8_t* b, uint8_t* out, uint64_t n, hipStream_t st);
// Per-node (count, digest) of a batch the message cache keeps (computed once
// when it is cached, read by every heartbeat's emitGossip while it is in the
// gossip window): msg_dig[k] = mix64(id_k + golden), word_dig[w] = the sum of
// word w's messages' digests.
hipError_t launch_mc_summary(const uint64_t* seen, uint32_t n_nodes, uint32_t n_words, uint32_t n_msgs,
                             const uint64_t* msg_dig, const uint64_t* word_dig, uint64_t* dig, uint32_t* cnt,
                             hipStream_t st);
// One message block of a batch (gsx_mcache_put): its rows [node][words], its
// messages are the batch's [off, off + n).
struct McPart {
    const uint64_t* rows;
    uint32_t off, n, words;
};
hipError_t launch_mc_merge(const McPart* parts, uint32_t n_parts, uint64_t* dst, uint32_t n_nodes, uint32_t n_words,
                           hipStream_t st);
// Peer exchange across range shards: the count pass of the cross-shard PX
// PRUNEs (per destination, into h.pxs_cnt) and the receivers' side of the
// entries other ranks sent.
hipError_t launch_hb_px_count(const HbState& h, uint32_t kind, hipStream_t st);
hipError_t launch_hb_px_recv(const DevState& s, const HbState& h, const uint32_t* entries, uint64_t n,
                             hipStream_t st);
hipError_t launch_hb_answer(const DevState& s, const HbState& h, hipStream_t st);
// Peer exchange of the round's PRUNEs (gsx.h): kind 0 = (A) PRUNEs, 1 = (B) answers.
hipError_t launch_hb_px(const DevState& s, const HbState& h, uint32_t kind, hipStream_t st);
hipError_t launch_hb_pack(const uint32_t* send_pair, uint64_t n_send, uint32_t stride, const uint64_t* a, const uint64_t* b,
                          uint64_t* out, hipStream_t st);

// ---- launchers (gsx_kernels.hip) ---------------------------------------------
hipError_t launch_purge(const DevState& s, int64_t now, hipStream_t st);
hipError_t launch_refresh_score(const DevState& s, const KernParams& kp, int64_t now, bool refresh, hipStream_t st);
struct DevIpMove {
    uint64_t pair;
    uint32_t g0, g1;  // the pair's new (observer, IP) groups, IPG_WL flagged, IPG_NONE for none
};
hipError_t launch_set_ips(const DevState& s, const DevIpMove* mv, const uint32_t* group_off, uint32_t n_groups,
                          hipStream_t st);
hipError_t launch_ip_colocation_export(const DevState& s, const DevPeerParams& pp, double* out, hipStream_t st);
hipError_t launch_mark_rows(const int64_t* row_ptr, const uint32_t* obs, uint32_t n, uint8_t* mask, uint8_t val,
                            hipStream_t st);
// only2: re-score the pairs marked in both masks (null: in `only`)
// gate (optional): two event counters whose marks fill only2; a zero sum skips the pass
hipError_t launch_score_subset(const DevState& s, const KernParams& kp, const uint8_t* only, hipStream_t st,
                               const uint8_t* only2 = nullptr, const unsigned long long* gate = nullptr);
hipError_t launch_apply_events(const DevState& s, const DevPeerParams& pp, const DevEvent* ev,
                               const uint32_t* group_off, uint32_t n_groups, hipStream_t st);
hipError_t launch_recap(const DevState& s, uint32_t topic, double cap2, double cap3, hipStream_t st);
// The drop-in round trip (k_dropin): events + score() of the pairs they change
// (prs; the whole row of the observers in obs: AddPeer / RemovePeer move their
// IP colocation counts) into the device vector and the host-mapped copy, then
// `tag` into the host-mapped flag (system scope).  One workgroup.
hipError_t launch_dropin(const DevState& s, const DevPeerParams& pp, const DevEvent* ev, const uint32_t* goff,
                         uint32_t n_groups, const uint32_t* obs, uint32_t n_obs, const uint64_t* prs, uint32_t n_prs,
                         const int64_t* row_ptr, double* hscore, uint32_t* flag, uint32_t tag, hipStream_t st);
hipError_t launch_gather_scores(const double* score, const uint64_t* pairs, uint64_t n, double* out, hipStream_t st);
hipError_t launch_rebuild_ipcount(const DevState& s, uint32_t n_groups_ip, hipStream_t st);
hipError_t launch_synthesize(const DevState& s, const int32_t* col, const DevSynthSpec& spec, hipStream_t st);
// Topic-major <-> tiled permutation of one record field (import / export).
// field < NFIELD: 8-byte field; field == NFIELD: the u8 flags (FRESH dropped
// on export, recomputed on import from mesh_time == 0); mesh_time is handled
// by launch_mesh_time_{export,import}.
hipError_t launch_tile_field(const DevState& s, int field, const void* topic_major, hipStream_t st);
hipError_t launch_untile_field(const DevState& s, int field, void* topic_major, hipStream_t st);
hipError_t launch_mesh_time_export(const DevState& s, int64_t* topic_major, hipStream_t st);
// Sets FRESH on in-mesh records whose imported meshTime is 0; counts records
// whose meshTime is neither 0 nor last_refresh - graftTime into *n_bad.
hipError_t launch_mesh_time_import(const DevState& s, const int64_t* topic_major, uint32_t* n_bad, hipStream_t st);
}  // namespace gsx
