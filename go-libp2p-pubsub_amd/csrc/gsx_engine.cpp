// gsx_engine.cpp — host side of the engine behind include/gsx.h.
//
// Owns the HBM state, orders all work on one HIP stream, keeps the
// reference's per-message delivery records (score.go:98-118, 686-870) on the
// host and turns tracer calls into counter events that the device applies.
// Every arithmetic update of scoring state happens in the HIP kernels of
// gsx_kernels.hip; this file only moves data and bookkeeps ids.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/gsx.h"
#include "gsx_device.h"

namespace {

constexpr int64_t kSecond = 1000000000LL;
constexpr int64_t kTimeCacheDuration = 120 * kSecond;  // pubsub.go:30
constexpr uint64_t kHostScoreMax = 1u << 16;  // engines up to this many pairs keep a host copy of the scores

bool invalid_number(double x) { return std::isnan(x) || std::isinf(x); }

enum { kDeliveryUnknown = 0, kDeliveryValid, kDeliveryInvalid, kDeliveryIgnored, kDeliveryThrottled };

struct RecKey {
    uint32_t obs;
    uint64_t msg;
    bool operator==(const RecKey& o) const { return obs == o.obs && msg == o.msg; }
};
struct RecKeyHash {
    size_t operator()(const RecKey& k) const {
        uint64_t x = k.msg ^ (uint64_t(k.obs) * 0x9E3779B97F4A7C15ULL);
        x ^= x >> 31;
        x *= 0xbf58476d1ce4e5b9ULL;
        x ^= x >> 29;
        return size_t(x);
    }
};
// deliveryRecord, score.go:98-103
struct DeliveryRecord {
    int status = kDeliveryUnknown;
    int64_t first_seen = 0;
    int64_t validated = 0;
    bool validated_set = false;  // !validated.IsZero()
    std::vector<uint64_t> peers;
    bool peers_nil = false;
};

}  // namespace

struct gsx_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr, ev_staged = nullptr;
    std::string err;

    uint32_t T = 0;
    gsx_peer_score_params pp{};
    bool pp_set = false;
    gsx_thresholds th{};
    gsx_topic_score_params tp[GSX_MAX_TOPICS]{};
    bool scored[GSX_MAX_TOPICS]{};
    gsx::DevTopicParams* d_tp = nullptr;

    // overlay
    bool loaded = false;
    uint32_t n_nodes = 0;
    uint64_t E = 0, rs = 0, n_tiles = 0;
    int64_t last_refresh = 0;  // now of the last refreshScores() pass
    std::vector<int64_t> row_ptr;
    std::vector<int32_t> col_host;
    std::vector<uint32_t> pair_obs;
    std::vector<uint32_t> ipg_host;  // 2 per pair, without WL bits
    std::vector<uint32_t> group_ip;  // IP id of each (observer, IP) group
    std::vector<uint8_t> ip_wl;      // per IP id: whitelisted
    uint32_t n_groups = 0;

    // device state
    double* d_rec = nullptr;      // tiled records, gsx_device.h
    uint8_t* d_rflags = nullptr;  // tiled record flags
    void* d_tmp = nullptr;        // import/export staging of one topic-major field
    uint32_t* d_nbad = nullptr;
    uint8_t *d_pflags = nullptr, *d_eflags = nullptr;
    int64_t* d_expire = nullptr;
    double *d_bp = nullptr, *d_app = nullptr, *d_score = nullptr;
    uint32_t *d_ipg = nullptr, *d_ipcount = nullptr;
    int32_t* d_col = nullptr;
    int64_t* d_row_ptr = nullptr;
    uint32_t* d_rev = nullptr;  // pair (u -> v) -> pair (v -> u)
    std::vector<uint8_t> eflags_host;
    bool floodsub_peers = true;  // some non-direct pair speaks no gossipsub (its publishes are score-gated)
    int64_t max_deg = 0;

    // heartbeat: router params, backoff [topic][pair], this round's control bytes
    gsx_gossipsub_params gp{};
    int64_t* d_backoff = nullptr;
    uint8_t* d_bo8 = nullptr;  // [topic / 8][pair] backoff presence bits
    uint64_t *d_ctl = nullptr, *d_resp = nullptr;  // d_ctl: [pair][2] GRAFT / PRUNE topic bits
    uint8_t* d_dirty = nullptr;
    uint32_t *d_long = nullptr, *d_nlong = nullptr;
    unsigned long long* d_hbstats = nullptr;
    uint32_t* d_rngk = nullptr;
    gsx::IhaveSlot* d_ihave_slot = nullptr;  // [topic][pair] (emitGossip's truncated-list IHAVE slots)
    gsx::IhaveSlot* d_ihave_unit = nullptr;  // [topic][node] (a unit's whole IHAVE list of the round)
    uint8_t* d_ihave_tag = nullptr;          // [topic][pair] this round's targets (HbState::ihave_tag)
    uint32_t *d_work = nullptr, *d_nwork = nullptr, *d_hubwork = nullptr, *d_hubs = nullptr;  // heartbeat worklists
    uint8_t* d_tcnt = nullptr;
    uint16_t* d_mcount = nullptr;
    std::vector<uint32_t> hubs_host;  // nodes with more than HB_LANE_DEG pairs
    std::vector<uint8_t> gossip_prev;  // per topic: IHAVE slots written last round
    // [topic][pair]: the heartbeat round that wrote the IHAVE slot (ihave_len /
    // ihave_hash hold a slot only under the current round's tag: no per-round clear)
    uint8_t* d_gelig = nullptr;  // [pair] HbState::gelig
    uint32_t ihave_round = 0;  // the IHAVE slots' tag of the last round (0: none yet)
    bool have_gossip = false;
    bool hb_clean = false;  // control words / answers / marks all zero (unsharded rounds clear what they read)
    bool hb_tracing = false;           // gsx_hb_set_tracing: keep the round's tracer Graft / Prune words
    uint64_t* d_tr_acc = nullptr;      // [pair] accepted GRAFT topics of the last round
    uint64_t* d_tr_hp = nullptr;       // [pair] handled PRUNE topics of the last round
    gsx::HbState hb{};  // the round in flight (gsx_hb_begin .. gsx_hb_end)
    bool hb_active = false;

    // The messages of one gossipsub propagate call (gossip exchange, gsx.h (D)):
    // who has seen each (first receipt or publish, and exchange receipts), the
    // validation outcomes, ids and digests; shared by the batch that cached
    // them and the batches of copies recovered later (reference counted).
    struct MsgSet {
        uint32_t serial = 0, n_msgs = 0, n_words = 0, topic = 0;
        uint64_t* d_all = nullptr;  // [node][word] (seen-row pool buffer)
        size_t all_words = 0;
        uint32_t* d_val = nullptr;  // [message] GSX_VALIDATION_*
        uint64_t* d_acc = nullptr;  // [word] accepted messages
        uint64_t* d_src = nullptr;  // [message] origin node << 32 | index, ascending (the forwarding's origin test)
        int64_t t0 = 0;             // now_ns of the call that made the set
        // per-node validation times of the copies (gsx::VcRef): code planes
        // [vc_p][node][word] (null: every code 0) and the time of each code
        uint64_t* d_vc = nullptr;
        size_t vc_words = 0;
        uint32_t vc_p = 0;
        std::vector<int64_t> vtime;
        // the arrival hops were kept (codes 0 .. n_hop - 1 = hops); a set cached
        // with the gossip exchange off keeps none: its copies' hop times may
        // only be read as one (gx_vcodes refuses a round whose window splits them)
        bool hops_kept = true;
        uint32_t n_hop = 1;
        uint64_t* d_dg = nullptr;   // [W * 64] id digests + [W] word digests (k_mc_summary)
        uint8_t* d_full = nullptr;  // [node]: every message seen (the exchange skips the set there)
        uint8_t* d_small = nullptr;  // the pooled block d_val / d_acc / d_dg live in
        size_t small_bytes = 0, full_bytes = 0;
        bool full_ok = false;       // d_full matches d_all
        // (one engine) the exchange's per-set prep kept across rounds while no
        // receipt changes d_all: the messages every node had (64 words), and a
        // receipt buffer a round left untouched (still zero)
        uint64_t* d_common = nullptr;
        size_t common_bytes = 0;
        bool common_ok = false;
        uint64_t* xs_spare = nullptr;
        std::vector<uint64_t> ids;
        int refs = 0;
    };
    uint32_t msg_serial = 0;
    // mcache (mcache.go): windows of cached gossipsub batches, front = history[0]
    struct McBatch {
        uint32_t topic = 0, n_msgs = 0, n_words = 0;
        uint64_t* d_seen = nullptr;  // [node][word]: the call's seen rows, handed over (no copy)
        size_t seen_words = 0;       // allocation size, for the buffer pool
        uint64_t* d_dig = nullptr;   // [node] summary of the batch (k_mc_summary), in the same allocation
        uint32_t* d_cnt = nullptr;
        std::vector<uint64_t> ids;
        MsgSet* set = nullptr;  // (unsharded engines)
        bool recovered = false;  // the receipt rows of an exchange (sparse: most nodes' rows empty)
    };
    std::deque<std::vector<McBatch>> mc;
    // gossip exchange state (allocated when first enabled)
    uint32_t *d_gxreq = nullptr, *d_gx_nodes = nullptr;
    uint32_t* d_gxflag = nullptr;  // [0] a GxSub bound broken, [1] a promise without a slot, [4] slots in use (max)
    uint64_t *d_prom_h = nullptr, *d_ihave_bits = nullptr;  // ihave_bits [2][E]: IHAVE topics, truncated ones (receiver's pair)
    bool ihave_tr_dirty = true;  // the truncated-list half of ihave_bits may hold bits (a round had a GxSub pool)
    int64_t* d_prom_e = nullptr;
    uint8_t* d_prom_any = nullptr;  // [pair] some promise slot may be in use (HbState::prom_any)
    unsigned long long* d_prom_cnt = nullptr;  // gsx_promise_count's device sum
    uint32_t prom_slots = 0;  // promise slots per pair (grown while every pair keeps one free before an exchange)
    // the truncated IHAVE lists of a round (GxSub per topic): rows for at most
    // tgt_bound targets of tw words each
    struct SubPool {
        uint64_t* pool = nullptr;
        uint32_t* idx = nullptr;
        size_t rows = 0, tw = 0;  // allocated
    };
    std::vector<SubPool> subp;
    uint32_t* d_sub_cnt = nullptr;  // [T]
    gsx::GxSub* d_gsubs = nullptr;  // [T]
    std::vector<gsx::GxSub> gsub_host;
    uint64_t tgt_bound = 0;  // sum over nodes of the most gossip targets it can pick (d_lazy, gossip_factor below)
    int32_t tgt_dlazy = -1;
    double tgt_gf = -1;
    // topic membership (A13), on once subscriptions / Join / Leave are used
    bool members_on = false;
    uint64_t mem_gen = 0;  // bumped whenever subscriptions or a fanout may have changed
    uint64_t *d_sub = nullptr, *d_psub = nullptr, *d_fanout = nullptr, *d_fan_has = nullptr;
    int64_t* d_lastpub = nullptr;
    uint32_t *d_mscratch = nullptr, *d_mlist = nullptr;
    uint8_t* d_mparts = nullptr;  // gsx_mcache_put's block descriptors
    size_t mparts_cap = 0;
    size_t mlist_cap = 0;
    // peer exchange on PRUNE (do_px): per-pair noPX bits, the candidate-list
    // scratch when membership is off, the connection-candidate log
    uint8_t* d_pxno = nullptr;
    uint32_t *d_pxscratch = nullptr, *d_pxlog = nullptr, *d_pxbase = nullptr;
    size_t px_cap = 0, pxlog_alloc = 0;
    uint64_t px_last = 0;  // the last round's connection candidates
    std::vector<uint64_t> h_sub;  // host copy of the joined topics per node
    // the exchange's round tables, one device arena (d_gxa) filled by one copy
    // from the pinned staging buffer: batches, offsets, word/set-word lists, prep + merge lists
    uint8_t* d_gxa = nullptr;
    size_t gxa_bytes = 0;
    gsx::GxBatch* d_gx = nullptr;     // (views into d_gxa)
    uint32_t* d_gx_off = nullptr;     // off[T + 1]: the batches of topic t
    uint32_t* d_gx_wb = nullptr;      // the flat word list's batch per word
    uint4* d_gx_sw = nullptr;         // every set's words (k_gx_node)
    gsx::GxSetPrep* d_gx_sp = nullptr;  // the exchange's sets (k_gx_setprep)
    gsx::GxSetMerge* d_gx_mg = nullptr;  // the same sets (k_gx_merge_sets)
    uint8_t* d_gx_got = nullptr;
    size_t gx_cap = 0;
    void* h_gxstage = nullptr;        // pinned staging of the exchange's batch list (hb_end)
    void* h_hbrb = nullptr;           // pinned: a round's counters, flags and per-set bytes (hb_finish)
    size_t h_hbrb_bytes = 0;
    size_t h_gxstage_bytes = 0;
    uint64_t* d_gx_rhm = nullptr;     // [node]: the advertised batches whose row holds an uncommon message
    uint8_t* d_gx_chg = nullptr;   // [set of the round]: a receipt changed its seen rows (k_gx_merge_sets; d_gx_got + gx_cap)
    uint64_t* d_gx_vin = nullptr;  // the round's inside-code bits of the mixed sets (GxRound::vin_host)
    size_t gx_vin_cap = 0;
    uint64_t* d_gx_common = nullptr;  // [set][64]: per message set of the exchange, the messages every node had
    size_t gx_common_cap = 0;         // (sets)
    // the forwarding of recovered messages (gsx.h (D); GxFwd), allocated with its first use
    uint64_t* d_gxf_mask = nullptr;   // fmask[2][N], rmask[N], srcm[N]
    uint32_t* d_gxf_list = nullptr;   // flist[2][N], rlist[N]
    uint32_t* d_gxf_cnt = nullptr;    // fcnt[GXF_MAX_HOPS + 1], rcnt[GXF_MAX_HOPS + 1]
    uint32_t* d_gxf_bst = nullptr;    // stamps: bst0[E], bst[2][E] (zeroed once; stamps only grow)
    uint32_t* d_gxf_b0 = nullptr;     // bcnt0[group][E]
    size_t gxf_b0_grps = 0;           // its groups
    uint16_t* d_gxf_b = nullptr;      // bcnt[2][E][GXF_SLOTS]
    uint16_t* d_gxf_fin = nullptr;    // [E] per run (GxFwd::fin)
    uint8_t* d_gxf_fout = nullptr;    // [E] per run (GxFwd::fout)
    uint4* d_gxf_fent = nullptr;      // [E] per run (GxFwd::fent; GSX_GXF_NO_COMPACT=1: null, the pull walks every pair)
    uint32_t* d_gxf_fend = nullptr;   // [N] per run (GxFwd::fend)
    gsx::GxFwdSet* d_gxf_sets = nullptr;  // [gxf_sets_cap] descriptors of the round's runs
    size_t gxf_sets_cap = 0;
    uint32_t* h_gxf_cnt = nullptr;    // pinned: the hop count of a run's last launched hop
    void* h_gxf_stage = nullptr;      // pinned: the runs' set descriptors
    hipEvent_t ev_gxf_stage = nullptr;  // recorded after the last copy out of h_gxf_stage
    bool gxf_stage_queued = false;
    size_t h_gxf_stage_bytes = 0;
    uint32_t gxf_stamp = 0;           // stamps of the IWANT back counts (one per round) and of the hops
    uint32_t* d_gxf_hst = nullptr;    // range shards: [2][E] GxFwd::hstamp, hidx
    uint64_t* d_gxs_out = nullptr;    // range shards: [2][E] HbState::gxs_out, gxs_tro
    uint8_t* d_gxs_rans = nullptr;    // range shards: [E] HbState::gxs_rans
    uint32_t* d_gxs_hidx = nullptr;   // range shards: [E] HbState::gxs_hidx
    unsigned long long* d_gxs_cnt = nullptr;  // range shards: [MAX_RANKS] entries per destination
    uint64_t* d_gxs_off = nullptr;            // range shards: [MAX_RANKS] their first entry
    uint64_t* d_gxs_send = nullptr;           // range shards: the entries this rank sends (grown)
    size_t gxs_send_cap = 0;
    std::vector<uint64_t> gxs_counts;         // the last count pass, per destination
    // The exchange (D) of the round in flight: hb_end prepares it; unsharded it
    // runs at once, on a range shard the gsx_gx_* / gsx_gxf_* steps run it and
    // gsx_gx_end finishes the round.
    struct GxfRun {
        std::vector<size_t> sets;   // indices into GxRound::sets
        std::vector<uint32_t> grps;  // its set groups (topic slots), GxRound::grp_*
    };
    struct GxRound {
        bool run = false, pending = false, exact = false, fwd_active = false;
        int stage = 0;  // range shards: 1 prepared, 2 common set, 3 IHAVEs in, 4 rows in, 5 exchanged
        gsx::HbState h{};
        std::vector<MsgSet*> sets;
        std::vector<uint32_t> set_grp;   // per set: its group (up to 64 sets / 65,535 messages of one topic)
        std::vector<uint32_t> grp_topic;  // per group
        std::vector<uint64_t*> xs;
        std::vector<std::pair<uint64_t*, size_t>> scratch;  // frontier rows, released after the round's sync
        uint32_t n_gx = 0, fw = 0;
        // per set: its old copies inside the P3 window (0 none, 1 all, 2 by
        // code: vc), the code this round's recovered copies take; the mixed
        // sets' inside-code bits (d_gx_vin)
        std::vector<uint32_t> old_in, vc_code;
        std::vector<gsx::VcRef> vc;
        std::vector<uint64_t> vin_host;
        std::vector<GxfRun> runs;
        gsx::GxFwd f{};
        uint32_t hops = 0;
    } gxr;
    std::vector<gsx::GossipBatch> gb_host;  // per heartbeat: batch descriptors of every topic
    std::vector<uint64_t> mc_digest_host;  // per cache slot: mix64(id + golden)
    std::vector<std::pair<size_t, uint64_t*>> seen_pool;  // (words, buffer) free seen-row buffers
    std::vector<std::pair<size_t, uint8_t*>> small_pool;  // message sets' small device arrays, recycled
    std::vector<void*> pool_slabs;  // the allocations both pools carve their buffers from (freed at teardown)
    std::unordered_map<const uint64_t*, size_t> seen_cap;  // each seen-row buffer's real capacity (words)
    gsx::GossipBatch* d_gb = nullptr;
    uint64_t* d_mc_digest = nullptr;
    size_t gb_cap = 0, ids_cap = 0;

    // propagation buffers (grown on demand) and the current / last call's shape
    struct {
        uint64_t *seen = nullptr, *hist = nullptr, *origin = nullptr, *from = nullptr, *sel = nullptr, *occ = nullptr;
        // the other frontier-history buffer: a gossipsub call's message set
        // builds its validation codes from its rows on vc_stream while the next
        // call writes these (allocated on the first such build)
        uint64_t *hist_alt = nullptr, *occ_alt = nullptr;
        uint32_t* corr = nullptr;
        uint8_t* fwd = nullptr;
        uint32_t* pin = nullptr;
        uint32_t *dup = nullptr, *first = nullptr;  // pending P2/P3 credit counts per pair
        uint32_t* inv = nullptr;    // pending invalid deliveries per pair (P4, REJECT messages)
        uint64_t* vmask = nullptr;  // [2][word]: messages validation drops / rejects, this call
        uint64_t* dseen = nullptr;  // [node][word]: hop-1 receipts of dropped messages (gsx_prop_results)
        size_t dseen_words = 0;
        bool has_drop = false;
        uint32_t* fcnt = nullptr;   // per pair, this call: first receipts
        uint64_t* flast = nullptr;  // per pair: hop << 32 | first receipts of its last such hop
        size_t from_words = 0;      // allocation of `from` (tracked first deliverers)
        gsx::DevMsg* msgs = nullptr;
        unsigned long long* stats = nullptr;
        unsigned long long* gray_pairs = nullptr;  // pairs with FWD_GIN of the current fwd (k_prop_fwd)
        uint2* cent = nullptr;                     // compacted senders (k_prop_compact)
        uint8_t* rfwd = nullptr;                   // fwd of each pair's reverse (k_prop_pin)
        uint32_t *cend = nullptr, *chg = nullptr, *nchg = nullptr;
        uint32_t* rcand = nullptr;  // [pair] RandomSub candidate lists (each node's over its own pair range)
        double* tterm = nullptr;    // [pair][topic] the re-scoring fold's topic-term cache (PropState::tterm)
        uint32_t* tgen = nullptr;   // [pair] the epoch its terms were written in
        uint32_t tepoch = 0;
        uint64_t t_rec_gen = 0;     // rec_gen as the last caching fold left it (unchanged since: terms current)
        uint64_t t_plain_gen = 0;   // rec_gen as the last re-scoring fold without the cache left it
        uint64_t* ndirty = nullptr;
        uint32_t chg_cap = 0;
        uint64_t* d_dig = nullptr;                 // message / word id digests of the call (k_mc_summary)
        size_t dig_cap = 0;
        void* h_stage = nullptr;  // pinned staging of a call's host-side inputs (messages, masks, set arrays)
        size_t h_stage_bytes = 0;
        uint32_t words_cap = 0, msgs_cap = 0, rows_cap = 0;
        size_t seen_words = 0;
        gsx::PropState last{};
        bool have_last = false;
        // the call in flight (gsx_prop_begin .. gsx_prop_end)
        bool active = false, sel_done = false;
        uint32_t h = 0;
        uint32_t rows_valid = 1;  // frontier-history rows written (skipped empty hops write none)
        uint32_t global_last = UINT32_MAX;  // range shards: the last hop delivering on any rank (gsx_prop_set_last_hop)
        gsx_prop_config cfg{};
        std::vector<uint64_t> ids;
        std::vector<uint32_t> vals;  // validation outcomes of this call
        std::vector<uint64_t> h_src;  // origins of this call's messages (set_sources; alive until the stream sync)
        std::vector<uint64_t> h_acc;  // accepted-message words (host copy, alive until the call's stream sync)
        // pending (deferred) credits: topic they belong to
        bool credit_pending = false;
        uint32_t credit_topic = 0;
        // per-hop kernel timing (gsx_propagate: one pair around its hop loop)
        std::vector<hipEvent_t> ev;
        uint32_t ev_used = 0;
        bool loop_timing = false;
        uint32_t launches = 0;
        // gsx_propagate's early stop: k_prop_mark reports every finished hop here
        uint32_t* hop_flag = nullptr;    // host-mapped [GSX_MAX_HOPS + 1]
        uint32_t* d_hop_flag = nullptr;  // its device address
        uint32_t hop_seq = 0;
        // fwd / pin of the last call, reused while nothing they read changed
        struct {
            bool valid = false;
            uint32_t router = 0, topic = 0, flood_publish = 0;
            uint64_t flag_gen = 0, score_gen = 0, mem_gen = 0;
            double publish_threshold = 0, graylist_threshold = 0;
        } fwd_key;
        bool fold_chg = false;  // the last call's fold listed fwd changes for the next call's pins
        bool flast_dirty = true;  // flast may hold a hop-tagged count of an earlier call (cleared before the next)
        // compacted shard exchange: the dense halo the received entries are
        // scattered into, the slots filled last hop, per-destination counts
        uint64_t* halo = nullptr;      // [receive slot][hop tag | W words] (PropState::halo_tag)
        uint64_t halo_tag = 0;         // this call's tag base: call serial << 8 (| hop)
        // replicated frontier (range shards, lean calls; PropState::rep)
        bool rep = false;
        uint64_t* front_g = nullptr;   // [2][n_total][W]
        uint64_t* occ_g = nullptr;     // [2][(n_total + 63) / 64 + 1]
        uint64_t* src_bits = nullptr;  // [(n_total + 63) / 64 + 1]
        uint64_t rep_words = 0;        // front_g capacity (words)
        uint32_t* src_ids = nullptr;   // [m] + the origin rows [m][W]
        uint64_t* src_rows = nullptr;
        uint64_t src_cap = 0;          // (messages x words)
        std::vector<uint32_t> h_src_ids;   // (host staging of the two above, alive until the call ends)
        std::vector<uint64_t> h_src_rows;
        uint64_t halo_calls = 0;
        uint32_t* pack_tab = nullptr;  // [pack block][rank] entry counts / offsets (k_pack_front)
        uint64_t pack_tab_cap = 0;
        uint64_t* hfrom = nullptr;     // [pair][word]: first receipts from the pair's remote sender, latest hop
        uint64_t* touch = nullptr;     // bit per node: marked by a sender (very sparse hops)
        uint64_t* vcnt = nullptr;      // per node: forwarded-set sizes (late duplicate accounting)
        uint64_t halo_cap = 0, hfrom_cap = 0;
        unsigned long long* dcount = nullptr;
    } prop;
    bool prop_track = true;  // gsx_prop_set_tracking: keep first-deliverer rows (gsx_prop_results)

    // range sharding (gsx_load_overlay_shard / gsx_shard_*_plan)
    uint32_t n_total = 0, node_lo = 0;
    uint32_t n_ranks = 1;
    std::vector<uint32_t> rank_lo;
    std::vector<uint64_t> recv_counts, send_counts;
    uint64_t n_recv = 0, n_send = 0;
    uint32_t* d_send_pair = nullptr;
    uint8_t* d_send_dest = nullptr;
    uint64_t *d_send_base = nullptr, *d_dest_halo_base = nullptr;
    uint32_t* d_pair_obs = nullptr;
    uint32_t* d_halo_node = nullptr;  // per receive slot: local node of its pair
    uint32_t* d_halo_pair = nullptr;  // per receive slot: its local pair (peer exchange)
    // replicated frontier (PropState::rep): the remote senders' global ids ascending,
    // and the local receiver of each (k_rep_scatter marks them on very sparse hops)
    uint32_t* d_rmark_v = nullptr;
    uint32_t* d_rmark_u = nullptr;
    uint32_t* d_send_slot = nullptr;  // per pair: its send slot, NO_PAIR if none (peer exchange)
    // peer exchange across shards: entries of this round's pack, per destination
    unsigned long long* d_pxs_cnt = nullptr;
    uint64_t* d_pxs_off = nullptr;
    std::vector<uint64_t> pxs_counts;
    bool pxs_packed[2] = {false, false};
    std::vector<uint32_t> rev_host;
    bool sharded() const { return n_ranks > 1 || node_lo != 0 || n_total != n_nodes; }
    hipStream_t own_stream = nullptr;
    // code-plane builds (k_prop_vcodes) beside the engine stream: vc_go marks
    // the engine-stream point a build starts after, vc_done[b] the last build
    // that read history buffer b (0: prop.hist as allocated, 1: hist_alt)
    hipStream_t vc_stream = nullptr;
    hipEvent_t vc_go = nullptr, vc_done[2] = {nullptr, nullptr};
    bool vc_busy[2] = {false, false};
    int hist_idx = 0, vc_last = -1;

    // events
    std::vector<gsx_event> pending;
    // what the queued events can change: their pairs' scores, and every score
    // of an observer with an AddPeer / RemovePeer (its IP groups' P6), so a
    // Score() of any other pair reads the host copy without a flush
    std::unordered_set<uint64_t> pend_pairs;
    std::unordered_set<uint32_t> pend_rows;
    void* h_stage = nullptr;
    size_t h_stage_bytes = 0;
    void* d_stage = nullptr;
    size_t d_stage_bytes = 0;
    bool staged_inflight = false;

    bool scores_valid = false;
    // Incremental re-scoring (gsx_score after events): an event touches only
    // its observer's state (the pair's counters, the observer's IP counts), so
    // when the scores were exact before a flush, only the flushed observers'
    // rows are re-scored (dirty_only + dirty_obs), through a pair mask.
    bool dirty_only = false;
    std::vector<uint32_t> dirty_obs;
    uint8_t* d_smask = nullptr;       // [pair] mask for launch_score_subset (kept all-zero between uses)
    uint32_t* d_dirty_obs = nullptr;  // observer list of the marking kernel
    size_t d_dirty_obs_cap = 0;
    // Host copy of the score vector for per-call Score() (engines up to
    // kHostScoreMax pairs, e.g. one router's peers): valid while no kernel has
    // written scores since it was taken (score_writes == h_score_tag).
    double* h_score = nullptr;  // pinned, host-mapped (k_dropin writes it; the full copy is one DMA)
    double* h_score_dev = nullptr;  // its device address
    size_t h_score_cap = 0;
    // the drop-in round trip (k_dropin): host-mapped [flag | events | groups | observers]
    void* h_dropin = nullptr;
    char* d_dropin = nullptr;  // its device address
    size_t h_dropin_bytes = 0;
    uint32_t dropin_tag = 0;
    uint64_t score_writes = 0, h_score_tag = ~0ull;
    bool dirty_zeroed = true;  // d_smask not cleared yet
    // Lazy folds (PropState::stale): the scores are exact but for the pairs
    // d_stale marks, whose stored score is a lower bound >= lazy_thr (every
    // fwd byte exact for thresholds up to lazy_thr); ensure_scores settles them.
    bool lazy = false;
    bool stale_marks = false;  // d_stale may hold marks (cleared before a lazy fold starts a new set)
    // Deferred folds (PropState::acc_s / acc_f): gossipsub calls sum the credits
    // of the pairs that keep their score instead of folding them; fold_deferred
    // folds the sums (topic def_topic) before anything reads records or scores.
    uint32_t *d_acc_s = nullptr, *d_acc_f = nullptr;
    bool deferred = false;
    uint32_t def_topic = 0, def_flood = 0;  // the topic and flood_publish setting the sums were deferred under
    double lazy_thr = 0;
    uint8_t* d_stale = nullptr;
    void invalidate_scores() {
        ++rec_gen;
        scores_valid = false;
        dirty_only = false;
        lazy = false;
        dirty_obs.clear();
    }
    void scores_exact() {  // every score was just computed
        scores_valid = true;
        dirty_only = false;
        lazy = false;
        dirty_obs.clear();
    }
    // generations: flag_gen moves with anything that may change pair / record
    // flags, the overlay or the thresholds; score_gen with anything that may
    // change a score (both with the former)
    uint64_t flag_gen = 1, score_gen = 1;
    uint64_t rec_gen = 1;  // with anything that may change a record other than the propagation fold
    void state_changed() {
        ++rec_gen;
        ++flag_gen;
        ++score_gen;
    }
    bool timed = false;
    // gsx_timing_begin/end: event pairs around each fused launch
    std::vector<hipEvent_t> tev;
    uint32_t t_max = 0, t_used = 0;
    bool t_active = false;

    // delivery records
    std::unordered_map<RecKey, DeliveryRecord, RecKeyHash> recs;
    std::unordered_map<uint32_t, std::deque<std::pair<uint64_t, int64_t>>> rec_queue;  // per observer FIFO
};

namespace {

int fail(gsx_engine* e, int code, const std::string& msg) {
    if (e) e->err = msg;
    return code;
}

#define HIPCHK(e, call)                                                                          \
    do {                                                                                         \
        hipError_t _st = (call);                                                                 \
        if (_st != hipSuccess)                                                                   \
            return fail((e), GSX_EDEVICE, std::string(#call ": ") + hipGetErrorString(_st));    \
    } while (0)

// Consecutive clears of a round queued as one k_zero_spans launch (flushed
// before the next kernel that reads them, or when full).
struct ZeroBatch {
    gsx_engine* e;
    gsx::ZeroSpans z{};
    explicit ZeroBatch(gsx_engine* e_) : e(e_) {}
    int add(void* p, size_t bytes) {
        if (!p || !bytes) return GSX_OK;
        if (z.k == gsx::ZERO_SPANS)
            if (int rc = flush()) return rc;
        z.p[z.k] = static_cast<uint8_t*>(p);
        z.n[z.k++] = bytes;
        return GSX_OK;
    }
    int flush() {
        if (!z.k) return GSX_OK;
        HIPCHK(e, gsx::launch_zero_spans(z, e->stream));
        z.k = 0;
        return GSX_OK;
    }
};

// A sharded gossip exchange (gsx_hb_end .. gsx_gx_end) holds the round's
// message sets, receipt rows and the mcache Shift: nothing that starts other
// work on the engine's state may run before gsx_gx_end.
int gx_busy(gsx_engine* e) {
    if (e->gxr.pending) return fail(e, GSX_ESTATE, "a sharded gossip exchange is in flight: gsx_gx_end first");
    return GSX_OK;
}

gsx::DevState dev_state(const gsx_engine* e) {
    gsx::DevState s{};
    s.rec = e->d_rec;
    s.rflags = e->d_rflags;
    s.pflags = e->d_pflags;
    s.expire = e->d_expire;
    s.bp = e->d_bp;
    s.app = e->d_app;
    s.ipg = e->d_ipg;
    s.ipcount = e->d_ipcount;
    s.score = e->d_score;
    s.tp = e->d_tp;
    s.n_pairs = e->E;
    s.n_topics = e->T;
    s.last_refresh = e->last_refresh;
    return s;
}

gsx::DevPeerParams dev_peer_params(const gsx_engine* e) {
    gsx::DevPeerParams d{};
    d.topic_score_cap = e->pp.topic_score_cap;
    d.w5 = e->pp.app_specific_weight;
    d.w6 = e->pp.ip_colocation_factor_weight;
    d.thr6 = e->pp.ip_colocation_factor_threshold;
    d.w7 = e->pp.behaviour_penalty_weight;
    d.thr7 = e->pp.behaviour_penalty_threshold;
    d.d7 = e->pp.behaviour_penalty_decay;
    d.decay_to_zero = e->pp.decay_to_zero;
    d.retain_ns = e->pp.retain_score_ns;
    return d;
}

gsx::DevTopicParams dev_topic_params(const gsx_engine* e, uint32_t t);

gsx::KernParams kern_params(const gsx_engine* e) {
    gsx::KernParams k{};
    k.pp = dev_peer_params(e);
    for (uint32_t t = 0; t < e->T && t < (uint32_t)gsx::KARG_TOPICS; ++t) k.tp[t] = dev_topic_params(e, t);
    return k;
}

gsx::DevTopicParams dev_topic_params(const gsx_engine* e, uint32_t t) {
    gsx::DevTopicParams d{};
    const gsx_topic_score_params& p = e->tp[t];
    d.topic_weight = p.topic_weight;
    d.w1 = p.time_in_mesh_weight;
    d.cap1 = p.time_in_mesh_cap;
    d.q1 = e->scored[t] ? p.time_in_mesh_quantum_ns : 1;  // unscored topics are skipped, never divided by
    d.w2 = p.first_message_deliveries_weight;
    d.d2 = p.first_message_deliveries_decay;
    d.cap2 = p.first_message_deliveries_cap;
    d.w3 = p.mesh_message_deliveries_weight;
    d.d3 = p.mesh_message_deliveries_decay;
    d.cap3 = p.mesh_message_deliveries_cap;
    d.thr3 = p.mesh_message_deliveries_threshold;
    d.win3 = p.mesh_message_deliveries_window_ns;
    d.act3 = p.mesh_message_deliveries_activation_ns;
    d.w3b = p.mesh_failure_penalty_weight;
    d.d3b = p.mesh_failure_penalty_decay;
    d.w4 = p.invalid_message_deliveries_weight;
    d.d4 = p.invalid_message_deliveries_decay;
    d.scored = e->scored[t] ? 1 : 0;
    return d;
}

int upload_topic_params(gsx_engine* e) {
    gsx::DevTopicParams h[GSX_MAX_TOPICS]{};
    for (uint32_t t = 0; t < e->T; ++t) h[t] = dev_topic_params(e, t);
    HIPCHK(e, hipMemcpyAsync(e->d_tp, h, sizeof(gsx::DevTopicParams) * GSX_MAX_TOPICS, hipMemcpyHostToDevice,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));  // `h` is on the stack
    return GSX_OK;
}

// Seen-row buffers cycle between the propagation call (its `seen`) and the
// message cache (a gossipsub batch keeps the call's buffer): a call hands its
// buffer to the cache instead of copying it, and takes one from this pool.
// Every buffer keeps the capacity it was carved with (seen_cap), whatever
// size the caller asked for, so a recycled buffer never looks smaller than
// it is; an acquisition takes the smallest free buffer that fits.
void seen_release(gsx_engine* e, uint64_t* p, size_t /*words*/) {
    if (!p) return;
    auto it = e->seen_cap.find(p);
    e->seen_pool.emplace_back(it != e->seen_cap.end() ? it->second : 0, p);
}
uint64_t* seen_acquire(gsx_engine* e, size_t words) {
    size_t best = e->seen_pool.size();
    for (size_t i = 0; i < e->seen_pool.size(); ++i)
        if (e->seen_pool[i].first >= words && (best == e->seen_pool.size() || e->seen_pool[i].first < e->seen_pool[best].first))
            best = i;
    if (best < e->seen_pool.size()) {
        uint64_t* p = e->seen_pool[best].second;
        e->seen_pool.erase(e->seen_pool.begin() + (long)best);
        return p;
    }
    // none free: small buffers come in slabs of kSlab (one hipMalloc per kSlab
    // acquisitions, not per propagation call: the call's host time is the
    // device's idle time between calls); a large one (a 10M-node overlay's
    // rows) is allocated alone, so the pool never reserves 4x a peak
    constexpr size_t kSlab = 4, kSlabMaxBytes = 64ull << 20;
    const size_t w = (std::max<size_t>(words, 1) + 31) & ~(size_t)31;  // (256-B aligned buffers)
    const size_t n = 8 * w <= kSlabMaxBytes ? kSlab : 1;
    uint64_t* p = nullptr;
    if (hipMalloc((void**)&p, 8 * w * n) != hipSuccess) {
        if (n == 1 || hipMalloc((void**)&p, 8 * w) != hipSuccess) return nullptr;  // (a tight device: one buffer)
        e->pool_slabs.push_back(p);
        e->seen_cap[p] = w;
        return p;
    }
    e->pool_slabs.push_back(p);
    for (size_t k = 0; k < n; ++k) e->seen_cap[p + k * w] = w;
    for (size_t k = 1; k < n; ++k) e->seen_pool.emplace_back(w, p + k * w);
    return p;
}
void seen_pool_free(gsx_engine* e) {
    e->seen_pool.clear();
    e->small_pool.clear();
    e->seen_cap.clear();
    for (void* x : e->pool_slabs) (void)hipFree(x);
    e->pool_slabs.clear();
}
// Small per-set device arrays (validation outcomes, accepted words, id
// digests, the `full` bytes) from a recycled pool: no hipMalloc / hipFree per
// propagation call (a hipFree waits for the whole device).
uint8_t* small_acquire(gsx_engine* e, size_t bytes, size_t* got) {
    for (size_t i = 0; i < e->small_pool.size(); ++i)
        if (e->small_pool[i].first >= bytes && e->small_pool[i].first <= 4 * bytes + 4096) {
            uint8_t* p = e->small_pool[i].second;
            *got = e->small_pool[i].first;
            e->small_pool.erase(e->small_pool.begin() + (long)i);
            return p;
        }
    constexpr size_t kSlab = 16;  // (as seen_acquire: one hipMalloc per kSlab arrays)
    const size_t b = (std::max<size_t>(bytes, 256) + 255) & ~(size_t)255;
    uint8_t* p = nullptr;
    if (hipMalloc((void**)&p, b * kSlab) != hipSuccess) return nullptr;
    e->pool_slabs.push_back(p);
    for (size_t k = 1; k < kSlab; ++k) e->small_pool.emplace_back(b, p + k * b);
    *got = b;
    return p;
}
void small_release(gsx_engine* e, uint8_t* p, size_t bytes) {
    if (p) e->small_pool.emplace_back(bytes, p);
}
// A message set's d_val (m u32) / d_acc (W u64) / d_dg (W * 64 + W u64) /
// d_src (m u64) in one pooled block.
bool set_small_alloc(gsx_engine* e, gsx_engine::MsgSet* set, size_t m, uint32_t W) {
    const size_t val_b = (4 * std::max<size_t>(m, 1) + 7) & ~(size_t)7;
    const size_t bytes = val_b + 8 * (size_t)W + 8 * ((size_t)W * 64 + W) + 8 * std::max<size_t>(m, 1);
    set->d_small = small_acquire(e, bytes, &set->small_bytes);
    if (!set->d_small) return false;
    set->d_val = reinterpret_cast<uint32_t*>(set->d_small);
    set->d_acc = reinterpret_cast<uint64_t*>(set->d_small + val_b);
    set->d_dg = set->d_acc + W;
    set->d_src = set->d_dg + (size_t)W * 64 + W;
    return true;
}
// The origins of a set's messages, (source << 32 | index) ascending.
void set_sources(std::vector<uint64_t>& out, const gsx_msg* msgs, size_t m) {
    out.resize(m);
    for (size_t k = 0; k < m; ++k) out[k] = (uint64_t)msgs[k].source << 32 | (uint64_t)k;
    std::sort(out.begin(), out.end());
}

template <class T>
int dalloc(gsx_engine* e, T** p, size_t n);
uint32_t bit_width32(uint32_t x) { return x ? 32u - (uint32_t)__builtin_clz(x) : 0u; }
// The engine stream waits for every queued code-plane build (before anything
// reads, copies, regrows or pools a set's planes).
int vc_fence(gsx_engine* e) {
    if (e->vc_last < 0) return GSX_OK;
    HIPCHK(e, hipStreamWaitEvent(e->stream, e->vc_done[e->vc_last], 0));
    e->vc_last = -1;
    return GSX_OK;
}
// A set's code planes grown to p planes (the new ones zero: code bits above
// the old width are 0); p <= VC_MAX_PLANES.
int vc_grow(gsx_engine* e, gsx_engine::MsgSet* st, uint32_t p) {
    if (p <= st->vc_p) return GSX_OK;
    if (st->d_vc)
        if (int rc = vc_fence(e)) return rc;
    if (p > gsx::VC_MAX_PLANES) return fail(e, GSX_ERANGE, "a message set's validation codes past 2^16 (recovered in 65k rounds)");
    const size_t plane = (size_t)st->n_words * e->n_nodes;
    const size_t words = std::max<size_t>(plane * p, 1);
    uint64_t* vc = seen_acquire(e, words);
    if (!vc) return fail(e, GSX_ENOMEM, "message set validation codes");
    if (st->d_vc && plane)
        HIPCHK(e, hipMemcpyAsync(vc, st->d_vc, 8 * plane * st->vc_p, hipMemcpyDeviceToDevice, e->stream));
    if (plane) HIPCHK(e, hipMemsetAsync(vc + plane * st->vc_p, 0, 8 * plane * (p - st->vc_p), e->stream));
    seen_release(e, st->d_vc, st->vc_words);
    st->d_vc = vc;
    st->vc_words = words;
    st->vc_p = p;
    return GSX_OK;
}

// A propagation call's arrival hops into its message set's code planes, on
// vc_stream after the engine stream's work so far; the next call writes the
// other history buffer (it waits for the build that read it two calls back).
int vc_build(gsx_engine* e, const gsx::PropState& ps, gsx_engine::MsgSet* set) {
    auto& P = e->prop;
    if (!e->vc_stream) {
        HIPCHK(e, hipStreamCreateWithFlags(&e->vc_stream, hipStreamNonBlocking));
        HIPCHK(e, hipEventCreateWithFlags(&e->vc_go, hipEventDisableTiming));
        for (auto& ev : e->vc_done) HIPCHK(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    if (!P.hist_alt) {
        const size_t N = e->n_nodes;
        if (int rc = dalloc(e, &P.hist_alt, (size_t)P.rows_cap * P.words_cap * N)) return rc;
        if (int rc = dalloc(e, &P.occ_alt, (size_t)P.rows_cap * ((N + 63) / 64))) return rc;
    }
    HIPCHK(e, hipEventRecord(e->vc_go, e->stream));
    HIPCHK(e, hipStreamWaitEvent(e->vc_stream, e->vc_go, 0));
    HIPCHK(e, gsx::launch_prop_vcodes(ps, set->d_vc, set->vc_p, e->vc_stream));
    const int b = e->hist_idx;
    HIPCHK(e, hipEventRecord(e->vc_done[b], e->vc_stream));
    e->vc_busy[b] = true;
    e->vc_last = b;
    std::swap(P.hist, P.hist_alt);
    std::swap(P.occ, P.occ_alt);
    e->hist_idx ^= 1;
    if (e->vc_busy[e->hist_idx]) {  // the buffer the next call writes: its build first
        HIPCHK(e, hipStreamWaitEvent(e->stream, e->vc_done[e->hist_idx], 0));
        e->vc_busy[e->hist_idx] = false;
    }
    return GSX_OK;
}

void set_release(gsx_engine* e, gsx_engine::MsgSet* st) {
    if (!st || --st->refs > 0) return;
    if (st->d_vc) (void)vc_fence(e);  // (a build may still write the planes going back to the pool)
    seen_release(e, st->d_all, st->all_words);
    seen_release(e, st->d_vc, st->vc_words);
    seen_release(e, st->xs_spare, 0);
    small_release(e, reinterpret_cast<uint8_t*>(st->d_common), st->common_bytes);
    small_release(e, st->d_small, st->small_bytes);
    small_release(e, st->d_full, st->full_bytes);
    delete st;
}
void batch_release(gsx_engine* e, gsx_engine::McBatch& b) {
    seen_release(e, b.d_seen, b.seen_words);
    set_release(e, b.set);
    b.d_seen = nullptr;
    b.set = nullptr;
}

void mcache_clear(gsx_engine* e) {
    for (auto& w : e->mc)
        for (auto& b : w) batch_release(e, b);
    e->mc.clear();
    e->mc.emplace_back();  // history[0], empty
}

// Drops the exchange in flight (a failed step, or teardown): its receipt
// rows, frontier rows and set references go back to the pools.
void gx_abort(gsx_engine* e) {
    auto& R = e->gxr;
    (void)hipStreamSynchronize(e->stream);
    for (auto& fr : R.scratch) seen_release(e, fr.first, fr.second);
    for (size_t i = 0; i < R.xs.size() && i < R.sets.size(); ++i)
        seen_release(e, R.xs[i], (size_t)R.sets[i]->n_words * e->n_nodes + 2 * (size_t)e->n_nodes);
    for (auto* ms : R.sets) {
        ms->full_ok = false;
        set_release(e, ms);
    }
    R.scratch.clear();
    R.sets.clear();
    R.xs.clear();
    R.runs.clear();
    R.pending = R.run = R.fwd_active = false;
    R.stage = 0;
}

void free_state(gsx_engine* e) {
    if (e->vc_stream) (void)hipStreamSynchronize(e->vc_stream);  // (code-plane builds in flight)
    e->vc_busy[0] = e->vc_busy[1] = false;
    e->hist_idx = 0;
    e->vc_last = -1;
    gx_abort(e);
    void* ptrs[] = {e->d_rec,    e->d_rflags, e->d_tmp, e->d_nbad,    e->d_pflags, e->d_eflags,
                    e->d_expire, e->d_bp,     e->d_app, e->d_score,   e->d_ipg,    e->d_ipcount,
                    e->d_col};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    e->d_rec = nullptr;
    e->d_tmp = nullptr;
    e->d_nbad = nullptr;
    e->d_rflags = e->d_pflags = e->d_eflags = nullptr;
    e->d_expire = nullptr;
    e->d_bp = e->d_app = e->d_score = nullptr;
    e->d_ipg = e->d_ipcount = nullptr;
    if (e->d_row_ptr) (void)hipFree(e->d_row_ptr);
    if (e->d_rev) (void)hipFree(e->d_rev);
    e->d_row_ptr = nullptr;
    e->d_rev = nullptr;
    if (e->d_smask) (void)hipFree(e->d_smask);
    if (e->d_dirty_obs) (void)hipFree(e->d_dirty_obs);
    if (e->d_stale) (void)hipFree(e->d_stale);
    e->d_stale = nullptr;
    if (e->d_acc_s) (void)hipFree(e->d_acc_s);
    if (e->d_acc_f) (void)hipFree(e->d_acc_f);
    e->d_acc_s = e->d_acc_f = nullptr;
    e->deferred = false;
    e->stale_marks = false;
    e->d_smask = nullptr;
    e->d_dirty_obs = nullptr;
    e->d_dirty_obs_cap = 0;
    e->dirty_zeroed = true;
    e->invalidate_scores();
    e->h_score_tag = ~0ull;
    // (prop.seen is a pool buffer: seen_pool_free below frees its slab)
    void* pp[] = {e->prop.hist, e->prop.origin, e->prop.from,
                  e->prop.sel,  e->prop.fwd,  e->prop.pin,    e->prop.dup,   e->prop.corr,
                  e->prop.first, e->prop.msgs, e->prop.stats, e->d_send_pair, e->d_pair_obs,
                  e->prop.halo, e->prop.pack_tab, e->prop.dcount, e->d_send_dest, e->d_send_base,
                  e->d_dest_halo_base, e->prop.fcnt, e->prop.flast, e->prop.hfrom, e->prop.inv, e->prop.vmask, e->prop.dseen,
                  e->prop.touch, e->prop.vcnt, e->d_halo_node, e->prop.occ, e->prop.gray_pairs,
                  e->prop.cent, e->prop.cend, e->prop.chg, e->prop.nchg, e->prop.ndirty, e->prop.rfwd,
                  e->d_halo_pair, e->d_send_slot, e->d_rmark_v, e->d_rmark_u, e->prop.front_g, e->prop.occ_g,
                  e->prop.src_bits, e->prop.src_ids, e->prop.src_rows,
                  e->prop.d_dig, e->prop.rcand, e->prop.tterm, e->prop.tgen, e->prop.hist_alt, e->prop.occ_alt};
    for (void* p : pp)
        if (p) (void)hipFree(p);
    std::vector<hipEvent_t> evs = std::move(e->prop.ev);
    uint32_t *hf = e->prop.hop_flag, *dhf = e->prop.d_hop_flag;
    const uint32_t hseq = e->prop.hop_seq;
    e->prop = {};
    e->prop.ev = std::move(evs);
    e->prop.hop_flag = hf;
    e->prop.d_hop_flag = dhf;
    e->prop.hop_seq = hseq;
    e->d_send_pair = e->d_pair_obs = e->d_halo_node = e->d_halo_pair = e->d_send_slot = nullptr;
    e->d_rmark_v = e->d_rmark_u = nullptr;
    e->d_send_dest = nullptr;
    e->d_send_base = e->d_dest_halo_base = nullptr;
    e->n_ranks = 1;
    e->rank_lo.clear();
    e->recv_counts.clear();
    e->send_counts.clear();
    e->n_recv = e->n_send = 0;
    e->d_col = nullptr;
    void* hb[] = {e->d_work, e->d_hubwork, e->d_nwork, e->d_hubs, e->d_tcnt, e->d_mcount,
                  e->d_backoff, e->d_bo8, e->d_ctl, e->d_resp,   e->d_dirty,     e->d_long,
                  e->d_nlong,   e->d_hbstats,   e->d_tr_acc,    e->d_tr_hp,   e->d_rngk,      e->d_ihave_slot, e->d_gelig, e->d_gb,
                  e->d_mc_digest, e->d_ihave_unit, e->d_ihave_tag};
    for (void* p : hb)
        if (p) (void)hipFree(p);
    e->d_backoff = nullptr;
    e->d_bo8 = nullptr;
    e->d_ctl = e->d_resp = nullptr;
    e->d_dirty = nullptr;
    e->d_long = e->d_nlong = nullptr;
    e->d_hbstats = nullptr;
    e->d_tr_acc = e->d_tr_hp = nullptr;
    {
        void* gxp[] = {e->d_gxreq, e->d_gxflag, e->d_prom_h,
                       e->d_ihave_bits, e->d_prom_e, e->d_prom_any, e->d_prom_cnt, e->d_gxa,
                       e->d_gx_got, e->d_gx_nodes,
                       e->d_gx_rhm, e->d_gx_common,
                       e->d_gxf_mask, e->d_gxf_list, e->d_gxf_cnt, e->d_gxf_bst, e->d_gxf_b0, e->d_gxf_b,
                       e->d_gxf_sets, e->d_gxf_fin, e->d_gxf_fout, e->d_gxf_fent, e->d_gxf_fend, e->d_gxf_hst, e->d_gxs_out, e->d_gxs_rans,
                       e->d_gxs_hidx, e->d_gxs_cnt, e->d_gxs_off, e->d_gxs_send};
        for (void* x : gxp)
            if (x) (void)hipFree(x);
        e->d_gxf_mask = nullptr;
        e->d_gxf_list = e->d_gxf_cnt = e->d_gxf_bst = nullptr;
        e->d_gxf_b0 = nullptr;
        e->gxf_b0_grps = 0;
        e->d_gxf_b = nullptr;
        e->d_gxf_sets = nullptr;
        e->d_gxf_fin = nullptr;
        e->d_gxf_fout = nullptr;
        e->d_gxf_fent = nullptr;
        e->d_gxf_fend = nullptr;
        e->d_gxf_hst = nullptr;
        e->d_gxs_out = nullptr;
        e->d_gxs_rans = nullptr;
        e->d_gxs_hidx = nullptr;
        e->d_gxs_cnt = nullptr;
        e->d_gxs_off = nullptr;
        e->d_gxs_send = nullptr;
        e->gxs_send_cap = 0;
        e->gxf_sets_cap = 0;
        e->d_gxreq = e->d_gxflag = e->d_gx_nodes = nullptr;
        e->d_prom_h = e->d_ihave_bits = nullptr;
        e->ihave_tr_dirty = true;  // (a new array is cleared whole)
        e->d_prom_e = nullptr;
        e->d_prom_any = nullptr;
        e->d_prom_cnt = nullptr;
        e->prom_slots = 0;
        for (auto& sp : e->subp) {
            if (sp.pool) (void)hipFree(sp.pool);
            if (sp.idx) (void)hipFree(sp.idx);
        }
        e->subp.clear();
        if (e->d_sub_cnt) (void)hipFree(e->d_sub_cnt);
        if (e->d_gsubs) (void)hipFree(e->d_gsubs);
        e->d_sub_cnt = nullptr;
        e->d_gsubs = nullptr;
        e->tgt_dlazy = -1;
        e->d_gxa = nullptr;
        e->gxa_bytes = 0;
        e->d_gx = nullptr;
        e->d_gx_off = nullptr;
        e->d_gx_got = nullptr;
        e->gx_cap = 0;
        e->d_gx_rhm = e->d_gx_common = nullptr;
        if (e->d_gx_vin) (void)hipFree(e->d_gx_vin);
        e->d_gx_vin = nullptr;
        e->gx_vin_cap = 0;
        e->d_gx_chg = nullptr;  // (d_gx_got's second half)
        e->d_gx_wb = nullptr;
        e->d_gx_sw = nullptr;
        e->d_gx_sp = nullptr;
        e->d_gx_mg = nullptr;
        e->gx_common_cap = 0;
        void* mbp[] = {e->d_sub, e->d_psub, e->d_fanout, e->d_fan_has, e->d_lastpub, e->d_mscratch, e->d_mlist};
        for (void* x : mbp)
            if (x) (void)hipFree(x);
        e->d_sub = e->d_psub = e->d_fanout = e->d_fan_has = nullptr;
        e->d_lastpub = nullptr;
        e->d_mscratch = e->d_mlist = nullptr;
        e->mlist_cap = 0;
        e->members_on = false;
        e->h_sub.clear();
        void* pxp[] = {e->d_pxno, e->d_pxscratch, e->d_pxlog, e->d_pxbase};
        for (void* x : pxp)
            if (x) (void)hipFree(x);
        e->d_pxno = nullptr;
        e->d_pxscratch = e->d_pxlog = e->d_pxbase = nullptr;
        e->pxlog_alloc = 0;
        e->px_last = 0;
    }
    e->d_rngk = nullptr;
    e->d_ihave_slot = e->d_ihave_unit = nullptr;
    e->d_ihave_tag = nullptr;
    e->d_work = e->d_hubwork = e->d_nwork = e->d_hubs = nullptr;
    e->d_tcnt = nullptr;
    e->d_mcount = nullptr;
    e->d_gelig = nullptr;
    e->ihave_round = 0;
    e->d_gb = nullptr;
    e->d_mc_digest = nullptr;
    e->gb_cap = e->ids_cap = 0;
    e->have_gossip = false;
    mcache_clear(e);
    seen_pool_free(e);
}

template <class T>
int dalloc(gsx_engine* e, T** p, size_t n) {
    hipError_t st = hipMalloc((void**)p, sizeof(T) * (n ? n : 1));
    if (st != hipSuccess) return fail(e, GSX_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(st));
    return GSX_OK;
}

// Staging buffer for one topic-major record field (import / export only).
int ensure_tmp(gsx_engine* e) {
    if (e->d_tmp) return GSX_OK;
    const size_t bytes = 8 * (size_t)e->T * (e->E ? e->E : 1);
    hipError_t st = hipMalloc(&e->d_tmp, bytes);
    if (st != hipSuccess) return fail(e, GSX_ENOMEM, std::string("hipMalloc(staging): ") + hipGetErrorString(st));
    return GSX_OK;
}

void release_tmp(gsx_engine* e) {
    if (e->d_tmp) (void)hipFree(e->d_tmp);
    e->d_tmp = nullptr;
}

int upload_ipg(gsx_engine* e) {
    std::vector<uint32_t> ipg(e->ipg_host.size());
    for (size_t i = 0; i < ipg.size(); ++i) {
        uint32_t g = e->ipg_host[i];
        if (g != gsx::IPG_NONE) {
            uint32_t ip = e->group_ip[g];
            if (ip < e->ip_wl.size() && e->ip_wl[ip]) g |= gsx::IPG_WL;
        }
        ipg[i] = g;
    }
    HIPCHK(e, hipMemcpy(e->d_ipg, ipg.data(), sizeof(uint32_t) * (ipg.size() ? ipg.size() : 0),
                        hipMemcpyHostToDevice));
    return GSX_OK;
}

void pending_note(gsx_engine* e, uint32_t kind, uint64_t pair) {
    if (kind == GSX_EV_ADD_PEER || kind == GSX_EV_REMOVE_PEER)
        e->pend_rows.insert(pair < e->pair_obs.size() ? e->pair_obs[pair] : 0xFFFFFFFFu);
    else
        e->pend_pairs.insert(pair);
}
void pending_clear(gsx_engine* e) {
    e->pending.clear();
    e->pend_pairs.clear();
    e->pend_rows.clear();
}
// Whether a queued event can change the score of `pair` (the pending sets).
bool pending_touches(const gsx_engine* e, uint64_t pair) {
    return e->pend_pairs.count(pair) || e->pend_rows.count(pair < e->pair_obs.size() ? e->pair_obs[pair] : 0u) ||
           e->pend_rows.count(0xFFFFFFFFu);
}

int fold_deferred(gsx_engine* e);

// Applies queued events on the device (score.go:588-974 via k_apply_events).
int flush(gsx_engine* e) {
    if (e->pending.empty()) return GSX_OK;
    if (int rc = fold_deferred(e)) return rc;  // the queued events came after the deferred credits
    if (!e->loaded) return fail(e, GSX_ESTATE, "events before gsx_load_overlay");
    const size_t n = e->pending.size();
    // stable grouping by observer: order inside each observer is preserved
    std::vector<uint32_t> obs(n);
    for (size_t i = 0; i < n; ++i) {
        if (e->pending[i].pair >= e->E) {
            pending_clear(e);
            return fail(e, GSX_ERANGE, "event pair out of range");
        }
        obs[i] = e->pair_obs[e->pending[i].pair];
    }
    std::vector<uint32_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return obs[a] < obs[b]; });
    std::vector<uint32_t> group_off;
    group_off.reserve(64);
    for (size_t i = 0; i < n; ++i)
        if (i == 0 || obs[order[i]] != obs[order[i - 1]]) group_off.push_back((uint32_t)i);
    const uint32_t n_groups = (uint32_t)group_off.size();
    group_off.push_back((uint32_t)n);

    const size_t ev_bytes = sizeof(gsx::DevEvent) * n;
    const size_t off_bytes = sizeof(uint32_t) * group_off.size();
    const size_t total = ev_bytes + off_bytes;
    if (e->staged_inflight) {
        HIPCHK(e, hipEventSynchronize(e->ev_staged));
        e->staged_inflight = false;
    }
    if (e->h_stage_bytes < total) {
        if (e->h_stage) (void)hipHostFree(e->h_stage);
        e->h_stage = nullptr;
        size_t want = std::max(total, e->h_stage_bytes * 2);
        HIPCHK(e, hipHostMalloc(&e->h_stage, want, hipHostMallocDefault));
        e->h_stage_bytes = want;
    }
    if (e->d_stage_bytes < total) {
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (e->d_stage) (void)hipFree(e->d_stage);
        e->d_stage = nullptr;
        size_t want = std::max(total, e->d_stage_bytes * 2);
        HIPCHK(e, hipMalloc(&e->d_stage, want));
        e->d_stage_bytes = want;
    }
    auto* hev = static_cast<gsx::DevEvent*>(e->h_stage);
    for (size_t i = 0; i < n; ++i) {
        const gsx_event& s = e->pending[order[i]];
        hev[i] = gsx::DevEvent{s.kind, s.topic, s.pair, s.now_ns, s.arg};
    }
    std::memcpy(static_cast<char*>(e->h_stage) + ev_bytes, group_off.data(), off_bytes);
    HIPCHK(e, hipMemcpyAsync(e->d_stage, e->h_stage, total, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipEventRecord(e->ev_staged, e->stream));
    e->staged_inflight = true;
    const auto* dev = static_cast<const gsx::DevEvent*>(e->d_stage);
    const auto* doff = reinterpret_cast<const uint32_t*>(static_cast<const char*>(e->d_stage) + ev_bytes);
    HIPCHK(e, gsx::launch_apply_events(dev_state(e), dev_peer_params(e), dev, doff, n_groups, e->stream));
    pending_clear(e);
    if (e->scores_valid || e->dirty_only || e->lazy) {  // exact but for these observers (and the stale pairs)
        for (uint32_t g = 0; g < n_groups; ++g) e->dirty_obs.push_back(obs[order[group_off[g]]]);
        e->scores_valid = false;
        e->dirty_only = true;
    }
    e->state_changed();
    return GSX_OK;
}

// IHAVE digest term of one message id (gsx.h, gsx_gossip_results)
uint64_t id_digest(uint64_t id) {
    uint64_t z = id + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Every score write goes through these two (the host score copy keys on score_writes).
hipError_t rescore_all(gsx_engine* e, const gsx::DevState& ds, int64_t now, bool refresh) {
    ++e->score_writes;
    return gsx::launch_refresh_score(ds, kern_params(e), now, refresh, e->stream);
}
hipError_t rescore_subset(gsx_engine* e, const gsx::DevState& ds, const gsx::KernParams& kp, const uint8_t* mask,
                          const uint8_t* mask2 = nullptr, const unsigned long long* gate = nullptr) {
    ++e->score_writes;
    return gsx::launch_score_subset(ds, kp, mask, e->stream, mask2, gate);
}
// The heartbeat's masked re-scores on one engine mark only pairs that carried
// control (GRAFT / PRUNE sent in (A): dirty, inbox; handled in (B), answered in
// (C)): with none sent the passes have nothing to do (the kernel reads the two
// counters and returns).  A range shard's (B) takes control from other ranks:
// never gated there.
const unsigned long long* hb_ctl_gate(const gsx_engine* e) {
    return e->sharded() ? nullptr : e->d_hbstats + gsx::HB_GRAFTS;  // (HB_GRAFTS, HB_PRUNES: adjacent)
}

// The largest threshold a propagation fwd byte tests (k_prop_fwd: publishThreshold, graylistThreshold).
double lazy_threshold(const gsx_engine* e) {
    return std::max(e->th.publish_threshold, e->th.graylist_threshold);
}

// Whether P2 / P3 credits can only raise a score: every scored topic has the
// signs TopicScoreParams.validate asks (score_params.go:207-236).
bool credits_raise_scores(const gsx_engine* e) {
    for (uint32_t t = 0; t < e->T; ++t) {
        if (!e->scored[t]) continue;
        const gsx_topic_score_params& p = e->tp[t];
        if (!(p.topic_weight >= 0 && p.first_message_deliveries_weight >= 0 && p.mesh_message_deliveries_weight <= 0))
            return false;
    }
    return true;
}

// The dirty observer list on the device (sorted, unique) -> GSX_OK.
int upload_dirty_obs(gsx_engine* e) {
    std::vector<uint32_t>& d = e->dirty_obs;
    if (!e->d_dirty_obs || e->d_dirty_obs_cap < d.size()) {
        if (e->d_dirty_obs) {
            HIPCHK(e, hipStreamSynchronize(e->stream));
            (void)hipFree(e->d_dirty_obs);
            e->d_dirty_obs = nullptr;
        }
        e->d_dirty_obs_cap = std::max<size_t>(d.size(), 2 * e->d_dirty_obs_cap);
        if (int rc = dalloc(e, &e->d_dirty_obs, e->d_dirty_obs_cap)) return rc;
    }
    HIPCHK(e, hipMemcpyAsync(e->d_dirty_obs, d.data(), 4 * d.size(), hipMemcpyHostToDevice, e->stream));
    return GSX_OK;
}

// The deferred folds' sums into the records (their pairs marked stale: the
// next settle re-scores them); a no-op when nothing is deferred.
int fold_deferred(gsx_engine* e) {
    if (!e->deferred) return GSX_OK;
    e->deferred = false;
    gsx::PropState ps{};
    ps.n_pairs = e->E;
    ps.topic = e->def_topic;
    ps.rev = e->d_rev;
    ps.acc_s = e->d_acc_s;
    ps.acc_f = e->d_acc_f;
    ps.stale = e->d_stale;
    HIPCHK(e, gsx::launch_prop_fold_acc(ps, dev_state(e), e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_acc_s, 0, 4 * std::max<size_t>(e->E, 1), e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_acc_f, 0, 4 * std::max<size_t>(e->E, 1), e->stream));
    e->stale_marks = true;
    ++e->rec_gen;  // (records changed: the fold's topic-term cache starts a new epoch)
    return GSX_OK;
}
// The records are being replaced (import, synthesis): the sums are dropped.
int drop_deferred(gsx_engine* e) {
    if (!e->deferred) return GSX_OK;
    e->deferred = false;
    HIPCHK(e, hipMemsetAsync(e->d_acc_s, 0, 4 * std::max<size_t>(e->E, 1), e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_acc_f, 0, 4 * std::max<size_t>(e->E, 1), e->stream));
    return GSX_OK;
}

// Lazy folds left stale pairs (PropState::stale): re-score them and the
// dirty observers' rows (events since), then clear the marks.
int settle_stale(gsx_engine* e) {
    std::vector<uint32_t>& d = e->dirty_obs;
    if (e->dirty_only && !d.empty()) {
        std::sort(d.begin(), d.end());
        d.erase(std::unique(d.begin(), d.end()), d.end());
        if (int rc = upload_dirty_obs(e)) return rc;
        HIPCHK(e, gsx::launch_mark_rows(e->d_row_ptr, e->d_dirty_obs, (uint32_t)d.size(), e->d_stale, 1, e->stream));
    }
    HIPCHK(e, rescore_subset(e, dev_state(e), kern_params(e), e->d_stale));
    HIPCHK(e, hipMemsetAsync(e->d_stale, 0, std::max<size_t>(e->E, 1), e->stream));
    e->stale_marks = false;
    if (e->dirty_only && !d.empty()) HIPCHK(e, hipStreamSynchronize(e->stream));  // (the list was read)
    e->scores_exact();
    return GSX_OK;
}

int ensure_scores(gsx_engine* e) {
    if (int rc = fold_deferred(e)) return rc;
    int rc = flush(e);
    if (rc) return rc;
    if (e->scores_valid) return GSX_OK;
    if (e->lazy) return settle_stale(e);
    std::vector<uint32_t>& d = e->dirty_obs;
    uint64_t n_dirty = 0;
    if (e->dirty_only) {
        std::sort(d.begin(), d.end());
        d.erase(std::unique(d.begin(), d.end()), d.end());
        for (uint32_t o : d) n_dirty += (uint64_t)(e->row_ptr[o + 1] - e->row_ptr[o]);
    }
    if (e->dirty_only && n_dirty * 8 < e->E) {  // a few observers: their rows only
        if (!e->d_smask && (rc = dalloc(e, &e->d_smask, e->E))) return rc;
        if ((rc = upload_dirty_obs(e))) return rc;
        if (e->dirty_zeroed) {  // first use: the mask starts all-zero
            HIPCHK(e, hipMemsetAsync(e->d_smask, 0, e->E, e->stream));
            e->dirty_zeroed = false;
        }
        HIPCHK(e, gsx::launch_mark_rows(e->d_row_ptr, e->d_dirty_obs, (uint32_t)d.size(), e->d_smask, 1, e->stream));
        HIPCHK(e, rescore_subset(e, dev_state(e), kern_params(e), e->d_smask));
        HIPCHK(e, gsx::launch_mark_rows(e->d_row_ptr, e->d_dirty_obs, (uint32_t)d.size(), e->d_smask, 0, e->stream));
        // the observer list is read by the kernels above: keep it until they ran
        HIPCHK(e, hipStreamSynchronize(e->stream));
    } else {
        HIPCHK(e, rescore_all(e, dev_state(e), 0, false));
    }
    e->scores_exact();
    return GSX_OK;
}

void push_event(gsx_engine* e, uint32_t kind, uint64_t pair, uint32_t topic, int64_t now, int64_t arg) {
    e->pending.push_back(gsx_event{kind, topic, pair, now, arg});
    pending_note(e, kind, pair);
}

// messageDeliveries.getRecord, score.go:833-854
DeliveryRecord& get_record(gsx_engine* e, uint32_t obs, uint64_t msg, int64_t now) {
    auto it = e->recs.find(RecKey{obs, msg});
    if (it != e->recs.end()) return it->second;
    DeliveryRecord& r = e->recs[RecKey{obs, msg}];
    r.first_seen = now;
    e->rec_queue[obs].emplace_back(msg, now + kTimeCacheDuration);
    return r;
}

// markDuplicateMessageDelivery's window test (score.go:962-967), on the host
// because it needs only the record's validated time; the inMesh test runs on
// the device.
void mark_duplicate(gsx_engine* e, uint64_t pair, uint32_t topic, bool validated_set, int64_t validated,
                    int64_t now) {
    if (topic >= e->T || !e->scored[topic]) return;
    if (validated_set && (now - validated) > e->tp[topic].mesh_message_deliveries_window_ns) return;
    push_event(e, GSX_EV_MESH_DELIVERY, pair, topic, now, 0);
}

bool has_peer(const DeliveryRecord& r, uint64_t p) {
    return std::find(r.peers.begin(), r.peers.end(), p) != r.peers.end();
}

int check_pair(gsx_engine* e, uint64_t pair) {
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (pair >= e->E) return fail(e, GSX_ERANGE, "pair out of range");
    return GSX_OK;
}

}  // namespace

// ==== C ABI ===================================================================

extern "C" {

int gsx_abi_version(void) { return GSX_ABI_VERSION; }

const char* gsx_last_error(gsx_engine* e) { return e ? e->err.c_str() : "null engine"; }

// PeerScoreThresholds.validate, score_params.go:34-51
int gsx_validate_thresholds(const gsx_thresholds* p) {
    if (!p) return GSX_EINVAL;
    if (p->gossip_threshold > 0 || invalid_number(p->gossip_threshold)) return GSX_EINVAL;
    if (p->publish_threshold > 0 || p->publish_threshold > p->gossip_threshold || invalid_number(p->publish_threshold))
        return GSX_EINVAL;
    if (p->graylist_threshold > 0 || p->graylist_threshold > p->publish_threshold ||
        invalid_number(p->graylist_threshold))
        return GSX_EINVAL;
    if (p->accept_px_threshold < 0 || invalid_number(p->accept_px_threshold)) return GSX_EINVAL;
    if (p->opportunistic_graft_threshold < 0 || invalid_number(p->opportunistic_graft_threshold)) return GSX_EINVAL;
    return GSX_OK;
}

// PeerScoreParams.validate, score_params.go:151-198 (without the Topics loop)
int gsx_validate_peer_params(const gsx_peer_score_params* p) {
    if (!p) return GSX_EINVAL;
    if (p->topic_score_cap < 0 || invalid_number(p->topic_score_cap)) return GSX_EINVAL;
    if (!p->app_specific_score_set) return GSX_EINVAL;
    if (p->ip_colocation_factor_weight > 0 || invalid_number(p->ip_colocation_factor_weight)) return GSX_EINVAL;
    if (p->ip_colocation_factor_weight != 0 && p->ip_colocation_factor_threshold < 1) return GSX_EINVAL;
    if (p->behaviour_penalty_weight > 0 || invalid_number(p->behaviour_penalty_weight)) return GSX_EINVAL;
    if (p->behaviour_penalty_weight != 0 &&
        (p->behaviour_penalty_decay <= 0 || p->behaviour_penalty_decay >= 1 || invalid_number(p->behaviour_penalty_decay)))
        return GSX_EINVAL;
    if (p->behaviour_penalty_threshold < 0 || invalid_number(p->behaviour_penalty_threshold)) return GSX_EINVAL;
    if (p->decay_interval_ns < kSecond) return GSX_EINVAL;
    if (p->decay_to_zero <= 0 || p->decay_to_zero >= 1 || invalid_number(p->decay_to_zero)) return GSX_EINVAL;
    return GSX_OK;
}

// TopicScoreParams.validate, score_params.go:200-268
int gsx_validate_topic_params(const gsx_topic_score_params* p) {
    if (!p) return GSX_EINVAL;
    if (p->topic_weight < 0 || invalid_number(p->topic_weight)) return GSX_EINVAL;
    if (p->time_in_mesh_quantum_ns == 0) return GSX_EINVAL;
    if (p->time_in_mesh_weight < 0 || invalid_number(p->time_in_mesh_weight)) return GSX_EINVAL;
    if (p->time_in_mesh_weight != 0 && p->time_in_mesh_quantum_ns <= 0) return GSX_EINVAL;
    if (p->time_in_mesh_weight != 0 && (p->time_in_mesh_cap <= 0 || invalid_number(p->time_in_mesh_cap)))
        return GSX_EINVAL;
    const double w2 = p->first_message_deliveries_weight;
    if (w2 < 0 || invalid_number(w2)) return GSX_EINVAL;
    if (w2 != 0 && (p->first_message_deliveries_decay <= 0 || p->first_message_deliveries_decay >= 1 ||
                    invalid_number(p->first_message_deliveries_decay)))
        return GSX_EINVAL;
    if (w2 != 0 && (p->first_message_deliveries_cap <= 0 || invalid_number(p->first_message_deliveries_cap)))
        return GSX_EINVAL;
    const double w3 = p->mesh_message_deliveries_weight;
    if (w3 > 0 || invalid_number(w3)) return GSX_EINVAL;
    if (w3 != 0 && (p->mesh_message_deliveries_decay <= 0 || p->mesh_message_deliveries_decay >= 1 ||
                    invalid_number(p->mesh_message_deliveries_decay)))
        return GSX_EINVAL;
    if (w3 != 0 && (p->mesh_message_deliveries_cap <= 0 || invalid_number(p->mesh_message_deliveries_cap)))
        return GSX_EINVAL;
    if (w3 != 0 &&
        (p->mesh_message_deliveries_threshold <= 0 || invalid_number(p->mesh_message_deliveries_threshold)))
        return GSX_EINVAL;
    if (p->mesh_message_deliveries_window_ns < 0) return GSX_EINVAL;
    if (w3 != 0 && p->mesh_message_deliveries_activation_ns < kSecond) return GSX_EINVAL;
    const double w3b = p->mesh_failure_penalty_weight;
    if (w3b > 0 || invalid_number(w3b)) return GSX_EINVAL;
    if (w3b != 0 && (invalid_number(p->mesh_failure_penalty_decay) || p->mesh_failure_penalty_decay <= 0 ||
                     p->mesh_failure_penalty_decay >= 1))
        return GSX_EINVAL;
    const double w4 = p->invalid_message_deliveries_weight;
    if (w4 > 0 || invalid_number(w4)) return GSX_EINVAL;
    if (p->invalid_message_deliveries_decay <= 0 || p->invalid_message_deliveries_decay >= 1 ||
        invalid_number(p->invalid_message_deliveries_decay))
        return GSX_EINVAL;
    return GSX_OK;
}

// ScoreParameterDecayWithBase, score_params.go:282-287
double gsx_score_parameter_decay_with_base(int64_t decay_ns, int64_t base_ns, double decay_to_zero) {
    const double ticks = double(decay_ns / base_ns);
    return std::pow(decay_to_zero, 1 / ticks);
}

double gsx_score_parameter_decay(int64_t decay_ns) {
    return gsx_score_parameter_decay_with_base(decay_ns, kSecond, 0.01);
}

int gsx_create(const gsx_config* cfg, gsx_engine** out) {
    if (!cfg || !out) return GSX_EINVAL;
    *out = nullptr;
    if (cfg->n_topics == 0 || cfg->n_topics > GSX_MAX_TOPICS) return GSX_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg->device || cfg->device < 0) return GSX_ENODEV;
    hipDeviceProp_t prop{};
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) return GSX_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return GSX_ENODEV;  // gfx950-only code objects
    auto* e = new (std::nothrow) gsx_engine();
    if (!e) return GSX_ENOMEM;
    e->device = cfg->device;
    e->T = cfg->n_topics;
    gsx_default_gossipsub_params(&e->gp);
    if (hipSetDevice(e->device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&e->ev_start) != hipSuccess || hipEventCreate(&e->ev_stop) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_staged, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_gxf_stage, hipEventDisableTiming) != hipSuccess ||
        hipMalloc((void**)&e->d_tp, sizeof(gsx::DevTopicParams) * GSX_MAX_TOPICS) != hipSuccess) {
        gsx_destroy(e);
        return GSX_EDEVICE;
    }
    e->own_stream = e->stream;
    if (upload_topic_params(e) != GSX_OK) {
        gsx_destroy(e);
        return GSX_EDEVICE;
    }
    *out = e;
    return GSX_OK;
}

int gsx_destroy(gsx_engine* e) {
    if (!e) return GSX_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    free_state(e);
    if (e->d_tp) (void)hipFree(e->d_tp);
    if (e->d_mparts) (void)hipFree(e->d_mparts);
    if (e->d_stage) (void)hipFree(e->d_stage);
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    if (e->h_gxstage) (void)hipHostFree(e->h_gxstage);
    if (e->h_hbrb) (void)hipHostFree(e->h_hbrb);
    if (e->h_gxf_stage) (void)hipHostFree(e->h_gxf_stage);
    if (e->h_gxf_cnt) (void)hipHostFree(e->h_gxf_cnt);
    if (e->h_score) (void)hipHostFree(e->h_score);
    if (e->h_dropin) (void)hipHostFree(e->h_dropin);
    if (e->ev_start) (void)hipEventDestroy(e->ev_start);
    if (e->ev_stop) (void)hipEventDestroy(e->ev_stop);
    if (e->ev_staged) (void)hipEventDestroy(e->ev_staged);
    if (e->ev_gxf_stage) (void)hipEventDestroy(e->ev_gxf_stage);
    if (e->vc_stream) (void)hipStreamSynchronize(e->vc_stream);
    if (e->vc_go) (void)hipEventDestroy(e->vc_go);
    for (hipEvent_t ev : e->vc_done)
        if (ev) (void)hipEventDestroy(ev);
    if (e->vc_stream) (void)hipStreamDestroy(e->vc_stream);
    for (hipEvent_t ev : e->tev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : e->prop.ev) (void)hipEventDestroy(ev);
    if (e->prop.hop_flag) (void)hipHostFree(e->prop.hop_flag);
    if (!e->own_stream) e->own_stream = e->stream;  // gsx_create failed before recording it
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    delete e;
    return GSX_OK;
}

int gsx_set_stream(gsx_engine* e, void* stream) {
    if (!e) return GSX_EINVAL;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->stream = stream ? static_cast<hipStream_t>(stream) : e->own_stream;
    return GSX_OK;
}

int gsx_set_peer_params(gsx_engine* e, const gsx_peer_score_params* p) {
    if (!e || !p) return GSX_EINVAL;
    int rc = flush(e);  // queued events see the params they were issued under
    if (rc) return rc;
    e->pp = *p;
    e->pp_set = true;
    e->invalidate_scores();
    e->state_changed();
    return GSX_OK;
}

int gsx_set_thresholds(gsx_engine* e, const gsx_thresholds* t) {
    if (!e || !t) return GSX_EINVAL;
    e->th = *t;
    e->state_changed();
    return GSX_OK;
}

// SetTopicScoreParams, score.go:194-234
int gsx_set_topic_params(gsx_engine* e, uint32_t topic, const gsx_topic_score_params* p) {
    if (!e || !p) return GSX_EINVAL;
    if (topic >= e->T) return fail(e, GSX_ERANGE, "topic out of range");
    if (p->time_in_mesh_quantum_ns == 0)  // Go would panic dividing by it in score()
        return fail(e, GSX_EINVAL, "TimeInMeshQuantum must be non zero");
    if (int rc = fold_deferred(e)) return rc;
    int rc = flush(e);
    if (rc) return rc;
    const bool exist = e->scored[topic];
    const gsx_topic_score_params old = e->tp[topic];
    e->tp[topic] = *p;
    e->scored[topic] = true;
    e->invalidate_scores();
    e->state_changed();
    rc = upload_topic_params(e);
    if (rc) return rc;
    if (!exist || !e->loaded) return GSX_OK;
    const bool recap = p->first_message_deliveries_cap < old.first_message_deliveries_cap ||
                       p->mesh_message_deliveries_cap < old.mesh_message_deliveries_cap;
    if (!recap) return GSX_OK;
    HIPCHK(e, gsx::launch_recap(dev_state(e), topic, p->first_message_deliveries_cap, p->mesh_message_deliveries_cap,
                                e->stream));
    return GSX_OK;
}

namespace {
// gsx_load_overlay and gsx_load_overlay_shard: rows for nodes
// node_lo .. node_lo + n_nodes - 1 of an n_total-node overlay; col holds
// global ids, node_ips covers all n_total nodes.
// The heartbeat's per-pair / per-node state, allocated with the overlay (so
// the first round does not pay for it) or on first use.
int hb_alloc(gsx_engine* e) {
    const size_t TE = (size_t)e->T * e->E;
    int rc = 0;
    const size_t E = e->E;
    if ((rc = dalloc(e, &e->d_ctl, 2 * E)) ||
        (rc = dalloc(e, &e->d_resp, E)) || (rc = dalloc(e, &e->d_dirty, 4 * E)) ||
        (rc = dalloc(e, &e->d_long, (size_t)e->n_nodes)) || (rc = dalloc(e, &e->d_nlong, 2 * std::max<size_t>(e->T, 1))) ||
        (rc = dalloc(e, &e->d_rngk, (size_t)e->T * e->n_nodes)) || (rc = dalloc(e, &e->d_ihave_slot, TE)) ||
        (rc = dalloc(e, &e->d_ihave_unit, 2 * (size_t)e->T * std::max<size_t>(e->n_nodes, 1))) ||
        (rc = dalloc(e, &e->d_ihave_tag, std::max<size_t>(TE, 1))) ||
        (rc = dalloc(e, &e->d_work, (size_t)e->T * 64 * ((e->n_nodes + 63) / 64))) ||
        (rc = dalloc(e, &e->d_tcnt, (size_t)e->T * ((e->n_nodes + 63) / 64) + 1)) ||
        (rc = dalloc(e, &e->d_mcount, (size_t)e->T * e->n_nodes + 1)) ||
        (rc = dalloc(e, &e->d_hubwork, (size_t)e->T * e->n_nodes)) ||
        (rc = dalloc(e, &e->d_nwork, 2 * (size_t)e->T)) ||
        (rc = dalloc(e, &e->d_hubs, std::max<size_t>(e->hubs_host.size(), 1))) ||
        (rc = dalloc(e, &e->d_gelig, E)) ||
        (rc = dalloc(e, &e->d_hbstats, (size_t)gsx::HB_STAT_WORDS)))
        return rc;
    HIPCHK(e, hipMemsetAsync(e->d_ihave_slot, 0, sizeof(gsx::IhaveSlot) * (TE ? TE : 1), e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_ihave_tag, 0, std::max<size_t>(TE, 1), e->stream));
    e->ihave_round = 0;
    if (!e->hubs_host.empty())
        HIPCHK(e, hipMemcpyAsync(e->d_hubs, e->hubs_host.data(), 4 * e->hubs_host.size(), hipMemcpyHostToDevice,
                                 e->stream));
    e->gossip_prev.assign(e->T, 0);
    e->hb_clean = false;
    return GSX_OK;
}

int load_overlay(gsx_engine* e, uint32_t n_total, uint32_t node_lo, uint32_t n_nodes, const int64_t* row_ptr,
                 const int32_t* col, const uint8_t* edge_flags, const uint32_t* node_ips) {
    if (!e || !row_ptr || (!col && row_ptr[n_nodes] > 0)) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if ((uint64_t)node_lo + n_nodes > n_total) return fail(e, GSX_EINVAL, "shard range outside the overlay");
    if (row_ptr[0] != 0) return fail(e, GSX_EINVAL, "row_ptr[0] must be 0");
    for (uint32_t i = 0; i < n_nodes; ++i)
        if (row_ptr[i + 1] < row_ptr[i]) return fail(e, GSX_EINVAL, "row_ptr not monotone");
    const uint64_t E = (uint64_t)row_ptr[n_nodes];
    if (E >= gsx::HALO) return fail(e, GSX_EINVAL, "too many pairs for one engine (2^31)");
    for (uint64_t p = 0; p < E; ++p)
        if (col[p] < 0 || (uint32_t)col[p] >= n_total) return fail(e, GSX_EINVAL, "col out of range");
    // each observer tracks a peer once, rows ascending: the order first
    // deliverers are chosen in (lowest sender first)
    for (uint32_t i = 0; i < n_nodes; ++i)
        for (int64_t p = row_ptr[i] + 1; p < row_ptr[i + 1]; ++p)
            if (col[p] <= col[p - 1]) return fail(e, GSX_EINVAL, "each row of col must be strictly ascending");
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    free_state(e);
    e->loaded = false;
    pending_clear(e);
    e->recs.clear();
    e->rec_queue.clear();
    e->n_nodes = n_nodes;
    e->n_total = n_total;
    e->node_lo = node_lo;
    e->E = E;
    e->rs = (E + 63) & ~uint64_t(63);
    e->n_tiles = (E + gsx::TILE - 1) / gsx::TILE;
    e->last_refresh = 0;
    e->row_ptr.assign(row_ptr, row_ptr + n_nodes + 1);
    e->col_host.assign(col, col + E);
    e->pair_obs.resize(E);
    for (uint32_t i = 0; i < n_nodes; ++i)
        for (int64_t p = row_ptr[i]; p < row_ptr[i + 1]; ++p) e->pair_obs[(size_t)p] = i;

    // (observer, IP) groups: the keys of each observer's ps.peerIPs map
    e->ipg_host.assign(2 * E, gsx::IPG_NONE);
    e->group_ip.clear();
    uint32_t next = 0;
    std::vector<std::pair<uint32_t, uint32_t>> small;  // (ip, gid) for low-degree observers
    std::unordered_map<uint32_t, uint32_t> big;
    for (uint32_t i = 0; i < n_nodes && node_ips; ++i) {
        const int64_t deg = row_ptr[i + 1] - row_ptr[i];
        small.clear();
        big.clear();
        for (int64_t p = row_ptr[i]; p < row_ptr[i + 1]; ++p) {
            const uint32_t nb = (uint32_t)col[p];
            for (int k = 0; k < 2; ++k) {
                const uint32_t ip = node_ips[2 * (size_t)nb + k];
                if (ip == GSX_NO_IP) continue;
                uint32_t gid;
                if (deg <= 64) {
                    auto it = std::find_if(small.begin(), small.end(), [&](auto& x) { return x.first == ip; });
                    if (it == small.end()) {
                        gid = next++;
                        small.emplace_back(ip, gid);
                        e->group_ip.push_back(ip);
                    } else {
                        gid = it->second;
                    }
                } else {
                    auto it = big.find(ip);
                    if (it == big.end()) {
                        gid = next++;
                        big.emplace(ip, gid);
                        e->group_ip.push_back(ip);
                    } else {
                        gid = it->second;
                    }
                }
                e->ipg_host[2 * (size_t)p + k] = gid;
            }
        }
    }
    e->n_groups = next;

    const size_t R = (size_t)e->T * e->n_tiles * gsx::TILE;  // record slots, tail of the last tile unused
    int rc = 0;
    if ((rc = dalloc(e, &e->d_rec, R * gsx::NFIELD)) || (rc = dalloc(e, &e->d_rflags, R)) ||
        (rc = dalloc(e, &e->d_nbad, 1)) || (rc = dalloc(e, &e->d_pflags, e->rs)) ||
        (rc = dalloc(e, &e->d_eflags, e->rs)) || (rc = dalloc(e, &e->d_expire, e->rs)) ||
        (rc = dalloc(e, &e->d_bp, e->rs)) || (rc = dalloc(e, &e->d_app, e->rs)) ||
        (rc = dalloc(e, &e->d_score, e->rs)) || (rc = dalloc(e, &e->d_ipg, 2 * e->rs)) ||
        (rc = dalloc(e, &e->d_ipcount, e->n_groups)) || (rc = dalloc(e, &e->d_col, E)) ||
        (rc = dalloc(e, &e->d_backoff, (size_t)e->T * E)) ||
        (rc = dalloc(e, &e->d_bo8, (size_t)((e->T + 7) / 8) * E + 4))) {
        free_state(e);
        return rc;
    }
    HIPCHK(e, hipMemsetAsync(e->d_rec, 0, sizeof(double) * R * gsx::NFIELD, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_rflags, 0, R, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_pflags, 0, e->rs, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_expire, 0, sizeof(int64_t) * e->rs, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_bp, 0, sizeof(double) * e->rs, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_app, 0, sizeof(double) * e->rs, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_score, 0, sizeof(double) * e->rs, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_ipcount, 0, sizeof(uint32_t) * (e->n_groups ? e->n_groups : 1), e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_backoff, 0, sizeof(int64_t) * e->T * (E ? E : 1), e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_bo8, 0, (size_t)((e->T + 7) / 8) * E + 4, e->stream));
    e->max_deg = 0;
    e->hubs_host.clear();
    for (uint32_t i = 0; i < n_nodes; ++i) {
        e->max_deg = std::max<int64_t>(e->max_deg, row_ptr[i + 1] - row_ptr[i]);
        if (row_ptr[i + 1] - row_ptr[i] > gsx::HB_LANE_DEG) e->hubs_host.push_back(i);
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (E) HIPCHK(e, hipMemcpy(e->d_col, col, sizeof(int32_t) * E, hipMemcpyHostToDevice));
    {  // reverse pairs for the pull-based propagation (NO_PAIR for remote neighbours until a shard plan)
        std::vector<uint32_t>& rev = e->rev_host;
        rev.assign(E, gsx::NO_PAIR);
        for (uint32_t u = 0; u < n_nodes; ++u)
            for (int64_t q = row_ptr[u]; q < row_ptr[u + 1]; ++q) {
                const uint32_t vg = (uint32_t)col[q];
                if (vg < node_lo || vg - node_lo >= n_nodes) continue;
                const uint32_t v = vg - node_lo;
                const int32_t* b = col + row_ptr[v];
                const int32_t* en = col + row_ptr[v + 1];
                const int32_t* it = std::lower_bound(b, en, (int32_t)(u + node_lo));
                if (it != en && *it == (int32_t)(u + node_lo)) rev[(size_t)q] = (uint32_t)(it - col);
            }
        if ((rc = dalloc(e, &e->d_rev, E)) || (rc = dalloc(e, &e->d_row_ptr, (size_t)n_nodes + 1)) ||
            (rc = dalloc(e, &e->d_pair_obs, E))) {
            free_state(e);
            return rc;
        }
        if (E) HIPCHK(e, hipMemcpy(e->d_rev, rev.data(), sizeof(uint32_t) * E, hipMemcpyHostToDevice));
        if (E) HIPCHK(e, hipMemcpy(e->d_pair_obs, e->pair_obs.data(), sizeof(uint32_t) * E, hipMemcpyHostToDevice));
        HIPCHK(e, hipMemcpy(e->d_row_ptr, row_ptr, sizeof(int64_t) * ((size_t)n_nodes + 1), hipMemcpyHostToDevice));
        e->eflags_host.assign(edge_flags ? edge_flags : nullptr, edge_flags ? edge_flags + E : nullptr);
    }
    e->floodsub_peers = !edge_flags || std::any_of(edge_flags, edge_flags + E, [](uint8_t f) {
        return !(f & gsx::EDGE_GOSSIPSUB) && !(f & gsx::EDGE_DIRECT);
    });
    if (edge_flags) HIPCHK(e, hipMemcpy(e->d_eflags, edge_flags, E, hipMemcpyHostToDevice));
    else HIPCHK(e, hipMemsetAsync(e->d_eflags, 0, e->rs, e->stream));
    rc = upload_ipg(e);
    if (rc) return rc;
    if ((rc = hb_alloc(e))) return rc;
    e->loaded = true;
    e->invalidate_scores();
    e->state_changed();
    return GSX_OK;
}
}  // namespace

int gsx_load_overlay(gsx_engine* e, uint32_t n_nodes, const int64_t* row_ptr, const int32_t* col,
                     const uint8_t* edge_flags, const uint32_t* node_ips) {
    return load_overlay(e, n_nodes, 0, n_nodes, row_ptr, col, edge_flags, node_ips);
}

int gsx_load_overlay_shard(gsx_engine* e, uint32_t n_total, uint32_t node_lo, uint32_t n_local,
                           const int64_t* row_ptr, const int32_t* col, const uint8_t* edge_flags,
                           const uint32_t* node_ips) {
    return load_overlay(e, n_total, node_lo, n_local, row_ptr, col, edge_flags, node_ips);
}

// Receive side of the shard plan: every pair (u -> v) whose v lives on rank
// S != this one gets a receive slot; slots run rank by rank, pairs ascending.
int gsx_shard_recv_plan(gsx_engine* e, uint32_t n_ranks, const uint32_t* rank_lo, uint64_t* recv_counts,
                        uint32_t* recv_u, uint32_t* recv_v) {
    if (!e || !rank_lo || !recv_counts || n_ranks == 0) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (rank_lo[0] != 0 || rank_lo[n_ranks] != e->n_total) return fail(e, GSX_EINVAL, "rank ranges must cover the overlay");
    bool mine = false;
    for (uint32_t k = 0; k < n_ranks; ++k) {
        if (rank_lo[k + 1] < rank_lo[k]) return fail(e, GSX_EINVAL, "rank ranges not monotone");
        if (rank_lo[k] == e->node_lo && rank_lo[k + 1] - rank_lo[k] == e->n_nodes) mine = true;
    }
    if (!mine) return fail(e, GSX_EINVAL, "no rank owns exactly this engine's nodes");
    auto owner = [&](uint32_t v) {
        return (uint32_t)(std::upper_bound(rank_lo, rank_lo + n_ranks + 1, v) - rank_lo) - 1;
    };
    const uint32_t self_lo = e->node_lo, self_n = e->n_nodes;
    std::vector<uint64_t> cnt(n_ranks, 0);
    std::vector<uint32_t> own(e->E, 0);
    for (uint64_t q = 0; q < e->E; ++q) {
        const uint32_t v = (uint32_t)e->col_host[q];
        if (v >= self_lo && v - self_lo < self_n) continue;
        own[q] = owner(v);
        ++cnt[own[q]];
    }
    std::vector<uint64_t> base(n_ranks + 1, 0);
    for (uint32_t k = 0; k < n_ranks; ++k) base[k + 1] = base[k] + cnt[k];
    if (base[n_ranks] > gsx::HALO_SLOT) return fail(e, GSX_ERANGE, "too many cross-shard pairs (2^30 receive slots)");
    std::vector<uint64_t> fill(base.begin(), base.end() - 1);
    std::vector<uint32_t> hnode(base[n_ranks]), hpair(base[n_ranks]);
    for (uint64_t q = 0; q < e->E; ++q) {
        const uint32_t v = (uint32_t)e->col_host[q];
        if (v >= self_lo && v - self_lo < self_n) continue;
        const uint64_t slot = fill[own[q]]++;
        e->rev_host[q] = gsx::HALO | (uint32_t)slot;
        hnode[slot] = e->pair_obs[q];
        hpair[slot] = (uint32_t)q;
        if (recv_u) recv_u[slot] = e->pair_obs[q] + self_lo;
        if (recv_v) recv_v[slot] = v;
    }
    for (uint32_t k = 0; k < n_ranks; ++k) recv_counts[k] = cnt[k];
    e->n_ranks = n_ranks;
    e->rank_lo.assign(rank_lo, rank_lo + n_ranks + 1);
    e->recv_counts = cnt;
    e->n_recv = base[n_ranks];
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->E) HIPCHK(e, hipMemcpy(e->d_rev, e->rev_host.data(), sizeof(uint32_t) * e->E, hipMemcpyHostToDevice));
    if (e->d_halo_node) (void)hipFree(e->d_halo_node);
    e->d_halo_node = nullptr;
    if (int rc = dalloc(e, &e->d_halo_node, hnode.size())) return rc;
    if (!hnode.empty())
        HIPCHK(e, hipMemcpy(e->d_halo_node, hnode.data(), sizeof(uint32_t) * hnode.size(), hipMemcpyHostToDevice));
    if (e->d_halo_pair) (void)hipFree(e->d_halo_pair);
    e->d_halo_pair = nullptr;
    if (int rc = dalloc(e, &e->d_halo_pair, hpair.size())) return rc;
    if (!hpair.empty())
        HIPCHK(e, hipMemcpy(e->d_halo_pair, hpair.data(), sizeof(uint32_t) * hpair.size(), hipMemcpyHostToDevice));
    {  // (remote sender, local receiver) by sender: the replicated frontier's receiver marks
        std::vector<uint64_t> key(hpair.size());
        for (size_t k = 0; k < hpair.size(); ++k) key[k] = ((uint64_t)e->col_host[hpair[k]] << 32) | hnode[k];
        std::sort(key.begin(), key.end());
        std::vector<uint32_t> mv(key.size()), mu(key.size());
        for (size_t k = 0; k < key.size(); ++k) {
            mv[k] = (uint32_t)(key[k] >> 32);
            mu[k] = (uint32_t)key[k];
        }
        for (uint32_t** p : {&e->d_rmark_v, &e->d_rmark_u}) {
            if (*p) (void)hipFree(*p);
            *p = nullptr;
        }
        if (int rc = dalloc(e, &e->d_rmark_v, mv.size())) return rc;
        if (int rc = dalloc(e, &e->d_rmark_u, mu.size())) return rc;
        if (!mv.empty()) {
            HIPCHK(e, hipMemcpy(e->d_rmark_v, mv.data(), 4 * mv.size(), hipMemcpyHostToDevice));
            HIPCHK(e, hipMemcpy(e->d_rmark_u, mu.data(), 4 * mu.size(), hipMemcpyHostToDevice));
        }
    }
    return GSX_OK;
}

// Send side: the concatenated (per rank, in rank order) receive lists of the
// other ranks; entry (u, v) asks this rank what its node v sends to u.
int gsx_shard_send_plan(gsx_engine* e, const uint64_t* send_counts, const uint32_t* req_u, const uint32_t* req_v) {
    if (!e || !send_counts) return GSX_EINVAL;
    if (!e->loaded || e->rank_lo.empty()) return fail(e, GSX_ESTATE, "gsx_shard_recv_plan first");
    uint64_t n = 0;
    for (uint32_t k = 0; k < e->n_ranks; ++k) n += send_counts[k];
    if (n && (!req_u || !req_v)) return GSX_EINVAL;
    std::vector<uint32_t> sp(n, gsx::NO_PAIR);
    for (uint64_t j = 0; j < n; ++j) {
        const uint32_t u = req_u[j], v = req_v[j];
        if (v < e->node_lo || v - e->node_lo >= e->n_nodes) return fail(e, GSX_EINVAL, "request for a node this rank does not own");
        const uint32_t lv = v - e->node_lo;
        const int32_t* b = e->col_host.data() + e->row_ptr[lv];
        const int32_t* en = e->col_host.data() + e->row_ptr[lv + 1];
        const int32_t* it = std::lower_bound(b, en, (int32_t)u);
        if (it != en && *it == (int32_t)u) sp[j] = (uint32_t)(it - e->col_host.data());
    }
    std::vector<uint8_t> dest(n);
    std::vector<uint64_t> base(e->n_ranks + 1, 0);
    for (uint32_t k = 0; k < e->n_ranks; ++k) {
        base[k + 1] = base[k] + send_counts[k];
        std::fill(dest.begin() + base[k], dest.begin() + base[k + 1], (uint8_t)k);
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    void* old[] = {e->d_send_pair, e->d_send_dest, e->d_send_base};
    for (void* p : old)
        if (p) (void)hipFree(p);
    e->d_send_pair = nullptr;
    e->d_send_dest = nullptr;
    e->d_send_base = nullptr;
    int rc = 0;
    if ((rc = dalloc(e, &e->d_send_pair, n)) || (rc = dalloc(e, &e->d_send_dest, n)) ||
        (rc = dalloc(e, &e->d_send_base, (size_t)e->n_ranks + 1)))
        return rc;
    if (n) HIPCHK(e, hipMemcpy(e->d_send_pair, sp.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice));
    if (n) HIPCHK(e, hipMemcpy(e->d_send_dest, dest.data(), n, hipMemcpyHostToDevice));
    {  // pair -> its send slot (a pair is asked for by at most one destination: its peer's owner)
        std::vector<uint32_t> slot_of(std::max<size_t>(e->E, 1), gsx::NO_PAIR);
        for (uint64_t j = 0; j < n; ++j)
            if (sp[j] != gsx::NO_PAIR) slot_of[sp[j]] = (uint32_t)j;
        if (e->d_send_slot) (void)hipFree(e->d_send_slot);
        e->d_send_slot = nullptr;
        if ((rc = dalloc(e, &e->d_send_slot, slot_of.size()))) return rc;
        HIPCHK(e, hipMemcpy(e->d_send_slot, slot_of.data(), sizeof(uint32_t) * slot_of.size(), hipMemcpyHostToDevice));
    }
    HIPCHK(e, hipMemcpy(e->d_send_base, base.data(), 8 * base.size(), hipMemcpyHostToDevice));
    e->send_counts.assign(send_counts, send_counts + e->n_ranks);
    e->n_send = n;
    return GSX_OK;
}

// For the compacted exchange: where each destination's rows start in ITS
// halo (the receive slot of the first row this rank sends it).
int gsx_shard_set_halo_bases(gsx_engine* e, const uint64_t* dest_halo_base) {
    if (!e || !dest_halo_base) return GSX_EINVAL;
    if (e->rank_lo.empty()) return fail(e, GSX_ESTATE, "gsx_shard_recv_plan first");
    if (e->n_ranks > gsx::MAX_RANKS) return fail(e, GSX_ERANGE, "too many ranks for the compacted exchange");
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->d_dest_halo_base) (void)hipFree(e->d_dest_halo_base);
    e->d_dest_halo_base = nullptr;
    if (int rc = dalloc(e, &e->d_dest_halo_base, e->n_ranks)) return rc;
    HIPCHK(e, hipMemcpy(e->d_dest_halo_base, dest_halo_base, 8 * (size_t)e->n_ranks, hipMemcpyHostToDevice));
    return GSX_OK;
}

int gsx_num_pairs(gsx_engine* e, uint64_t* out) {
    if (!e || !out) return GSX_EINVAL;
    *out = e->E;
    return GSX_OK;
}

int gsx_set_ip_whitelist(gsx_engine* e, const uint32_t* ip_ids, size_t n) {
    if (!e || (n && !ip_ids)) return GSX_EINVAL;
    int rc = flush(e);
    if (rc) return rc;
    e->ip_wl.clear();
    for (size_t i = 0; i < n; ++i) {
        if (ip_ids[i] == GSX_NO_IP) continue;
        if (ip_ids[i] >= e->ip_wl.size()) e->ip_wl.resize((size_t)ip_ids[i] + 1, 0);
        e->ip_wl[ip_ids[i]] = 1;
    }
    e->invalidate_scores();
    e->state_changed();
    if (!e->loaded) return GSX_OK;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return upload_ipg(e);
}

int gsx_set_app_scores(gsx_engine* e, const double* app, size_t n) {
    if (!e || !app) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (n != e->E) return fail(e, GSX_EINVAL, "app score count != pairs");
    int rc = flush(e);  // a queued RemovePeer must see the app score it was issued under
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(e->d_app, app, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->invalidate_scores();
    e->state_changed();
    return GSX_OK;
}

// setIPs for pairs whose peer's IP list changed (refreshIPs, score.go:560-586)
int gsx_set_pair_ips(gsx_engine* e, const uint64_t* pairs, const uint32_t* ips, size_t n) {
    if (!e || (n && (!pairs || !ips))) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    for (size_t i = 0; i < n; ++i)
        if (pairs[i] >= e->E) return fail(e, GSX_ERANGE, "pair out of range");
    if (n == 0) return GSX_OK;
    if (int rc = flush(e)) return rc;  // queued events count under the lists they were issued with
    // the (observer, IP) group of each new IP: an existing key of the
    // observer's ps.peerIPs map, or a new one
    const uint32_t groups0 = e->n_groups;
    auto group_of = [&](uint32_t u, uint32_t ip) -> uint32_t {
        if (ip == GSX_NO_IP) return gsx::IPG_NONE;
        for (int64_t q = e->row_ptr[u]; q < e->row_ptr[u + 1]; ++q)
            for (int k = 0; k < 2; ++k) {
                const uint32_t g = e->ipg_host[2 * (size_t)q + k];
                if (g != gsx::IPG_NONE && e->group_ip[g] == ip) return g;
            }
        e->group_ip.push_back(ip);
        return e->n_groups++;
    };
    std::vector<uint32_t> obs(n), order(n);
    std::vector<gsx::DevIpMove> mv(n);
    for (size_t i = 0; i < n; ++i) {
        const uint64_t p = pairs[i];
        const uint32_t u = e->pair_obs[p];
        obs[i] = u;
        order[i] = (uint32_t)i;
        uint32_t g[2];
        for (int k = 0; k < 2; ++k) {
            g[k] = group_of(u, ips[2 * i + k]);
            e->ipg_host[2 * (size_t)p + k] = g[k];
            if (g[k] != gsx::IPG_NONE && ips[2 * i + k] < e->ip_wl.size() && e->ip_wl[ips[2 * i + k]]) g[k] |= gsx::IPG_WL;
        }
        mv[i] = gsx::DevIpMove{p, g[0], g[1]};
    }
    if (e->n_groups > groups0) {  // new keys: a longer count array, the old counts kept
        uint32_t* nc = nullptr;
        if (int rc = dalloc(e, &nc, e->n_groups)) return rc;
        HIPCHK(e, hipMemsetAsync(nc, 0, sizeof(uint32_t) * e->n_groups, e->stream));
        if (groups0) HIPCHK(e, hipMemcpyAsync(nc, e->d_ipcount, sizeof(uint32_t) * groups0, hipMemcpyDeviceToDevice, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        (void)hipFree(e->d_ipcount);
        e->d_ipcount = nc;
    }
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return obs[a] < obs[b]; });
    std::vector<gsx::DevIpMove> sorted(n);
    std::vector<uint32_t> off;
    for (size_t i = 0; i < n; ++i) {
        sorted[i] = mv[order[i]];
        if (i == 0 || obs[order[i]] != obs[order[i - 1]]) off.push_back((uint32_t)i);
    }
    const uint32_t n_grp = (uint32_t)off.size();
    off.push_back((uint32_t)n);
    gsx::DevIpMove* d_mv = nullptr;
    uint32_t* d_off = nullptr;
    if (int rc = dalloc(e, &d_mv, n)) return rc;
    if (int rc = dalloc(e, &d_off, off.size())) {
        (void)hipFree(d_mv);
        return rc;
    }
    HIPCHK(e, hipMemcpyAsync(d_mv, sorted.data(), sizeof(gsx::DevIpMove) * n, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(d_off, off.data(), sizeof(uint32_t) * off.size(), hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, gsx::launch_set_ips(dev_state(e), d_mv, d_off, n_grp, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    (void)hipFree(d_mv);
    (void)hipFree(d_off);
    if (e->scores_valid || e->dirty_only || e->lazy) {  // only these observers' P6 moved
        for (uint32_t g = 0; g < n_grp; ++g) e->dirty_obs.push_back(obs[order[off[g]]]);
        e->scores_valid = false;
        e->dirty_only = true;
    }
    e->state_changed();
    return GSX_OK;
}

int gsx_apply_events(gsx_engine* e, const gsx_event* ev, size_t n) {
    if (!e || (n && !ev)) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    for (size_t i = 0; i < n; ++i) {
        if (ev[i].pair >= e->E) return fail(e, GSX_ERANGE, "event pair out of range");
        if (ev[i].kind < GSX_EV_ADD_PEER || ev[i].kind > GSX_EV_APP_SCORE) return fail(e, GSX_EINVAL, "bad event kind");
    }
    e->pending.insert(e->pending.end(), ev, ev + n);
    for (size_t i = 0; i < n; ++i) pending_note(e, ev[i].kind, ev[i].pair);
    return GSX_OK;
}

int gsx_flush(gsx_engine* e) {
    if (!e) return GSX_EINVAL;
    return flush(e);
}

// ValidateMessage, score.go:686-693
int gsx_trace_validate(gsx_engine* e, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now) {
    (void)topic;
    if (!e) return GSX_EINVAL;
    if (int rc = check_pair(e, pair)) return rc;
    (void)get_record(e, e->pair_obs[pair], msg_id, now);
    return GSX_OK;
}

// DeliverMessage, score.go:695-719
int gsx_trace_deliver(gsx_engine* e, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now) {
    if (!e) return GSX_EINVAL;
    if (int rc = check_pair(e, pair)) return rc;
    push_event(e, GSX_EV_FIRST_DELIVERY, pair, topic, now, 0);
    DeliveryRecord& r = get_record(e, e->pair_obs[pair], msg_id, now);
    if (r.status != kDeliveryUnknown) return GSX_OK;
    r.status = kDeliveryValid;
    r.validated = now;
    r.validated_set = true;
    for (uint64_t q : r.peers)
        if (q != pair) mark_duplicate(e, q, topic, false, 0, now);
    return GSX_OK;
}

// RejectMessage, score.go:721-786
int gsx_trace_reject(gsx_engine* e, uint64_t pair, uint64_t msg_id, uint32_t topic, int32_t reason, int64_t now) {
    if (!e) return GSX_EINVAL;
    if (int rc = check_pair(e, pair)) return rc;
    switch (reason) {
    case GSX_REJECT_MISSING_SIGNATURE:
    case GSX_REJECT_INVALID_SIGNATURE:
    case GSX_REJECT_UNEXPECTED_SIGNATURE:
    case GSX_REJECT_UNEXPECTED_AUTH_INFO:
    case GSX_REJECT_SELF_ORIGIN: push_event(e, GSX_EV_INVALID_DELIVERY, pair, topic, now, 0); return GSX_OK;
    case GSX_REJECT_BLACKLISTED_PEER:
    case GSX_REJECT_BLACKLISTED_SOURCE:
    case GSX_REJECT_VALIDATION_QUEUE_FULL: return GSX_OK;
    case GSX_REJECT_VALIDATION_THROTTLED:
    case GSX_REJECT_VALIDATION_IGNORED:
    case GSX_REJECT_VALIDATION_FAILED: break;
    default: return fail(e, GSX_EINVAL, "unknown reject reason");
    }
    DeliveryRecord& r = get_record(e, e->pair_obs[pair], msg_id, now);
    if (r.status != kDeliveryUnknown) return GSX_OK;
    if (reason == GSX_REJECT_VALIDATION_THROTTLED || reason == GSX_REJECT_VALIDATION_IGNORED) {
        r.status = reason == GSX_REJECT_VALIDATION_THROTTLED ? kDeliveryThrottled : kDeliveryIgnored;
        r.peers.clear();
        r.peers.shrink_to_fit();
        r.peers_nil = true;
        return GSX_OK;
    }
    r.status = kDeliveryInvalid;
    push_event(e, GSX_EV_INVALID_DELIVERY, pair, topic, now, 0);
    for (uint64_t q : r.peers) push_event(e, GSX_EV_INVALID_DELIVERY, q, topic, now, 0);
    r.peers.clear();
    r.peers.shrink_to_fit();
    r.peers_nil = true;
    return GSX_OK;
}

// DuplicateMessage, score.go:788-820
int gsx_trace_duplicate(gsx_engine* e, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now) {
    if (!e) return GSX_EINVAL;
    if (int rc = check_pair(e, pair)) return rc;
    DeliveryRecord& r = get_record(e, e->pair_obs[pair], msg_id, now);
    if (!r.peers_nil && has_peer(r, pair)) return GSX_OK;
    switch (r.status) {
    case kDeliveryUnknown: r.peers.push_back(pair); break;
    case kDeliveryValid:
        r.peers.push_back(pair);
        mark_duplicate(e, pair, topic, r.validated_set, r.validated, now);
        break;
    case kDeliveryInvalid: push_event(e, GSX_EV_INVALID_DELIVERY, pair, topic, now, 0); break;
    default: break;
    }
    return GSX_OK;
}

// messageDeliveries.gc, score.go:856-870
int gsx_gc_deliveries(gsx_engine* e, int64_t now) {
    if (!e) return GSX_EINVAL;
    for (auto it = e->rec_queue.begin(); it != e->rec_queue.end();) {
        auto& q = it->second;
        while (!q.empty() && now > q.front().second) {
            e->recs.erase(RecKey{it->first, q.front().first});
            q.pop_front();
        }
        it = q.empty() ? e->rec_queue.erase(it) : std::next(it);
    }
    return GSX_OK;
}

int gsx_num_delivery_records(gsx_engine* e, uint64_t* out) {
    if (!e || !out) return GSX_EINVAL;
    *out = e->recs.size();
    return GSX_OK;
}

// refreshScores, score.go:497-558, fused with score() for every pair
int gsx_refresh(gsx_engine* e, int64_t now) {
    if (!e) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (int rc = fold_deferred(e)) return rc;  // (the decay follows the credits)
    int rc = flush(e);
    if (rc) return rc;
    const gsx::DevState s = dev_state(e);
    HIPCHK(e, gsx::launch_purge(s, now, e->stream));
    const bool region = e->t_active && e->t_used < e->t_max;
    HIPCHK(e, hipEventRecord(region ? e->tev[2 * e->t_used] : e->ev_start, e->stream));
    HIPCHK(e, rescore_all(e, s, now, true));
    HIPCHK(e, hipEventRecord(region ? e->tev[2 * e->t_used + 1] : e->ev_stop, e->stream));
    if (region) ++e->t_used;
    e->timed = !region;
    e->scores_exact();
    e->state_changed();
    e->last_refresh = now;
    return GSX_OK;
}

int gsx_last_refresh_ms(gsx_engine* e, float* ms) {
    if (!e || !ms) return GSX_EINVAL;
    if (!e->timed) return fail(e, GSX_ESTATE, "no refresh timed yet");
    HIPCHK(e, hipEventSynchronize(e->ev_stop));
    HIPCHK(e, hipEventElapsedTime(ms, e->ev_start, e->ev_stop));
    return GSX_OK;
}

int gsx_timing_begin(gsx_engine* e, uint32_t max_launches) {
    if (!e || max_launches == 0) return GSX_EINVAL;
    while (e->tev.size() < 2 * (size_t)max_launches) {
        hipEvent_t ev;
        HIPCHK(e, hipEventCreate(&ev));
        e->tev.push_back(ev);
    }
    e->t_max = max_launches;
    e->t_used = 0;
    e->t_active = true;
    return GSX_OK;
}

int gsx_timing_end(gsx_engine* e, double* total_ms, double* min_ms, double* max_ms, uint32_t* n) {
    if (!e || !total_ms || !n) return GSX_EINVAL;
    if (!e->t_active) return fail(e, GSX_ESTATE, "gsx_timing_begin not called");
    e->t_active = false;
    double sum = 0, lo = 0, hi = 0;
    for (uint32_t i = 0; i < e->t_used; ++i) {
        HIPCHK(e, hipEventSynchronize(e->tev[2 * i + 1]));
        float ms = 0;
        HIPCHK(e, hipEventElapsedTime(&ms, e->tev[2 * i], e->tev[2 * i + 1]));
        sum += ms;
        lo = i == 0 ? ms : std::min(lo, (double)ms);
        hi = i == 0 ? ms : std::max(hi, (double)ms);
    }
    *total_ms = sum;
    *n = e->t_used;
    if (min_ms) *min_ms = lo;
    if (max_ms) *max_ms = hi;
    return GSX_OK;
}

int gsx_scores(gsx_engine* e, double* out, size_t n) {
    if (!e || (n && !out)) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (n != e->E) return fail(e, GSX_EINVAL, "score buffer size != pairs");
    if (int rc = ensure_scores(e)) return rc;
    HIPCHK(e, hipMemcpyAsync(out, e->d_score, sizeof(double) * n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

// The drop-in round trip in one launch (k_dropin): the queued tracer events
// of a small engine whose host score copy was current are applied and the
// scores they change re-scored into both copies — the event pairs, and the
// rows of observers with an AddPeer / RemovePeer (their IP groups' P6) — so
// the cost follows the events, not the router's peer count; the host polls a
// mapped flag.  Returns 1 when it ran, 0 when the case does not apply (the
// general path follows), < 0 on error.
constexpr size_t kDropinMaxEvents = 4096, kDropinMaxObs = 64;
int dropin_fast(gsx_engine* e) {
    if (e->pending.empty() || e->E > kHostScoreMax || !e->h_score_dev || e->h_score_cap < e->E ||
        e->h_score_tag != e->score_writes || !e->scores_valid || e->dirty_only || e->pending.size() > kDropinMaxEvents)
        return 0;
    const size_t n = e->pending.size();
    std::vector<uint32_t> obs(n);
    for (size_t i = 0; i < n; ++i) {
        if (e->pending[i].pair >= e->E) {
            pending_clear(e);
            return fail(e, GSX_ERANGE, "event pair out of range");
        }
        obs[i] = e->pair_obs[e->pending[i].pair];
    }
    std::vector<uint32_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return obs[a] < obs[b]; });
    std::vector<uint32_t> goff, gobs, rows;
    std::vector<uint64_t> prs;
    for (size_t i = 0; i < n; ++i)
        if (i == 0 || obs[order[i]] != obs[order[i - 1]]) {
            goff.push_back((uint32_t)i);
            gobs.push_back(obs[order[i]]);
        }
    if (gobs.size() > kDropinMaxObs) return 0;
    goff.push_back((uint32_t)n);
    for (size_t g = 0; g + 1 < goff.size(); ++g) {  // per observer: its whole row, or the event pairs
        bool row = false;
        for (uint32_t i = goff[g]; i < goff[g + 1] && !row; ++i) {
            const uint32_t k = e->pending[order[i]].kind;
            row = k == GSX_EV_ADD_PEER || k == GSX_EV_REMOVE_PEER;
        }
        if (row) {
            rows.push_back(gobs[g]);
            continue;
        }
        const size_t p0 = prs.size();
        for (uint32_t i = goff[g]; i < goff[g + 1]; ++i) prs.push_back(e->pending[order[i]].pair);
        std::sort(prs.begin() + (long)p0, prs.end());
        prs.erase(std::unique(prs.begin() + (long)p0, prs.end()), prs.end());
    }
    const size_t ev_off = 64, ev_b = sizeof(gsx::DevEvent) * n;
    const size_t go_off = ev_off + ev_b, go_b = 4 * goff.size();
    const size_t ob_off = go_off + go_b, ob_b = 4 * std::max<size_t>(rows.size(), 1);
    const size_t pr_off = (ob_off + ob_b + 7) & ~(size_t)7, pr_b = 8 * std::max<size_t>(prs.size(), 1);
    const size_t need = pr_off + pr_b;
    if (e->h_dropin_bytes < need) {
        if (e->h_dropin) (void)hipHostFree(e->h_dropin);
        e->h_dropin = nullptr;
        e->h_dropin_bytes = 0;
        const size_t want =
            std::max<size_t>(need, 128 + (sizeof(gsx::DevEvent) + 16) * kDropinMaxEvents + 8 * kDropinMaxObs);
        HIPCHK(e, hipHostMalloc(&e->h_dropin, want, hipHostMallocMapped | hipHostMallocCoherent));
        void* dp = nullptr;
        HIPCHK(e, hipHostGetDevicePointer(&dp, e->h_dropin, 0));
        e->d_dropin = static_cast<char*>(dp);
        e->h_dropin_bytes = want;
        *static_cast<volatile uint32_t*>(e->h_dropin) = e->dropin_tag;
    }
    char* hb = static_cast<char*>(e->h_dropin);
    auto* hev = reinterpret_cast<gsx::DevEvent*>(hb + ev_off);
    for (size_t i = 0; i < n; ++i) {
        const gsx_event& x = e->pending[order[i]];
        hev[i] = gsx::DevEvent{x.kind, x.topic, x.pair, x.now_ns, x.arg};
    }
    std::memcpy(hb + go_off, goff.data(), go_b);
    if (!rows.empty()) std::memcpy(hb + ob_off, rows.data(), 4 * rows.size());
    if (!prs.empty()) std::memcpy(hb + pr_off, prs.data(), 8 * prs.size());
    std::atomic_thread_fence(std::memory_order_release);
    const uint32_t tag = ++e->dropin_tag;
    HIPCHK(e, gsx::launch_dropin(dev_state(e), dev_peer_params(e), reinterpret_cast<const gsx::DevEvent*>(e->d_dropin + ev_off),
                                 reinterpret_cast<const uint32_t*>(e->d_dropin + go_off), (uint32_t)gobs.size(),
                                 reinterpret_cast<const uint32_t*>(e->d_dropin + ob_off), (uint32_t)rows.size(),
                                 reinterpret_cast<const uint64_t*>(e->d_dropin + pr_off), (uint32_t)prs.size(),
                                 e->d_row_ptr, e->h_score_dev, reinterpret_cast<uint32_t*>(e->d_dropin), tag, e->stream));
    pending_clear(e);
    const volatile uint32_t* flag = static_cast<const volatile uint32_t*>(e->h_dropin);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0; *flag != tag; ++spin) {
        if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
            HIPCHK(e, hipStreamSynchronize(e->stream));  // (a busy device: wait for the stream instead)
            if (*flag != tag) return fail(e, GSX_EDEVICE, "drop-in round trip: the kernel did not signal");
            break;
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    e->state_changed();
    ++e->score_writes;
    e->scores_exact();
    e->h_score_tag = e->score_writes;
    return 1;
}

// The host copy equals the device scores as the queued events found them.
bool host_copy_current(const gsx_engine* e) {
    return e->h_score && e->h_score_cap >= e->E && e->scores_valid && !e->dirty_only &&
           e->h_score_tag == e->score_writes;
}

// The host copy of every score (engines up to kHostScoreMax pairs), current.
int host_scores(gsx_engine* e) {
    if (e->pending.empty() && e->scores_valid && e->h_score_tag == e->score_writes) return GSX_OK;
    if (int r = dropin_fast(e)) return r < 0 ? r : GSX_OK;
    if (int rc = ensure_scores(e)) return rc;
    if (e->h_score_cap < e->E) {
        if (e->h_score) (void)hipHostFree(e->h_score);
        e->h_score = e->h_score_dev = nullptr;
        e->h_score_cap = 0;
        HIPCHK(e, hipHostMalloc((void**)&e->h_score, sizeof(double) * std::max<size_t>(e->E, 1),
                                hipHostMallocMapped | hipHostMallocCoherent));
        void* dp = nullptr;
        HIPCHK(e, hipHostGetDevicePointer(&dp, e->h_score, 0));
        e->h_score_dev = static_cast<double*>(dp);
        e->h_score_cap = e->E;
    }
    HIPCHK(e, hipMemcpyAsync(e->h_score, e->d_score, sizeof(double) * e->E, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->h_score_tag = e->score_writes;
    return GSX_OK;
}

// Score(p), score.go:247-256
int gsx_score(gsx_engine* e, uint64_t pair, double* out) {
    if (!e || !out) return GSX_EINVAL;
    if (int rc = check_pair(e, pair)) return rc;
    if (e->E <= kHostScoreMax) {  // small engine (one router's peers): keep the whole vector on the host
        // the host copy was current before the queued events, which leave this
        // pair's score alone: no round trip (the events stay queued)
        if (host_copy_current(e) && !pending_touches(e, pair)) {
            *out = e->h_score[pair];
            return GSX_OK;
        }
        if (int rc = host_scores(e)) return rc;
        *out = e->h_score[pair];
        return GSX_OK;
    }
    if (int rc = ensure_scores(e)) return rc;
    HIPCHK(e, hipMemcpyAsync(out, e->d_score + pair, sizeof(double), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

// Score(p) of many pairs: one flush, one re-score, one copy (gsx.h)
int gsx_score_many(gsx_engine* e, const uint64_t* pairs, size_t n, double* out) {
    if (!e || (n && (!pairs || !out))) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    for (size_t i = 0; i < n; ++i)
        if (pairs[i] >= e->E) return fail(e, GSX_ERANGE, "pair out of range");
    if (e->E <= kHostScoreMax) {
        bool touched = !host_copy_current(e);
        for (size_t i = 0; i < n && !touched; ++i) touched = pending_touches(e, pairs[i]);
        if (touched)
            if (int rc = host_scores(e)) return rc;
        for (size_t i = 0; i < n; ++i) out[i] = e->h_score[pairs[i]];
        return GSX_OK;
    }
    if (int rc = ensure_scores(e)) return rc;
    if (n == 0) return GSX_OK;
    uint64_t* dp = nullptr;
    double* dout = nullptr;
    if (int rc = dalloc(e, &dp, n)) return rc;
    if (int rc = dalloc(e, &dout, n)) {
        (void)hipFree(dp);
        return rc;
    }
    hipError_t st = hipMemcpyAsync(dp, pairs, 8 * n, hipMemcpyHostToDevice, e->stream);
    if (st == hipSuccess) st = gsx::launch_gather_scores(e->d_score, dp, n, dout, e->stream);
    if (st == hipSuccess) st = hipMemcpyAsync(out, dout, 8 * n, hipMemcpyDeviceToHost, e->stream);
    if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    (void)hipFree(dp);
    (void)hipFree(dout);
    if (st != hipSuccess) return fail(e, GSX_EDEVICE, std::string("gsx_score_many: ") + hipGetErrorString(st));
    return GSX_OK;
}

int gsx_device_scores(gsx_engine* e, const double** dptr) {
    if (!e || !dptr) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (int rc = ensure_scores(e)) return rc;
    *dptr = e->d_score;
    return GSX_OK;
}

int gsx_settle_scores(gsx_engine* e) {
    if (!e) return GSX_EINVAL;
    if (!e->loaded) return GSX_OK;
    return ensure_scores(e);
}

int gsx_sync(gsx_engine* e) {
    if (!e) return GSX_EINVAL;
    if (int rc = flush(e)) return rc;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_import_state(gsx_engine* e, const gsx_state_view* s) {
    if (!e || !s) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (!s->first_message_deliveries || !s->mesh_message_deliveries || !s->mesh_failure_penalty ||
        !s->invalid_message_deliveries || !s->graft_time_ns || !s->mesh_time_ns || !s->rec_flags ||
        !s->pair_flags || !s->expire_ns || !s->behaviour_penalty)
        return fail(e, GSX_EINVAL, "import needs every state array");
    if (int rc = flush(e)) return rc;
    if (int rc = drop_deferred(e)) return rc;
    const size_t E = e->E, R = (size_t)e->T * E;
    if (int rc = ensure_tmp(e)) return rc;
    e->last_refresh = s->last_refresh_ns;
    const gsx::DevState ds = dev_state(e);
    const void* fields[gsx::NFIELD] = {s->first_message_deliveries, s->mesh_message_deliveries,
                                       s->mesh_failure_penalty, s->invalid_message_deliveries, s->graft_time_ns};
    for (int f = 0; f < gsx::NFIELD; ++f) {
        HIPCHK(e, hipMemcpyAsync(e->d_tmp, fields[f], 8 * R, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, gsx::launch_tile_field(ds, f, e->d_tmp, e->stream));
    }
    HIPCHK(e, hipMemcpyAsync(e->d_tmp, s->rec_flags, R, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, gsx::launch_tile_field(ds, gsx::NFIELD, e->d_tmp, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_nbad, 0, sizeof(uint32_t), e->stream));
    HIPCHK(e, hipMemcpyAsync(e->d_tmp, s->mesh_time_ns, 8 * R, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, gsx::launch_mesh_time_import(ds, static_cast<const int64_t*>(e->d_tmp), e->d_nbad, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->d_pflags, s->pair_flags, E, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->d_expire, s->expire_ns, 8 * E, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->d_bp, s->behaviour_penalty, 8 * E, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, gsx::launch_rebuild_ipcount(ds, e->n_groups, e->stream));
    uint32_t n_bad = 0;
    HIPCHK(e, hipMemcpyAsync(&n_bad, e->d_nbad, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    release_tmp(e);
    e->invalidate_scores();
    e->state_changed();
    if (n_bad) return fail(e, GSX_EINVAL, std::to_string(n_bad) + " in-mesh records have a meshTime that is neither 0 "
                                          "nor last_refresh_ns - graftTime");
    return GSX_OK;
}

int gsx_synthesize_state(gsx_engine* e, const gsx_synth_spec* sp) {
    if (!e || !sp) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (int rc = flush(e)) return rc;
    if (int rc = drop_deferred(e)) return rc;
    gsx::DevSynthSpec d{};
    d.seed = sp->seed;
    d.now = sp->now_ns;
    d.fmd_max = sp->fmd_max;
    d.mmd_max = sp->mmd_max;
    d.mfp_max = sp->mfp_max;
    d.imd_max = sp->imd_max_sybil;
    d.p_in_mesh = sp->p_in_mesh;
    d.graft_window = sp->graft_window_ns;
    d.bp_max = sp->bp_max;
    d.p_disc = sp->p_disconnected;
    d.p_abs = sp->p_absent;
    d.expire_jitter = sp->expire_jitter_ns;
    d.sybil_first = sp->sybil_first_node;
    e->last_refresh = sp->now_ns;  // meshTime = now - graftTime for every in-mesh record
    const gsx::DevState s = dev_state(e);
    HIPCHK(e, gsx::launch_synthesize(s, e->d_col, d, e->stream));
    HIPCHK(e, gsx::launch_rebuild_ipcount(s, e->n_groups, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->invalidate_scores();
    e->state_changed();
    return GSX_OK;
}

int gsx_export_state(gsx_engine* e, gsx_state_view* s) {
    if (!e || !s) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (int rc = fold_deferred(e)) return rc;
    if (int rc = flush(e)) return rc;
    const size_t E = e->E, R = (size_t)e->T * E;
    if (int rc = ensure_tmp(e)) return rc;
    const gsx::DevState ds = dev_state(e);
    void* fields[gsx::NFIELD] = {s->first_message_deliveries, s->mesh_message_deliveries, s->mesh_failure_penalty,
                                 s->invalid_message_deliveries, s->graft_time_ns};
    for (int f = 0; f < gsx::NFIELD; ++f) {
        if (!fields[f]) continue;
        HIPCHK(e, gsx::launch_untile_field(ds, f, e->d_tmp, e->stream));
        HIPCHK(e, hipMemcpyAsync(fields[f], e->d_tmp, 8 * R, hipMemcpyDeviceToHost, e->stream));
    }
    if (s->mesh_time_ns) {
        HIPCHK(e, gsx::launch_mesh_time_export(ds, static_cast<int64_t*>(e->d_tmp), e->stream));
        HIPCHK(e, hipMemcpyAsync(s->mesh_time_ns, e->d_tmp, 8 * R, hipMemcpyDeviceToHost, e->stream));
    }
    if (s->rec_flags) {
        HIPCHK(e, gsx::launch_untile_field(ds, gsx::NFIELD, e->d_tmp, e->stream));
        HIPCHK(e, hipMemcpyAsync(s->rec_flags, e->d_tmp, R, hipMemcpyDeviceToHost, e->stream));
    }
    if (s->pair_flags) HIPCHK(e, hipMemcpyAsync(s->pair_flags, e->d_pflags, E, hipMemcpyDeviceToHost, e->stream));
    if (s->expire_ns) HIPCHK(e, hipMemcpyAsync(s->expire_ns, e->d_expire, 8 * E, hipMemcpyDeviceToHost, e->stream));
    if (s->behaviour_penalty) HIPCHK(e, hipMemcpyAsync(s->behaviour_penalty, e->d_bp, 8 * E, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    release_tmp(e);
    s->last_refresh_ns = e->last_refresh;
    return GSX_OK;
}

// inspectScoresExtended, score.go:463-493
int gsx_peer_score_snapshot(gsx_engine* e, gsx_score_snapshot* s) {
    if (!e || !s) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (int rc = ensure_scores(e)) return rc;
    const size_t E = e->E;
    if (s->score) HIPCHK(e, hipMemcpyAsync(s->score, e->d_score, 8 * E, hipMemcpyDeviceToHost, e->stream));
    if (s->app_specific_score) HIPCHK(e, hipMemcpyAsync(s->app_specific_score, e->d_app, 8 * E, hipMemcpyDeviceToHost, e->stream));
    if (s->ip_colocation_factor && E) {
        double* d = nullptr;
        if (int rc = dalloc(e, &d, E)) return rc;
        HIPCHK(e, gsx::launch_ip_colocation_export(dev_state(e), dev_peer_params(e), d, e->stream));
        HIPCHK(e, hipMemcpyAsync(s->ip_colocation_factor, d, 8 * E, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        (void)hipFree(d);
    }
    std::vector<uint8_t> pf;
    if (s->present) pf.resize(E);
    gsx_state_view v{};
    v.pair_flags = s->present ? pf.data() : nullptr;
    v.behaviour_penalty = s->behaviour_penalty;
    v.first_message_deliveries = s->first_message_deliveries;
    v.mesh_message_deliveries = s->mesh_message_deliveries;
    v.invalid_message_deliveries = s->invalid_message_deliveries;
    v.mesh_time_ns = s->time_in_mesh_ns;  // 0 outside the mesh, as the snapshot (score.go:479-481)
    if (int rc = gsx_export_state(e, &v)) return rc;
    for (size_t p = 0; p < pf.size(); ++p) s->present[p] = (pf[p] & GSX_PAIR_PRESENT) ? 1 : 0;
    return GSX_OK;
}

// Message propagation, see gsx.h and gsx_propagate.hip.
namespace {

// Words per call: 1, 2, or a multiple of 4 (the hop kernel's register chunk).
uint32_t prop_words(size_t m) {
    const uint32_t w = (uint32_t)((m + 63) / 64);
    if (w <= 2) return std::max<uint32_t>(w, 1);
    return (w + 3) & ~3u;
}

int prop_free_buffers(gsx_engine* e) {
    auto& P = e->prop;
    seen_release(e, P.seen, P.seen_words);
    if (e->vc_stream) (void)hipStreamSynchronize(e->vc_stream);  // (builds reading the history rows)
    e->vc_busy[0] = e->vc_busy[1] = false;
    e->hist_idx = 0;
    e->vc_last = -1;
    void* pp[] = {P.hist, P.origin, P.from, P.sel, P.occ, P.msgs, P.stats, P.touch, P.vcnt, P.vmask, P.hist_alt, P.occ_alt};
    for (void* p : pp)
        if (p) (void)hipFree(p);
    P.seen = P.hist = P.origin = P.from = P.sel = P.occ = P.touch = P.vcnt = P.vmask = nullptr;
    P.hist_alt = P.occ_alt = nullptr;
    P.from_words = 0;
    P.msgs = nullptr;
    P.stats = nullptr;
    P.words_cap = P.msgs_cap = P.rows_cap = 0;
    return GSX_OK;
}

// ---- topic membership (A13) ---------------------------------------------------

// Allocates the membership state with every node joined to every topic and
// no fanout (the state before any gsx_set_subscriptions / Join / Leave).
int members_init(gsx_engine* e) {
    if (e->members_on) return GSX_OK;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (e->sharded()) return fail(e, GSX_ESTATE, "topic membership runs on unsharded engines only");
    const size_t N = std::max<size_t>(e->n_nodes, 1), E = std::max<size_t>(e->E, 1);
    int rc = 0;
    if ((rc = dalloc(e, &e->d_sub, N)) || (rc = dalloc(e, &e->d_psub, E)) || (rc = dalloc(e, &e->d_fanout, E)) ||
        (rc = dalloc(e, &e->d_fan_has, N)) || (rc = dalloc(e, &e->d_lastpub, N * e->T)) ||
        (rc = dalloc(e, &e->d_mscratch, E)))
        return rc;
    const uint64_t all = e->T >= 64 ? ~0ull : ((1ull << e->T) - 1);
    e->h_sub.assign(e->n_nodes, all);
    HIPCHK(e, hipMemcpy(e->d_sub, e->h_sub.data(), 8 * (size_t)e->n_nodes, hipMemcpyHostToDevice));
    HIPCHK(e, gsx::launch_psub(e->d_col, e->d_sub, e->d_psub, e->E, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_fanout, 0, 8 * E, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_fan_has, 0, 8 * N, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_lastpub, 0, 8 * N * e->T, e->stream));
    e->members_on = true;
    ++e->mem_gen;
    return GSX_OK;
}

// The membership fields of a kernel state (the rest of the HbState is filled
// by hb_begin for heartbeats).
void member_fill(gsx_engine* e, gsx::HbState& h) {
    if (!e->members_on) return;
    h.psub = e->d_psub;
    h.sub = e->d_sub;
    h.fanout = e->d_fanout;
    h.fan_has = e->d_fan_has;
    h.lastpub = e->d_lastpub;
    h.mscratch = e->d_mscratch;
    h.pair_obs = e->d_pair_obs;
}
gsx::HbState member_state(gsx_engine* e) {
    gsx::HbState h{};
    h.row_ptr = e->d_row_ptr;
    h.rev = e->d_rev;
    h.eflags = e->d_eflags;
    h.n_pairs = e->E;
    h.n_nodes = e->n_nodes;
    h.gp.d = e->gp.d;
    h.publish_threshold = e->th.publish_threshold;
    member_fill(e, h);
    return h;
}
int member_list(gsx_engine* e, const std::vector<uint32_t>& v) {
    if (v.size() > e->mlist_cap) {
        if (e->d_mlist) (void)hipFree(e->d_mlist);
        e->d_mlist = nullptr;
        e->mlist_cap = std::max<size_t>(v.size(), 1024);
        if (int rc = dalloc(e, &e->d_mlist, 2 * e->mlist_cap)) return rc;
    }
    if (!v.empty()) HIPCHK(e, hipMemcpy(e->d_mlist, v.data(), 4 * v.size(), hipMemcpyHostToDevice));
    return GSX_OK;
}

gsx::PropState prop_state(gsx_engine* e, uint32_t W, size_t m, const gsx_prop_config* cfg) {
    auto& P = e->prop;
    gsx::PropState ps{};
    ps.row_ptr = e->d_row_ptr;
    ps.col = e->d_col;
    ps.rev = e->d_rev;
    ps.pair_obs = e->d_pair_obs;
    ps.eflags = e->d_eflags;
    ps.fwd = P.fwd;
    ps.pin = P.pin;
    ps.cent = P.cent;
    ps.rfwd = P.rfwd;
    ps.cend = P.cend;
    ps.chg = P.chg;
    ps.nchg = P.nchg;
    ps.ndirty = P.ndirty;
    ps.chg_cap = P.chg_cap;
    ps.corr = P.corr;
    ps.occ = P.occ;
    ps.max_hops = cfg->max_hops;
    ps.msgs = P.msgs;
    ps.seen = P.seen;
    ps.origin = P.origin;
    // first-deliverer rows: when tracked, and always for RandomSub (its draws exclude `from`)
    ps.from_mask = (e->prop_track || cfg->router == GSX_ROUTER_RANDOMSUB) ? P.from : nullptr;
    ps.fcnt = P.fcnt;
    ps.flast = P.flast;
    ps.invcnt = P.inv;
    ps.drop = P.has_drop ? P.vmask : nullptr;
    ps.dseen = P.has_drop ? P.dseen : nullptr;
    ps.reject = P.vmask ? P.vmask + W : nullptr;
    ps.hfrom = P.hfrom;
    ps.halo_tag = 0;
    ps.send_slot = e->d_send_slot;
    static const uint32_t occ_div = [] {
        const char* v = getenv("GSX_OCC_DIV");
        return v && atoi(v) > 0 ? (uint32_t)atoi(v) : 4u;
    }();
    ps.occ_div = occ_div;
    // (one-word rows: pushing marks costs more than the lean hop's walk of a frontier up to n / 128
    // — 64-message batch 1.42 -> 1.35 ms, tools/prop_ab.py; wider rows keep n / 16)
    static const uint32_t mark_div = [] {
        const char* v = getenv("GSX_MARK_DIV");
        return v && atoi(v) > 0 ? (uint32_t)atoi(v) : 0u;
    }();
    ps.mark_div = mark_div ? mark_div : (W == 1 ? 128u : 16u);
    ps.touch = P.touch;
    ps.halo_node = e->d_halo_node;
    ps.sel = cfg->router == GSX_ROUTER_RANDOMSUB ? P.sel : nullptr;
    ps.rcand = P.rcand;
    ps.hist = P.hist;
    ps.n_rows = 1;
    ps.dupcnt = P.dup;
    ps.firstcnt = P.first;
    ps.stats = P.stats;
    ps.send_pair = e->d_send_pair;
    ps.send_dest = e->d_send_dest;
    ps.send_base = e->d_send_base;
    ps.dest_halo_base = e->d_dest_halo_base;
    ps.n_ranks = e->n_ranks;
    ps.n_send = e->n_send;
    ps.n_pairs = e->E;
    ps.n_nodes = e->n_nodes;
    ps.n_words = W;
    ps.n_msgs = (uint32_t)m;
    ps.node_lo = e->node_lo;
    ps.router = cfg->router;
    ps.topic = cfg->topic;
    ps.flood_publish = cfg->flood_publish;
    if (e->members_on) {
        ps.psub = e->d_psub;
        ps.sub = e->d_sub;
        ps.fanout = e->d_fanout;
    }
    const bool scored = cfg->topic < e->T && e->scored[cfg->topic];
    ps.credit = (cfg->credit_scores && scored) ? 1 : 0;
    ps.window = scored ? e->tp[cfg->topic].mesh_message_deliveries_window_ns : 0;
    ps.hop_latency = cfg->hop_latency_ns;
    // A hop takes L = latency + validation delay D; a copy arriving g hops
    // after the first one is (g * L - D) after the first finished validating,
    // so it is inside the P3 window iff g * L <= window + D.
    const int64_t L = cfg->hop_latency_ns + cfg->validation_delay_ns, WD = ps.window + cfg->validation_delay_ns;
    ps.all_dups_in_window = ((int64_t)cfg->max_hops * L <= WD) ? 1 : 0;
    if (ps.window < 0) ps.win_hops = 0;
    else if (L == 0) ps.win_hops = GSX_MAX_HOPS + 1;
    else ps.win_hops = (uint32_t)std::min<int64_t>(WD / L, GSX_MAX_HOPS + 1);
    ps.back_in_window = (2 * L <= WD) ? 1 : 0;
    ps.late = (!ps.credit || ps.all_dups_in_window) ? 1 : 0;
    ps.pending = (P.credit_pending || !ps.late || e->sharded() || cfg->credit_scores == GSX_CREDIT_DEFER) ? 1 : 0;
    ps.rsub_sqrt = (uint32_t)std::ceil(std::sqrt((double)cfg->randomsub_size));
    ps.publish_threshold = e->th.publish_threshold;
    // AcceptFrom (gossipsub.go:583-594): only gossipsub graylists; floodsub and
    // RandomSub accept every RPC (their AcceptFrom returns AcceptAll)
    ps.gate = cfg->router == GSX_ROUTER_GOSSIPSUB ? 1 : 0;
    ps.graylist_threshold = e->th.graylist_threshold;
    ps.gray_pairs = P.gray_pairs;
    ps.seed = cfg->seed;
    ps.sharded = e->sharded() ? 1 : 0;
    {  // one-word lean calls on one engine: k_prop_hop_fast1 skips saturated receivers, and
       // STAT_EDGE_SENDS is counted at the call's end (GSX_NO_SAT_SKIP=1: A/B)
        static const bool no_skip = getenv("GSX_NO_SAT_SKIP") != nullptr || getenv("GSX_HOP_NO_FAST1") != nullptr;
        ps.edge_late = (!e->sharded() && W == 1 && m > 0 && gsx::hop_lean(ps) && !no_skip) ? 1u : 0u;
        ps.full1 = m >= 64 ? ~0ull : ((1ull << m) - 1);
    }
    return ps;
}

int prop_event_pair(gsx_engine* e, hipEvent_t* a, hipEvent_t* b) {
    auto& P = e->prop;
    while (P.ev.size() < (size_t)P.ev_used + 2) {
        hipEvent_t ev;
        HIPCHK(e, hipEventCreate(&ev));
        P.ev.push_back(ev);
    }
    *a = P.ev[P.ev_used++];
    *b = P.ev[P.ev_used++];
    return GSX_OK;
}

// Publish at sources that have not joined the topic: their fanout (gossipsub.go:981-998)
int fanout_publish(gsx_engine* e, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg) {
    if (!(e->members_on && cfg->router == GSX_ROUTER_GOSSIPSUB && !cfg->flood_publish && cfg->topic < e->T))
        return GSX_OK;
    // the pick reads scores against PublishThreshold, which deferred gossipsub pairs may not have reached yet
    if (int rc = fold_deferred(e)) return rc;
    if (e->lazy)
        if (int rc = ensure_scores(e)) return rc;
    const size_t N = e->n_nodes;
    std::vector<uint32_t> src;
    std::vector<uint8_t> done(N, 0);
    for (size_t k = 0; k < m; ++k) {
        const uint32_t v = msgs[k].source;
        if (v < N && !done[v] && !((e->h_sub[v] >> cfg->topic) & 1)) {
            done[v] = 1;
            src.push_back(v);
        }
    }
    if (src.empty()) return GSX_OK;
    if (int rc = member_list(e, src)) return rc;
    gsx::HbState hm = member_state(e);
    HIPCHK(e, gsx::launch_fanout_pick(dev_state(e), hm, e->d_mlist, (uint32_t)src.size(), cfg->topic, cfg->now_ns,
                                      cfg->seed, e->th.publish_threshold, e->stream));
    ++e->mem_gen;
    HIPCHK(e, hipStreamSynchronize(e->stream));  // `src` is on the host stack
    return GSX_OK;
}

int prop_begin(gsx_engine* e, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg) {
    if (!e || !cfg || (m && !msgs)) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (cfg->max_hops > GSX_MAX_HOPS || cfg->router > GSX_ROUTER_RANDOMSUB || m > 0xFFFFFFFFull ||
        cfg->credit_scores > GSX_CREDIT_DEFER || cfg->hop_latency_ns < 0)
        return fail(e, GSX_EINVAL, "bad propagation config");
    for (size_t k = 0; k < m; ++k) {
        if (msgs[k].source >= e->n_total) return fail(e, GSX_ERANGE, "message source out of range");
        if (msgs[k].validation > GSX_VALIDATION_THROTTLE) return fail(e, GSX_EINVAL, "bad message validation outcome");
    }
    if (cfg->validation_delay_ns < 0) return fail(e, GSX_EINVAL, "negative validation delay");
    if (cfg->router == GSX_ROUTER_GOSSIPSUB && e->gp.gossip_exchange && m > GSX_GX_MAX_SET_MSGS)
        return fail(e, GSX_ERANGE, "gossipsub batch above GSX_GX_MAX_SET_MSGS messages with the gossip exchange on "
                                   "(split it over several calls)");
    if (e->n_nodes > gsx::PIN_NODE_MASK) return fail(e, GSX_ERANGE, "propagation needs < 2^28 nodes per engine");
    auto& P = e->prop;
    const bool scored = cfg->topic < e->T && e->scored[cfg->topic];
    if (cfg->credit_scores && scored && P.credit_pending && P.credit_topic != cfg->topic)
        return fail(e, GSX_ESTATE, "deferred credits of another topic are pending: gsx_prop_fold_credits first");
    // gossipsub reads current scores (AcceptFrom's graylist gate on every pair,
    // publishThreshold for floodsub peers and flood publishing: k_prop_fwd);
    // the other routers never
    const bool need_score = cfg->router == GSX_ROUTER_GOSSIPSUB;
    // deferred credits of another topic (or a call that folds its own way) land first
    // (a gossipsub pair defers above the graylist threshold alone unless the call flood-publishes: k_prop_defer)
    if (e->deferred && (cfg->topic != e->def_topic || cfg->credit_scores != GSX_CREDIT_NOW ||
                        cfg->router != GSX_ROUTER_GOSSIPSUB || cfg->flood_publish != e->def_flood))
        if (int rc = fold_deferred(e)) return rc;
    if (int rc = flush(e)) return rc;  // queued events land first either way
    // (after lazy folds the fwd bytes stand for thresholds up to lazy_thr: the stale scores wait)
    const bool lazy_ok = e->lazy && !e->dirty_only && lazy_threshold(e) <= e->lazy_thr;
    if (need_score && !lazy_ok)
        if (int rc = ensure_scores(e)) return rc;
    const uint32_t W = prop_words(m);
    const size_t N = e->n_nodes, E = e->E;
    const uint32_t rows = cfg->max_hops + 1;
    if (W > P.words_cap || m > P.msgs_cap || rows > P.rows_cap || !P.fwd) {
        HIPCHK(e, hipStreamSynchronize(e->stream));
        prop_free_buffers(e);
        const size_t mm = std::max<size_t>(m, 1);
        int rc = 0;
        const uint32_t rc_rows = std::max<uint32_t>(rows, GSX_MAX_HOPS / 2 + 1);
        if ((rc = dalloc(e, &P.hist, (size_t)rc_rows * W * N)) ||
            (rc = dalloc(e, &P.occ, (size_t)rc_rows * ((N + 63) / 64))) ||
            (rc = dalloc(e, &P.touch, 2 * ((N + 63) / 64))) || (rc = dalloc(e, &P.vcnt, std::max<size_t>(N, 1))) ||
            (rc = dalloc(e, &P.origin, W * N)) || (rc = dalloc(e, &P.vmask, 2 * (size_t)W)) ||
            (rc = dalloc(e, &P.msgs, mm)) ||
            (rc = dalloc(e, &P.stats, (size_t)gsx::STAT_WORDS)))
            return rc;
        if (!P.fwd) {
            P.chg_cap = (uint32_t)std::min<size_t>(std::max<size_t>(E / 16, 1024), 1u << 24);
            if ((rc = dalloc(e, &P.fwd, E)) || (rc = dalloc(e, &P.pin, E)) || (rc = dalloc(e, &P.dup, E)) ||
                (rc = dalloc(e, &P.corr, E)) || (rc = dalloc(e, &P.fcnt, E)) || (rc = dalloc(e, &P.flast, E)) ||
                (rc = dalloc(e, &P.first, E)) || (rc = dalloc(e, &P.inv, E)) || (rc = dalloc(e, &P.gray_pairs, 1)) ||
                (rc = dalloc(e, &P.cent, E)) || (rc = dalloc(e, &P.cend, std::max<size_t>(N, 1))) ||
                (rc = dalloc(e, &P.rfwd, E)) ||
                (rc = dalloc(e, &P.chg, P.chg_cap)) || (rc = dalloc(e, &P.nchg, 1)) ||
                (rc = dalloc(e, &P.ndirty, (N + 63) / 64 + 1)))
                return rc;
            HIPCHK(e, hipMemsetAsync(P.nchg, 0, 4, e->stream));
            HIPCHK(e, hipMemsetAsync(P.ndirty, 0, 8 * ((N + 63) / 64 + 1), e->stream));
            HIPCHK(e, hipMemsetAsync(P.inv, 0, 4 * std::max<size_t>(E, 1), e->stream));
            HIPCHK(e, hipMemsetAsync(P.dup, 0, 4 * std::max<size_t>(E, 1), e->stream));
            HIPCHK(e, hipMemsetAsync(P.first, 0, 4 * std::max<size_t>(E, 1), e->stream));
        }
        P.words_cap = W;
        P.msgs_cap = (uint32_t)mm;
        P.rows_cap = rc_rows;
    }
    if (!P.seen) {  // handed to the message cache by the previous gossipsub call
        // the rows, then (kept by the message cache) the batch's per-node summary: dig[N] u64, cnt[N] u32
        P.seen_words = (size_t)P.words_cap * N + 2 * N;
        P.seen = seen_acquire(e, P.seen_words);
        if (!P.seen) return fail(e, GSX_ENOMEM, "hipMalloc: seen rows");
    }
    const bool rsub = cfg->router == GSX_ROUTER_RANDOMSUB;
    if (rsub && !P.sel) {
        if (int rc = dalloc(e, &P.sel, (size_t)P.words_cap * E)) return rc;
    }
    if (rsub && !P.rcand) {
        if (int rc = dalloc(e, &P.rcand, std::max<size_t>(E, 1))) return rc;
    }
    const bool track = e->prop_track || rsub;
    if (track && P.from_words < (size_t)P.words_cap * E) {
        if (P.from) (void)hipFree(P.from);
        P.from = nullptr;
        P.from_words = 0;
        if (int rc = dalloc(e, &P.from, (size_t)P.words_cap * E)) return rc;
        P.from_words = (size_t)P.words_cap * E;
    }
    if (e->n_recv) {  // compacted exchange: engine-owned halo of tagged rows (no clears: a row
                      // is empty unless its tag is this call's and hop's)
        if (P.halo_cap < (uint64_t)(W + 1) * e->n_recv) {
            if (P.halo) (void)hipFree(P.halo);
            P.halo = nullptr;
            P.halo_cap = 0;
            if (int rc = dalloc(e, &P.halo, (size_t)(W + 1) * e->n_recv)) return rc;
            HIPCHK(e, hipMemsetAsync(P.halo, 0, 8 * (size_t)(W + 1) * e->n_recv, e->stream));  // (tag 0: no call's)
            P.halo_cap = (uint64_t)(W + 1) * e->n_recv;
        }
        P.halo_tag = (uint64_t)(++P.halo_calls) << 8;  // (hops < 256)
    }
    if (e->n_send) {  // the compacted pack's per-(block, rank) table
        const uint64_t words = gsx::pack_table_words((uint32_t)N, e->n_ranks);
        if (P.pack_tab_cap < words) {
            if (P.pack_tab) (void)hipFree(P.pack_tab);
            P.pack_tab = nullptr;
            P.pack_tab_cap = 0;
            if (int rc = dalloc(e, &P.pack_tab, std::max<uint64_t>(words, 1))) return rc;
            P.pack_tab_cap = words;
        }
    }
    if (e->n_recv) {  // first receipts per remote sender, at the receiver's own pair (the pack reads
                      // them along the sender's row)
        if (P.hfrom_cap < (uint64_t)W * E) {
            if (P.hfrom) (void)hipFree(P.hfrom);
            P.hfrom = nullptr;
            if (int rc = dalloc(e, &P.hfrom, (size_t)W * E)) return rc;
            P.hfrom_cap = (uint64_t)W * E;
        }
        HIPCHK(e, hipMemsetAsync(P.hfrom, 0, 8 * (size_t)W * E, e->stream));
    }
    if (!P.dcount) {
        if (int rc = dalloc(e, &P.dcount, (size_t)gsx::MAX_RANKS)) return rc;
    }
    // pinned staging of the call's host inputs (the previous call ended with a
    // stream sync: nothing still reads it): [messages | drop / reject masks]
    // here, [the message set's arrays] in prop_end
    const size_t st_msgs = (sizeof(gsx::DevMsg) * m + 255) & ~(size_t)255;
    const size_t st_vm = (16 * (size_t)W + 255) & ~(size_t)255;
    const size_t st_set = ((4 * m + 7) & ~(size_t)7) + 8 * (size_t)W + 8 * ((size_t)W * 64 + W) + 8 * m + 256;
    if (P.h_stage_bytes < st_msgs + st_vm + st_set) {
        if (P.h_stage) (void)hipHostFree(P.h_stage);
        P.h_stage = nullptr;
        P.h_stage_bytes = 0;
        const size_t want = 2 * (st_msgs + st_vm + st_set);
        HIPCHK(e, hipHostMalloc(&P.h_stage, want, hipHostMallocDefault));
        P.h_stage_bytes = want;
    }
    uint64_t* vm = reinterpret_cast<uint64_t*>(static_cast<char*>(P.h_stage) + st_msgs);
    std::fill(vm, vm + 2 * (size_t)W, 0ull);
    {  // validation outcomes of this call: dropped / rejected message bits
        P.has_drop = false;
        for (size_t k = 0; k < m; ++k)
            if (msgs[k].validation != GSX_VALIDATION_ACCEPT) {
                vm[k / 64] |= 1ull << (k % 64);
                if (msgs[k].validation == GSX_VALIDATION_REJECT) vm[W + k / 64] |= 1ull << (k % 64);
                P.has_drop = true;
            }
        if (P.has_drop) {
            HIPCHK(e, hipMemcpyAsync(P.vmask, vm, 16 * (size_t)W, hipMemcpyHostToDevice, e->stream));
            if (P.dseen_words < (size_t)W * N) {
                if (P.dseen) (void)hipFree(P.dseen);
                P.dseen = nullptr;
                P.dseen_words = 0;
                if (int rc = dalloc(e, &P.dseen, (size_t)W * N)) return rc;
                P.dseen_words = (size_t)W * N;
            }
        }
    }
    gsx::PropState ps = prop_state(e, W, m, cfg);
    // Range shards, lean calls: the replicated frontier (PropState::rep) instead
    // of the per-pair halo (GSX_SHARD_PAIRS=1 keeps the per-pair exchange: A/B)
    static const bool no_rep = getenv("GSX_SHARD_PAIRS") != nullptr;
    P.rep = e->sharded() && e->n_ranks > 1 && m > 0 && gsx::hop_lean(ps) && !no_rep &&
            e->n_total <= gsx::PIN_NODE_MASK;
    if (P.rep && W == 1 && !getenv("GSX_NO_SAT_SKIP") && !getenv("GSX_HOP_NO_FAST1")) {
        // one-word lean calls on the replicated frontier: saturated receivers skipped as on
        // one engine; a cross pair's edge sends go with its end-of-call sends (k_rep_sends)
        ps.edge_late = 1;
    }
    if (P.rep) {
        const size_t NT = e->n_total, ow = (NT + 63) / 64 + 1;  // (the kernels' occ_g row: one spare word)
        if (P.rep_words < 2 * (uint64_t)NT * W) {
            for (uint64_t** p : {&P.front_g, &P.occ_g, &P.src_bits}) {
                if (*p) (void)hipFree(*p);
                *p = nullptr;
            }
            P.rep_words = 0;
            int rc = 0;
            if ((rc = dalloc(e, &P.front_g, 2 * NT * W)) || (rc = dalloc(e, &P.occ_g, 2 * ow)) ||
                (rc = dalloc(e, &P.src_bits, ow)))
                return rc;
            P.rep_words = 2 * (uint64_t)NT * W;
        }
        HIPCHK(e, hipMemsetAsync(P.occ_g, 0, 8 * ow, e->stream));  // parity 0: k_rep_init's sources
        HIPCHK(e, hipMemsetAsync(P.src_bits, 0, 8 * ow, e->stream));
        // the call's sources, ascending, with their origin rows (a remote receiver's own
        // messages at the end-of-call accounting, k_rep_sends)
        std::vector<std::pair<uint32_t, uint32_t>> sk(m);
        for (size_t k = 0; k < m; ++k) sk[k] = {msgs[k].source, (uint32_t)k};
        std::sort(sk.begin(), sk.end());
        P.h_src_ids.clear();
        P.h_src_rows.clear();
        for (size_t i = 0; i < m; ++i) {
            if (P.h_src_ids.empty() || P.h_src_ids.back() != sk[i].first) {
                P.h_src_ids.push_back(sk[i].first);
                P.h_src_rows.resize(P.h_src_rows.size() + W, 0);
            }
            P.h_src_rows[(P.h_src_ids.size() - 1) * W + sk[i].second / 64] |= 1ull << (sk[i].second % 64);
        }
        if (P.src_cap < (uint64_t)m * W || !P.src_ids) {
            if (P.src_ids) (void)hipFree(P.src_ids);
            if (P.src_rows) (void)hipFree(P.src_rows);
            P.src_ids = nullptr;
            P.src_rows = nullptr;
            int rc = 0;
            if ((rc = dalloc(e, &P.src_ids, m)) || (rc = dalloc(e, &P.src_rows, (size_t)m * W))) return rc;
            P.src_cap = (uint64_t)m * W;
        }
        HIPCHK(e, hipMemcpyAsync(P.src_ids, P.h_src_ids.data(), 4 * P.h_src_ids.size(), hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(P.src_rows, P.h_src_rows.data(), 8 * P.h_src_rows.size(), hipMemcpyHostToDevice,
                                 e->stream));
        ps.rep = 1;
        ps.n_total = e->n_total;
        ps.front_g = P.front_g;
        ps.occ_g = P.occ_g;
        ps.rmark_v = e->d_rmark_v;
        ps.rmark_u = e->d_rmark_u;
        ps.n_rmark = e->n_recv;
        ps.src_bits = P.src_bits;
        ps.src_ids = P.src_ids;
        ps.src_rows = P.src_rows;
        ps.n_src = (uint32_t)P.h_src_ids.size();
    }
    P.last = ps;
    P.have_last = true;
    P.cfg = *cfg;
    P.h = 0;
    P.global_last = UINT32_MAX;
    P.sel_done = false;
    P.ev_used = 0;
    P.launches = 0;
    P.loop_timing = false;
    P.ids.resize(m);
    P.vals.resize(m);
    for (size_t k = 0; k < m; ++k) {
        P.ids[k] = msgs[k].msg_id;
        P.vals[k] = msgs[k].validation;
    }
    if (cfg->router == GSX_ROUTER_GOSSIPSUB) set_sources(P.h_src, msgs, m);
    P.active = true;
    if (m == 0) {
        HIPCHK(e, hipMemsetAsync(P.stats, 0, 8 * (size_t)gsx::STAT_WORDS, e->stream));
        return GSX_OK;
    }
    auto* hm = static_cast<gsx::DevMsg*>(P.h_stage);
    for (size_t k = 0; k < m; ++k) hm[k] = gsx::DevMsg{msgs[k].source, msgs[k].validation, msgs[k].msg_id};
    HIPCHK(e, hipMemcpyAsync(P.msgs, hm, sizeof(gsx::DevMsg) * m, hipMemcpyHostToDevice, e->stream));
    // one launch clears the seen rows, first-receipt counts, occupancy row 0
    // (hist row 0 and origin: only the sources' rows are read, under it, and
    // cleared by k_prop_zero_src), both touch buffers, the counters; flast
    // only when a hop wrote it (k_prop_hop_fast: the max_hops cut), corr when
    // the per-hop accounting adds to it (the late one writes every pair it reads)
    HIPCHK(e, gsx::launch_prop_clear(ps, P.flast_dirty, !ps.late, e->stream));
    P.flast_dirty = false;
    if (track) HIPCHK(e, hipMemsetAsync(P.from, 0, 8 * (size_t)W * E, e->stream));
    if (rsub) HIPCHK(e, hipMemsetAsync(P.sel, 0, 8 * (size_t)W * E, e->stream));
    const gsx::DevState ds = dev_state(e);
    // fwd / pin (k_prop_fwd, k_prop_pin) read the router config, the pair and
    // record flags, the overlay and, where a threshold decides, the scores:
    // the last call's are reused while none of those moved (unsharded only:
    // a shard plan rewrites the reverse pairs)
    if (int rc = fanout_publish(e, msgs, m, cfg)) return rc;
    auto& K = P.fwd_key;
    const bool fwd_same = K.valid && !e->sharded() && K.router == cfg->router && K.topic == cfg->topic &&
                          K.flood_publish == cfg->flood_publish && K.flag_gen == e->flag_gen &&
                          K.publish_threshold == e->th.publish_threshold &&
                          K.graylist_threshold == e->th.graylist_threshold && K.mem_gen == e->mem_gen &&
                          (!need_score || K.score_gen == e->score_gen);
    if (fwd_same && P.fold_chg) {  // the last call's fold kept the bytes: its listed changes reach the pins
        gsx::PropState pf = ps;
        pf.inc = 1u;
        HIPCHK(e, gsx::launch_prop_fwd(pf, ds, e->stream, true));
    }
    P.fold_chg = false;
    if (!fwd_same) {
        HIPCHK(e, hipMemsetAsync(P.gray_pairs, 0, 8, e->stream));
        // the last call's fwd bytes, pins and compacted senders stand: update
        // what the changed bytes feed (unsharded: a shard's reverse pairs are its plan's)
        gsx::PropState pf = ps;
        pf.inc = (K.valid && !e->sharded()) ? 1u : 0u;
        // (replicated frontier: the remote pins arrive with the senders' fwd bytes, then compaction)
        HIPCHK(e, gsx::launch_prop_fwd(pf, ds, e->stream, false, !P.rep));
        K.valid = true;
        K.router = cfg->router;
        K.topic = cfg->topic;
        K.flood_publish = cfg->flood_publish;
        K.flag_gen = e->flag_gen;
        K.score_gen = e->score_gen;
        K.mem_gen = e->mem_gen;
        K.publish_threshold = e->th.publish_threshold;
        K.graylist_threshold = e->th.graylist_threshold;
    }
    HIPCHK(e, gsx::launch_prop_init(ps, P.hist, e->stream));
    if (P.rep) HIPCHK(e, gsx::launch_rep_init(ps, e->stream));
    return GSX_OK;
}

// Runs hop h = ++P.h; halo = the received rows of remote senders (sharded).
int prop_hop(gsx_engine* e, const uint64_t* halo) {
    auto& P = e->prop;
    gsx::PropState ps = P.last;
    if (ps.n_msgs == 0) {
        ++P.h;
        return GSX_OK;
    }
    ps.halo = halo;
    ps.halo_tag = (halo && halo == P.halo) ? P.halo_tag : 0;  // compacted: tagged rows (the dense exchange's are not)
    const uint32_t h = ++P.h;
    ++P.launches;
    hipEvent_t a = nullptr, b = nullptr;
    if (!P.loop_timing) {
        if (int rc = prop_event_pair(e, &a, &b)) return rc;
        HIPCHK(e, hipEventRecord(a, e->stream));
    }
    const size_t row = (size_t)ps.n_nodes * ps.n_words;
    const uint64_t* front = P.hist + (size_t)(h - 1) * row;
    const uint64_t* front_occ = P.occ + (size_t)(h - 1) * ((ps.n_nodes + 63) / 64);
    HIPCHK(e, gsx::launch_prop_mark(ps, h, front_occ, e->stream));  // also clears occupancy row h
    if (ps.sel && !P.sel_done) HIPCHK(e, gsx::launch_rsub_select(ps, front, front_occ, e->stream));
    P.sel_done = false;
    HIPCHK(e, gsx::launch_prop_hop(ps, h, front, P.hist + (size_t)h * row, e->stream));
    if (!P.loop_timing) HIPCHK(e, hipEventRecord(b, e->stream));
    return GSX_OK;
}

// gsx_propagate's early stop: whether hop h delivered anything, from the
// report k_prop_mark(h + 1) stores in host-mapped memory once hop h is done.
// Waits for the report; without one (the stream drained first, or failed)
// the answer is "yes" (the caller just launches the hop, which then does
// nothing).
bool hop_delivered(gsx_engine* e, uint32_t h) {
    auto& P = e->prop;
    const uint32_t want = P.hop_seq << 1;
    for (uint32_t spin = 1;; ++spin) {
        const uint32_t v = __atomic_load_n(P.hop_flag + h, __ATOMIC_ACQUIRE);
        if ((v & ~1u) == want) return v & 1u;
        if (spin % 64 == 0) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q != hipErrorNotReady) {
                const uint32_t w = __atomic_load_n(P.hop_flag + h, __ATOMIC_ACQUIRE);
                return (w & ~1u) == want ? (w & 1u) : true;
            }
        }
    }
}

int prop_fold(gsx_engine* e, const gsx::PropState& ps) {
    auto& P = e->prop;
    // (k_prop_fold leaves P.first / P.dup / P.inv (= ps.invcnt) empty)
    HIPCHK(e, gsx::launch_prop_fold(ps, dev_state(e), P.first, P.dup, e->stream));
    P.credit_pending = false;
    e->invalidate_scores();
    ++e->score_gen;
    return GSX_OK;
}

int prop_end(gsx_engine* e, gsx_prop_out* out) {
    auto& P = e->prop;
    const gsx::PropState& ps = P.last;
    std::memset(out, 0, sizeof(*out));
    P.active = false;
    if (ps.n_msgs == 0) return GSX_OK;
    {  // the lean hop kernels write flast only at the max_hops cut (or every hop when stepped)
        static const bool general = getenv("GSX_HOP_GENERAL") != nullptr;
        const bool lean = ps.late && !ps.sharded && !ps.sel && !ps.from_mask && !general;
        if (!lean || ps.flast_every || P.h >= ps.max_hops) P.flast_dirty = true;
    }
    const bool fold_now = ps.credit && P.cfg.credit_scores != GSX_CREDIT_DEFER;
    // the folded pairs are re-scored in the fold when every other score is
    // exact (gossipsub calls start from exact scores) and the fwd bytes match
    // this call's settings (unsharded, incremental fwd state)
    const bool rescore = fold_now && (e->scores_valid || (e->lazy && !e->dirty_only)) && e->pending.empty() &&
                         !e->sharded() && P.fwd_key.valid && P.fwd_key.score_gen == e->score_gen &&
                         P.cfg.router == GSX_ROUTER_GOSSIPSUB;
    // lazy: the credited pairs at or above every threshold keep a stale score (PropState::stale)
    static const bool no_lazy = getenv("GSX_NO_LAZY_FOLD") != nullptr;
    const double thr = lazy_threshold(e);
    const bool lazy = rescore && !no_lazy && credits_raise_scores(e) && (!e->lazy || thr <= e->lazy_thr);
    // deferred folds (PropState::acc_s / acc_f): the lazy pairs' credits are
    // summed over calls instead of folded per call; only the pairs below the
    // threshold (or with a P4 credit) fold now.  Late accounting on one engine
    // with no user-deferred counts (GSX_CREDIT_NOW), one topic's sums at a time
    static const bool no_defer = getenv("GSX_NO_DEFER_FOLD") != nullptr;
    const bool defer = lazy && !no_defer && ps.late && ps.credit && !e->sharded() && !P.credit_pending &&
                       P.cfg.credit_scores == GSX_CREDIT_NOW && ps.topic < e->T && e->scored[ps.topic] &&
                       (!e->deferred || (e->def_topic == ps.topic && e->def_flood == ps.flood_publish));
    if (defer && !e->d_acc_s) {
        const size_t E = std::max<size_t>(e->E, 1);
        if (int rc = dalloc(e, &e->d_acc_s, E)) return rc;
        if (int rc = dalloc(e, &e->d_acc_f, E)) return rc;
        HIPCHK(e, hipMemsetAsync(e->d_acc_s, 0, 4 * E, e->stream));
        HIPCHK(e, hipMemsetAsync(e->d_acc_f, 0, 4 * E, e->stream));
    }
    {
        gsx::PropState pd = ps;
        pd.flast_live = P.flast_dirty ? 1u : 0u;  // (flast is cleared at a call's start once written)
        if (defer) {
            pd.acc_s = e->d_acc_s;
            pd.acc_f = e->d_acc_f;
        }
        if (ps.late) HIPCHK(e, gsx::launch_prop_dups(pd, P.h, P.vcnt, false, e->stream));
        // per-hop accounting counts duplicates on arrival; the copies graylisting
        // receivers drop from local senders are counted here (the kernels return at
        // once when no pair is gated)
        else if (ps.gate) HIPCHK(e, gsx::launch_prop_dups(pd, P.h, P.vcnt, true, e->stream));
    }
    if (ps.credit || ps.late) {
        gsx::PropState pc = ps;
        // the topic-term cache (several topics: a fold then re-reads one topic's record, not all)
        static const bool no_tt = getenv("GSX_NO_TERM_CACHE") != nullptr;
        // A fold right after other changes (e.g. alternating with heartbeats)
        // runs without it (its terms would be stale before any later fold reads
        // them); the second of consecutive folds starts a cache epoch.
        const bool consecutive = P.t_rec_gen == e->rec_gen || P.t_plain_gen == e->rec_gen;
        if (rescore && !defer && e->T >= 2 && e->T <= 16 && !no_tt && consecutive) {
            if (!P.tterm) {
                if (int rc = dalloc(e, &P.tterm, (size_t)e->E * e->T)) return rc;
                if (int rc = dalloc(e, &P.tgen, (size_t)e->E)) return rc;
                HIPCHK(e, hipMemsetAsync(P.tgen, 0, 4 * std::max<size_t>(e->E, 1), e->stream));
                P.tepoch = 0;
                P.t_rec_gen = 0;
            }
            if (P.t_rec_gen != e->rec_gen) ++P.tepoch;  // records changed since: every pair's terms stale
            pc.tterm = P.tterm;
            pc.tgen = P.tgen;
            pc.tepoch = P.tepoch;
        }
        if (lazy) {
            if (!e->d_stale) {
                if (int rc = dalloc(e, &e->d_stale, std::max<size_t>(e->E, 1))) return rc;
                e->stale_marks = true;
            }
            if (!e->lazy && e->stale_marks)  // a new stale set
                HIPCHK(e, hipMemsetAsync(e->d_stale, 0, std::max<size_t>(e->E, 1), e->stream));
            pc.stale = e->d_stale;
            pc.lazy_thr = thr;
        }
        if (defer) {
            pc.acc_s = e->d_acc_s;
            pc.acc_f = e->d_acc_f;
            HIPCHK(e, gsx::launch_prop_defer(pc, dev_state(e), dev_peer_params(e), e->stream));
            e->deferred = true;
            e->def_topic = ps.topic;
            e->def_flood = ps.flood_publish;
            ++e->rec_gen;  // (the immediate folds bypass the topic-term cache)
        } else {
            HIPCHK(e, gsx::launch_prop_count(pc, dev_state(e), fold_now, rescore, dev_peer_params(e), e->stream));
            if (pc.tterm) P.t_rec_gen = e->rec_gen;
            else if (rescore) P.t_plain_gen = e->rec_gen;
        }
    }
    if (ps.credit) {
        // GSX_CREDIT_NOW: k_prop_count folded this call's counts (and any
        // pending ones of the topic) and left the pending counts empty
        P.credit_pending = !fold_now;
        P.credit_topic = ps.topic;
        if (rescore && lazy) {  // every fwd byte exact, every score but the stale pairs'
            ++e->score_writes;
            const bool was = e->lazy;
            e->scores_exact();
            e->scores_valid = false;
            e->lazy = true;
            e->stale_marks = true;
            e->lazy_thr = was ? std::min(e->lazy_thr, thr) : thr;
            ++e->score_gen;
            P.fwd_key.score_gen = e->score_gen;
            P.fold_chg = true;
        } else if (rescore) {  // every score exact again, the fwd bytes with them
            ++e->score_writes;
            e->scores_exact();
            ++e->score_gen;
            P.fwd_key.score_gen = e->score_gen;
            P.fold_chg = true;
        } else if (fold_now) {
            e->invalidate_scores();
            ++e->score_gen;
        }
    }
    const uint32_t W = ps.n_words;
    gsx_engine::MsgSet* set = nullptr;
    if (P.cfg.router == GSX_ROUTER_GOSSIPSUB) {  // the call's seen rows, before the uncache (a shard: its nodes')
        const size_t N = ps.n_nodes;
        set = new gsx_engine::MsgSet;
        set->serial = ++e->msg_serial;
        set->n_msgs = ps.n_msgs;
        set->n_words = W;
        set->topic = P.cfg.topic;
        set->ids = P.ids;
        set->refs = 1;
        set->all_words = (size_t)W * N;
        set->d_all = seen_acquire(e, set->all_words);
        if (!set->d_all) {
            delete set;
            return fail(e, GSX_ENOMEM, "seen rows of the message set");
        }
        HIPCHK(e, hipMemcpyAsync(set->d_all, P.seen, 8 * set->all_words, hipMemcpyDeviceToDevice, e->stream));
        std::vector<uint64_t>& acc = P.h_acc;
        acc.assign(W, 0);
        for (size_t k = 0; k < P.vals.size(); ++k)
            if (P.vals[k] == GSX_VALIDATION_ACCEPT) acc[k / 64] |= 1ull << (k % 64);
        const size_t mv = P.vals.size();
        if (!set_small_alloc(e, set, mv, W)) return fail(e, GSX_ENOMEM, "message set arrays");
        set->t0 = P.cfg.now_ns;
        {  // the set's block [validation | accepted words | id digests | origins], staged and copied at once
            const size_t st_off = ((sizeof(gsx::DevMsg) * mv + 255) & ~(size_t)255) + ((16 * (size_t)W + 255) & ~(size_t)255);
            char* blk = static_cast<char*>(P.h_stage) + st_off;
            const size_t val_b = (4 * std::max<size_t>(mv, 1) + 7) & ~(size_t)7;
            const size_t bytes = val_b + 8 * (size_t)W + 8 * ((size_t)W * 64 + W) + 8 * std::max<size_t>(mv, 1);
            std::memset(blk, 0, bytes);
            std::memcpy(blk, P.vals.data(), 4 * mv);
            std::memcpy(blk + val_b, acc.data(), 8 * (size_t)W);
            auto* dg = reinterpret_cast<uint64_t*>(blk + val_b + 8 * (size_t)W);  // ids: gsx.h (k_mc_summary)
            for (size_t k = 0; k < P.ids.size(); ++k) {
                dg[k] = id_digest(P.ids[k]);
                dg[(size_t)W * 64 + k / 64] += dg[k];
            }
            if (!P.h_src.empty())
                std::memcpy(blk + val_b + 8 * (size_t)W + 8 * ((size_t)W * 64 + W), P.h_src.data(), 8 * P.h_src.size());
            HIPCHK(e, hipMemcpyAsync(set->d_small, blk, bytes, hipMemcpyHostToDevice, e->stream));
        }
    }
    if (ps.drop) HIPCHK(e, gsx::launch_prop_uncache(ps, P.cfg.router == GSX_ROUTER_GOSSIPSUB, e->stream));
    if (P.cfg.router == GSX_ROUTER_GOSSIPSUB) {  // Publish Puts each processed message into the mcache
        gsx_engine::McBatch b;
        b.topic = P.cfg.topic;
        b.n_msgs = ps.n_msgs;
        b.n_words = W;
        b.d_seen = P.seen;  // the cache keeps this call's seen rows; the next call takes a pooled buffer
        b.seen_words = P.seen_words;
        {  // per-node (count, digest) summary of the batch for emitGossip (the set's id digests: gsx.h)
            const size_t N = ps.n_nodes;
            b.d_dig = P.seen + (size_t)W * N;
            b.d_cnt = reinterpret_cast<uint32_t*>(P.seen + (size_t)W * N + N);
            HIPCHK(e, gsx::launch_mc_summary(P.seen, (uint32_t)N, W, ps.n_msgs, set->d_dg, set->d_dg + (size_t)W * 64,
                                             b.d_dig, b.d_cnt, e->stream));
        }
        P.seen = nullptr;
        b.ids = P.ids;
        b.set = set;
        if (e->mc.empty()) e->mc.emplace_back();
        e->mc.front().push_back(std::move(b));
    }
    unsigned long long st[gsx::STAT_WORDS];
    HIPCHK(e, hipMemcpyAsync(st, P.stats, sizeof(st), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    out->duplicates = st[gsx::STAT_DUPS] - st[gsx::STAT_BACKSENDS];
    for (uint32_t h = 1; h <= GSX_MAX_HOPS; ++h) {
        out->hop_deliveries[h] = st[gsx::STAT_HOP0 + h];
        out->deliveries += st[gsx::STAT_HOP0 + h];
        if (st[gsx::STAT_HOP0 + h]) out->hops = h;
    }
    out->rejected = st[gsx::STAT_REJECTED];
    out->ignored = st[gsx::STAT_IGNORED];
    out->graylisted = st[gsx::STAT_GRAY];
    out->transmissions = out->deliveries + out->duplicates + out->rejected + out->ignored + out->graylisted;
    P.rows_valid = P.h + 1;
    for (uint32_t h = 1; h <= P.h && !ps.sharded; ++h)
        if (st[gsx::STAT_HOP0 + h] == 0) {  // hop h ran and wrote an empty row; later hops were skipped
            P.rows_valid = h + 1;
            break;
        }
    if (set) {  // the copies' validation times: code = arrival hop (gsx.h (D), VcRef)
        const int64_t step = P.cfg.hop_latency_ns + P.cfg.validation_delay_ns;
        // the last hop that delivered here: no code of this engine's nodes is later (the
        // hops launched past it — gsx_propagate's look-ahead, a shard's empty chunk
        // tail — differ between one engine and shards and hold no copy)
        // (a range shard told the ranks' last delivering hop takes it: every rank keeps the
        // same table, so the ranks classify the set's copies alike; not told: every hop run)
        uint32_t H = 0;
        if (ps.sharded) H = std::min(P.global_last, P.h);
        else
            for (uint32_t h = 1; h <= P.h && h <= GSX_MAX_HOPS; ++h)
                if (st[gsx::STAT_HOP0 + h]) H = h;
        set->vtime.resize(step > 0 ? H + 1 : 1);
        for (uint32_t h = 0; h < set->vtime.size(); ++h) set->vtime[h] = P.cfg.now_ns + (int64_t)h * step;
        set->n_hop = (uint32_t)set->vtime.size();
        // only the gossip exchange reads them (a propagation-only engine skips the build)
        if (step > 0 && H >= 1 && P.rows_valid > 1 && !e->gp.gossip_exchange) set->hops_kept = false;
        else if (step > 0 && H >= 1 && P.rows_valid > 1) {
            // (room for the next code: a recovery round's, without regrowing the planes)
            if (int rc = vc_grow(e, set, bit_width32(H + 1))) return rc;
            gsx::PropState pv = ps;
            pv.n_rows = P.rows_valid;
            if (int rc = vc_build(e, pv, set)) return rc;
        }
    }
    out->edge_sends = st[gsx::STAT_EDGE_SENDS];
    out->new_words = st[gsx::STAT_NEW_WORDS];
    double ms = 0;
    for (uint32_t i = 0; i + 1 < P.ev_used; i += 2) {
        float t = 0;
        HIPCHK(e, hipEventElapsedTime(&t, P.ev[i], P.ev[i + 1]));
        ms += t;
    }
    out->hop_kernel_ms = ms;
    out->hop_launches = P.launches;
    return GSX_OK;
}

}  // namespace

int gsx_propagate(gsx_engine* e, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg, gsx_prop_out* out) {
    if (!e || !cfg || !out) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (e->loaded && e->sharded())
        return fail(e, GSX_ESTATE, "sharded engine: drive hops with gsx_prop_begin/pack/step/end");
    if (e->prop.active) return fail(e, GSX_ESTATE, "a stepped propagation is in flight");
    if (int rc = prop_begin(e, msgs, m, cfg)) return rc;
    auto& P = e->prop;
    // Hops run back to back under one event pair.  Once a hop has delivered
    // nothing every later one is empty (its kernels return at once), so the
    // loop stops launching: before hop h it waits for hop h - 2's report
    // (hop h - 1 is queued meanwhile, the device never idles on the host).
    if (P.last.n_msgs && !P.hop_flag) {
        void* hf = nullptr;
        HIPCHK(e, hipHostMalloc(&hf, 4 * (GSX_MAX_HOPS + 1), hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(hf, 0, 4 * (GSX_MAX_HOPS + 1));
        P.hop_flag = static_cast<uint32_t*>(hf);
        void* dp = nullptr;
        HIPCHK(e, hipHostGetDevicePointer(&dp, hf, 0));
        P.d_hop_flag = static_cast<uint32_t*>(dp);
    }
    if (P.last.n_msgs) {
        P.hop_seq = (P.hop_seq + 1) & 0x7FFFFFFFu;
        if (P.hop_seq == 0) P.hop_seq = 1;
        P.last.hop_flag = P.d_hop_flag;
        P.last.hop_seq = P.hop_seq;
        P.loop_timing = true;
    }
    hipEvent_t a = nullptr, b = nullptr;
    if (P.loop_timing) {
        if (int rc = prop_event_pair(e, &a, &b)) return rc;
        HIPCHK(e, hipEventRecord(a, e->stream));
    }
    // (GSX_PROP_AHEAD: hops queued past the one the host waits for, A/B)
    static const uint32_t ahead = [] {
        const char* v = getenv("GSX_PROP_AHEAD");
        return v && atoi(v) > 0 ? (uint32_t)atoi(v) : 2u;
    }();
    for (uint32_t h = 1; h <= cfg->max_hops; ++h) {
        if (P.loop_timing && h > ahead && !hop_delivered(e, h - ahead)) break;
        if (int rc = prop_hop(e, nullptr)) return rc;
    }
    if (P.loop_timing) HIPCHK(e, hipEventRecord(b, e->stream));
    P.last.hop_flag = nullptr;  // the stepped entry points leave it off
    return prop_end(e, out);
}

int gsx_prop_begin(gsx_engine* e, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg) {
    if (!e) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (e->prop.active) return fail(e, GSX_ESTATE, "a stepped propagation is in flight");
    if (e->loaded && e->sharded() && (e->n_ranks > 1) && !e->d_send_pair)
        return fail(e, GSX_ESTATE, "shard plan incomplete: gsx_shard_send_plan first");
    if (e->loaded && e->sharded() && e->n_ranks == 1 && e->n_total != e->n_nodes)
        return fail(e, GSX_ESTATE, "shard plan missing: gsx_shard_recv_plan / gsx_shard_send_plan first");
    if (int rc = prop_begin(e, msgs, m, cfg)) return rc;
    e->prop.last.flast_every = 1;  // the caller may end the call after any hop
    return GSX_OK;
}

int gsx_prop_pack(gsx_engine* e, uint64_t* send) {
    if (!e) return GSX_EINVAL;
    auto& P = e->prop;
    if (!P.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    if (P.rep) return fail(e, GSX_ESTATE, "this call runs the replicated frontier (gsx_prop_rep_*)");
    if (e->n_send && !send) return GSX_EINVAL;
    if (P.h >= P.cfg.max_hops) return fail(e, GSX_ERANGE, "max_hops reached");
    const gsx::PropState& ps = P.last;
    if (ps.n_msgs == 0 || e->n_send == 0) return GSX_OK;
    hipEvent_t a, b;
    if (int rc = prop_event_pair(e, &a, &b)) return rc;
    HIPCHK(e, hipEventRecord(a, e->stream));
    const uint64_t* front = P.hist + (size_t)P.h * ps.n_nodes * ps.n_words;
    const uint64_t* front_occ = P.occ + (size_t)P.h * ((ps.n_nodes + 63) / 64);
    if (ps.sel) HIPCHK(e, gsx::launch_rsub_select(ps, front, front_occ, e->stream));
    P.sel_done = true;
    ++P.launches;
    HIPCHK(e, gsx::launch_prop_pack(ps, front, front_occ, send, e->stream));
    HIPCHK(e, hipEventRecord(b, e->stream));
    return GSX_OK;
}

int gsx_prop_step(gsx_engine* e, const uint64_t* recv, uint64_t* n_new) {
    if (!e) return GSX_EINVAL;
    auto& P = e->prop;
    if (!P.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    if (P.rep) return fail(e, GSX_ESTATE, "this call runs the replicated frontier (gsx_prop_rep_*)");
    if (e->n_recv && !recv) return GSX_EINVAL;
    if (P.h >= P.cfg.max_hops) return fail(e, GSX_ERANGE, "max_hops reached");
    if (int rc = prop_hop(e, recv)) return rc;
    if (n_new) {
        unsigned long long c = 0;
        if (P.last.n_msgs)
            HIPCHK(e, hipMemcpyAsync(&c, P.stats + gsx::STAT_HOP0 + P.h, 8, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        *n_new = c;
    }
    return GSX_OK;
}

int gsx_prop_hop_counts_dev(gsx_engine* e, int64_t* d_out) {
    if (!e || !d_out) return GSX_EINVAL;
    auto& P = e->prop;
    if (!P.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    if (P.last.n_msgs == 0) {
        HIPCHK(e, hipMemsetAsync(d_out, 0, 8 * (GSX_MAX_HOPS + 1), e->stream));
        return GSX_OK;
    }
    HIPCHK(e, hipMemcpyAsync(d_out, P.stats + gsx::STAT_HOP0, 8 * (GSX_MAX_HOPS + 1), hipMemcpyDeviceToDevice,
                             e->stream));
    return GSX_OK;
}

namespace {
// Pack the compacted exchange of hop P.h + 1 (the entry counts stay in P.dcount).
int pack_compact(gsx_engine* e, uint64_t* out, bool* packed) {
    auto& P = e->prop;
    *packed = false;
    if (!P.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    if (P.rep) return fail(e, GSX_ESTATE, "this call runs the replicated frontier (gsx_prop_rep_*)");
    if (e->n_send && !out) return GSX_EINVAL;
    if (e->n_send && !e->d_dest_halo_base) return fail(e, GSX_ESTATE, "gsx_shard_set_halo_bases first");
    if (P.h >= P.cfg.max_hops) return fail(e, GSX_ERANGE, "max_hops reached");
    const gsx::PropState& ps = P.last;
    if (ps.n_msgs == 0 || e->n_send == 0) return GSX_OK;
    const uint64_t* front = P.hist + (size_t)P.h * ps.n_nodes * ps.n_words;
    const uint64_t* front_occ = P.occ + (size_t)P.h * ((ps.n_nodes + 63) / 64);
    hipEvent_t a, b;
    if (int rc = prop_event_pair(e, &a, &b)) return rc;
    HIPCHK(e, hipEventRecord(a, e->stream));
    if (ps.sel) HIPCHK(e, gsx::launch_rsub_select(ps, front, front_occ, e->stream));
    P.sel_done = true;
    HIPCHK(e, hipMemsetAsync(P.dcount, 0, 8 * (size_t)e->n_ranks, e->stream));
    ++P.launches;
    HIPCHK(e, gsx::launch_prop_pack_compact(ps, front, front_occ, out, P.dcount, P.pack_tab, e->stream));
    HIPCHK(e, hipEventRecord(b, e->stream));
    *packed = true;
    return GSX_OK;
}
}  // namespace

int gsx_prop_pack_compact(gsx_engine* e, uint64_t* out, uint64_t* counts) {
    if (!e || !counts) return GSX_EINVAL;
    bool packed = false;
    if (int rc = pack_compact(e, out, &packed)) return rc;
    std::memset(counts, 0, 8 * (size_t)e->n_ranks);
    if (!packed) return GSX_OK;
    HIPCHK(e, hipMemcpyAsync(counts, e->prop.dcount, 8 * (size_t)e->n_ranks, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_prop_pack_compact_dev(gsx_engine* e, uint64_t* out, int64_t* d_counts) {
    if (!e || !d_counts) return GSX_EINVAL;
    bool packed = false;
    if (int rc = pack_compact(e, out, &packed)) return rc;
    auto& P = e->prop;
    const unsigned long long* hop_new = P.last.n_msgs ? P.stats + gsx::STAT_HOP0 + P.h : nullptr;
    HIPCHK(e, gsx::launch_pack_counts(packed ? P.dcount : nullptr, hop_new, e->n_ranks, d_counts, e->stream));
    return GSX_OK;
}

int gsx_prop_step_compact(gsx_engine* e, const uint64_t* entries, uint64_t n_entries, uint64_t* n_new) {
    if (!e) return GSX_EINVAL;
    auto& P = e->prop;
    if (!P.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    if (n_entries && !entries) return GSX_EINVAL;
    if (n_entries > e->n_recv) return fail(e, GSX_ERANGE, "more entries than receive slots");
    if (P.h >= P.cfg.max_hops) return fail(e, GSX_ERANGE, "max_hops reached");
    const gsx::PropState& ps = P.last;
    if (ps.n_msgs && e->n_recv) {
        gsx::PropState pt = ps;
        pt.halo = P.halo;
        pt.halo_tag = P.halo_tag;
        HIPCHK(e, gsx::launch_halo_scatter(pt, P.halo, entries, n_entries, P.h + 1, e->stream));
    }
    return gsx_prop_step(e, e->n_recv ? P.halo : nullptr, n_new);
}

int gsx_prop_set_last_hop(gsx_engine* e, uint32_t last_hop) {
    if (!e) return GSX_EINVAL;
    if (!e->prop.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    if (last_hop > GSX_MAX_HOPS) return fail(e, GSX_ERANGE, "last hop above GSX_MAX_HOPS");
    e->prop.global_last = last_hop;
    return GSX_OK;
}

int gsx_prop_end(gsx_engine* e, gsx_prop_out* out) {
    if (!e || !out) return GSX_EINVAL;
    if (!e->prop.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    return prop_end(e, out);
}

// ---- range shards, replicated frontier (gsx.h) ----
namespace {
int rep_ready(gsx_engine* e, bool before_hops) {
    auto& P = e->prop;
    if (!P.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    if (!P.rep) return fail(e, GSX_ESTATE, "this call runs the per-pair exchange (gsx_prop_rep says 0)");
    if (before_hops && P.h != 0) return fail(e, GSX_ESTATE, "the fwd bytes go before the first hop");
    return GSX_OK;
}
}  // namespace

int gsx_prop_rep(gsx_engine* e, uint32_t* on) {
    if (!e || !on) return GSX_EINVAL;
    if (!e->prop.active) return fail(e, GSX_ESTATE, "no propagation in flight");
    *on = e->prop.rep ? 1u : 0u;
    return GSX_OK;
}

int gsx_prop_rep_fwd_pack(gsx_engine* e, uint8_t* out) {
    if (!e || (e->n_send && !out)) return GSX_EINVAL;
    if (int rc = rep_ready(e, true)) return rc;
    HIPCHK(e, gsx::launch_rep_fwd_pack(e->prop.last, out, e->stream));
    return GSX_OK;
}

int gsx_prop_rep_fwd_recv(gsx_engine* e, const uint8_t* in) {
    if (!e || (e->n_recv && !in)) return GSX_EINVAL;
    if (int rc = rep_ready(e, true)) return rc;
    const gsx::PropState& ps = e->prop.last;
    HIPCHK(e, gsx::launch_rep_fwd_recv(ps, in, e->stream));
    HIPCHK(e, gsx::launch_prop_compact(ps, e->stream));
    return GSX_OK;
}

int gsx_prop_rep_pack_dev(gsx_engine* e, uint64_t* out, int64_t* d_counts) {
    if (!e || !out || !d_counts) return GSX_EINVAL;
    if (int rc = rep_ready(e, false)) return rc;
    auto& P = e->prop;
    if (P.h == 0) return fail(e, GSX_ESTATE, "hop 0 is every rank's already: step hop 1 first");
    hipEvent_t a, b;  // (in the call's hop_kernel_ms, with the hops and the scatters)
    if (int rc = prop_event_pair(e, &a, &b)) return rc;
    HIPCHK(e, hipEventRecord(a, e->stream));
    HIPCHK(e, hipMemsetAsync(P.dcount, 0, 8, e->stream));
    HIPCHK(e, gsx::launch_rep_pack(P.last, P.h, out, P.dcount, e->stream));
    HIPCHK(e, gsx::launch_pack_counts(P.dcount, P.stats + gsx::STAT_HOP0 + P.h, 1, d_counts, e->stream));
    HIPCHK(e, hipEventRecord(b, e->stream));
    return GSX_OK;
}

int gsx_prop_rep_step(gsx_engine* e, uint32_t n_parts, const uint64_t* const* parts, const uint64_t* counts) {
    if (!e || (n_parts && (!parts || !counts))) return GSX_EINVAL;
    if (n_parts > gsx::MAX_RANKS) return fail(e, GSX_ERANGE, "more parts than ranks");
    if (int rc = rep_ready(e, false)) return rc;
    auto& P = e->prop;
    if (P.h >= P.cfg.max_hops) return fail(e, GSX_ERANGE, "max_hops reached");
    uint64_t total = 0;
    for (uint32_t k = 0; k < n_parts; ++k) {
        if (counts[k] && !parts[k]) return GSX_EINVAL;
        total += counts[k];
    }
    if (total > (uint64_t)e->n_total) return fail(e, GSX_ERANGE, "more frontier rows than nodes");
    if (P.h > 0 && P.h < P.cfg.max_hops) {
        P.last.rep_in = total;  // (hop P.h + 1's marking counts them: mark_hop)
        if (total) {
            hipEvent_t a, b;
            if (int rc = prop_event_pair(e, &a, &b)) return rc;
            HIPCHK(e, hipEventRecord(a, e->stream));
            gsx::RepParts rp{};
            for (uint32_t k = 0; k < n_parts; ++k) {
                if (!counts[k]) continue;
                rp.p[rp.n] = parts[k];
                rp.off[rp.n + 1] = rp.off[rp.n] + counts[k];
                ++rp.n;
            }
            HIPCHK(e, gsx::launch_rep_scatter(P.last, P.h, rp, e->stream));
            HIPCHK(e, hipEventRecord(b, e->stream));
        }
    } else if (total) {
        return fail(e, GSX_ESTATE, "hop 0's rows need no exchange");
    } else {
        P.last.rep_in = 0;
    }
    return prop_hop(e, nullptr);
}

int gsx_prop_rep_rows(gsx_engine* e, uint32_t on) {
    if (!e) return GSX_EINVAL;
    if (int rc = rep_ready(e, true)) return rc;
    e->prop.last.rep_rows = on ? 1u : 0u;
    return GSX_OK;
}

int gsx_prop_rep_rows_export(gsx_engine* e, uint64_t* rows, uint64_t* occ) {
    if (!e || !rows || !occ) return GSX_EINVAL;
    if (int rc = rep_ready(e, false)) return rc;
    auto& P = e->prop;
    if (!P.last.rep_rows) return fail(e, GSX_ESTATE, "gsx_prop_rep_rows(e, 1) before the first hop");
    if (P.h == 0) return fail(e, GSX_ESTATE, "hop 0 is every rank's already: step hop 1 first");
    const size_t W = P.last.n_words, NT = e->n_total, ow = (NT + 63) / 64 + 1;
    const uint64_t* fg = P.front_g + (size_t)(P.h & 1) * NT * W;
    HIPCHK(e, hipMemcpyAsync(rows, fg + (size_t)e->node_lo * W, 8 * W * e->n_nodes, hipMemcpyDeviceToDevice,
                             e->stream));
    HIPCHK(e, hipMemcpyAsync(occ, P.occ_g + (size_t)(P.h & 1) * ow, 8 * ow, hipMemcpyDeviceToDevice, e->stream));
    return GSX_OK;
}

int gsx_prop_rep_rows_step(gsx_engine* e, uint32_t n_parts, const uint64_t* const* parts, const uint64_t* occ_sum) {
    if (!e || !parts || !occ_sum) return GSX_EINVAL;
    if (int rc = rep_ready(e, false)) return rc;
    auto& P = e->prop;
    if (!P.last.rep_rows) return fail(e, GSX_ESTATE, "gsx_prop_rep_rows(e, 1) before the first hop");
    if (n_parts != e->n_ranks || e->rank_lo.size() != (size_t)n_parts + 1)
        return fail(e, GSX_EINVAL, "one part per rank of the shard plan");
    if (P.h == 0) return fail(e, GSX_ESTATE, "hop 0's rows need no exchange");
    if (P.h >= P.cfg.max_hops) return fail(e, GSX_ERANGE, "max_hops reached");
    const size_t W = P.last.n_words, NT = e->n_total, ow = (NT + 63) / 64 + 1;
    uint64_t* fg = P.front_g + (size_t)(P.h & 1) * NT * W;
    hipEvent_t a, b;  // (in the call's hop_kernel_ms, with the hops)
    if (int rc = prop_event_pair(e, &a, &b)) return rc;
    HIPCHK(e, hipEventRecord(a, e->stream));
    for (uint32_t k = 0; k < n_parts; ++k) {  // every other rank's slice of the hop's rows, in place
        const uint32_t lo = e->rank_lo[k], n = e->rank_lo[k + 1] - lo;
        if (lo == e->node_lo || !n) continue;  // (this rank's rows are there already)
        if (!parts[k]) return GSX_EINVAL;
        HIPCHK(e, hipMemcpyAsync(fg + (size_t)lo * W, parts[k], 8 * W * n, hipMemcpyDeviceToDevice, e->stream));
    }
    // every rank's occupancy bits of the hop: the sum of bit rows whose ranks own disjoint bits
    HIPCHK(e, hipMemcpyAsync(P.occ_g + (size_t)(P.h & 1) * ow, occ_sum, 8 * ow, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipEventRecord(b, e->stream));
    P.last.rep_in = NT;  // (remote rows may reach every hop: it never returns early on the local count)
    return prop_hop(e, nullptr);
}

int gsx_prop_rep_sends_pack(gsx_engine* e, uint64_t* out) {
    if (!e || (e->n_send && !out)) return GSX_EINVAL;
    if (int rc = rep_ready(e, false)) return rc;
    auto& P = e->prop;
    HIPCHK(e, gsx::launch_rep_sends(P.last, P.h, P.vcnt, out, e->stream));
    return GSX_OK;
}

int gsx_prop_rep_sends_recv(gsx_engine* e, const uint64_t* in) {
    if (!e || (e->n_recv && !in)) return GSX_EINVAL;
    if (int rc = rep_ready(e, false)) return rc;
    HIPCHK(e, gsx::launch_rep_sends_recv(e->prop.last, in, e->stream));
    return GSX_OK;
}

// Device memory on both sides: the copies stay ordered on the engine's
// stream (a caller's stream via gsx_set_stream) and the call returns at once;
// host memory: the call waits for them.
bool on_device(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable host memory: not a HIP allocation
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

int gsx_prop_pending_credits(gsx_engine* e, uint32_t* first, uint32_t* dup) {
    if (!e) return GSX_EINVAL;
    if (!e->loaded || !e->prop.first) return fail(e, GSX_ESTATE, "no propagation yet");
    if (int rc = fold_deferred(e)) return rc;
    if (first) HIPCHK(e, hipMemcpyAsync(first, e->prop.first, 4 * e->E, hipMemcpyDefault, e->stream));
    if (dup) HIPCHK(e, hipMemcpyAsync(dup, e->prop.dup, 4 * e->E, hipMemcpyDefault, e->stream));
    if ((first && !on_device(first)) || (dup && !on_device(dup))) HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_prop_pending_invalid(gsx_engine* e, uint32_t* inv) {
    if (!e || !inv) return GSX_EINVAL;
    if (!e->loaded || !e->prop.inv) return fail(e, GSX_ESTATE, "no propagation yet");
    if (int rc = fold_deferred(e)) return rc;
    HIPCHK(e, hipMemcpyAsync(inv, e->prop.inv, 4 * e->E, hipMemcpyDefault, e->stream));
    if (!on_device(inv)) HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_prop_replace_pending_invalid(gsx_engine* e, const uint32_t* inv) {
    if (!e || !inv) return GSX_EINVAL;
    if (!e->loaded || !e->prop.inv) return fail(e, GSX_ESTATE, "no propagation yet");
    if (e->prop.active) return fail(e, GSX_ESTATE, "a stepped propagation is in flight");
    if (int rc = fold_deferred(e)) return rc;
    HIPCHK(e, hipMemcpyAsync(e->prop.inv, inv, 4 * e->E, hipMemcpyDefault, e->stream));
    if (!on_device(inv)) HIPCHK(e, hipStreamSynchronize(e->stream));
    e->prop.credit_pending = true;
    return GSX_OK;
}

int gsx_prop_fold_credits(gsx_engine* e, const uint32_t* first, const uint32_t* dup) {
    if (!e) return GSX_EINVAL;
    if (!e->loaded || !e->prop.first) return fail(e, GSX_ESTATE, "no propagation yet");
    if ((first == nullptr) != (dup == nullptr)) return GSX_EINVAL;
    auto& P = e->prop;
    if (P.active) return fail(e, GSX_ESTATE, "a stepped propagation is in flight");
    if (int rc = fold_deferred(e)) return rc;
    if (first) {
        HIPCHK(e, hipMemcpyAsync(P.first, first, 4 * e->E, hipMemcpyDefault, e->stream));
        HIPCHK(e, hipMemcpyAsync(P.dup, dup, 4 * e->E, hipMemcpyDefault, e->stream));
    } else if (!P.credit_pending) {
        return GSX_OK;
    }
    gsx::PropState ps = P.last;
    ps.topic = P.credit_pending ? P.credit_topic : P.cfg.topic;
    if (int rc = prop_fold(e, ps)) return rc;
    if (first && (!on_device(first) || !on_device(dup))) HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_prop_set_tracking(gsx_engine* e, uint32_t first_deliverers) {
    if (!e) return GSX_EINVAL;
    if (e->prop.active) return fail(e, GSX_ESTATE, "a stepped propagation is in flight");
    e->prop_track = first_deliverers != 0;
    return GSX_OK;
}

int gsx_prop_results(gsx_engine* e, uint8_t* hop, int32_t* first_from) {
    if (!e) return GSX_EINVAL;
    if (!e->prop.have_last) return fail(e, GSX_ESTATE, "no gsx_propagate call yet");
    gsx::PropState ps = e->prop.last;
    ps.n_rows = e->prop.rows_valid;
    const size_t cells = (size_t)ps.n_msgs * ps.n_nodes;
    if (cells == 0) return GSX_OK;
    if (hop) {
        uint8_t* d_h = nullptr;
        if (int rc = dalloc(e, &d_h, cells)) return rc;
        HIPCHK(e, gsx::launch_prop_hops_export(ps, d_h, e->stream));
        HIPCHK(e, hipMemcpyAsync(hop, d_h, cells, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        (void)hipFree(d_h);
    }
    if (first_from) {
        if (!ps.from_mask)
            return fail(e, GSX_ESTATE, "first deliverers were not tracked in the last call (gsx_prop_set_tracking)");
        int32_t* d_ff = nullptr;
        if (int rc = dalloc(e, &d_ff, cells)) return rc;
        HIPCHK(e, hipMemsetAsync(d_ff, 0xFF, 4 * cells, e->stream));
        HIPCHK(e, gsx::launch_prop_from(ps, d_ff, e->stream));
        HIPCHK(e, hipMemcpyAsync(first_from, d_ff, 4 * cells, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        (void)hipFree(d_ff);
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_prop_duplicates(gsx_engine* e, uint64_t* rows, size_t n_words) {
    if (!e || !rows) return GSX_EINVAL;
    if (!e->prop.have_last) return fail(e, GSX_ESTATE, "no gsx_propagate call yet");
    if (e->prop.active) return fail(e, GSX_ESTATE, "a stepped propagation is in flight");
    if (e->sharded()) return fail(e, GSX_EINVAL, "duplicate rows are exported by unsharded engines only");
    gsx::PropState ps = e->prop.last;
    if (!ps.from_mask)
        return fail(e, GSX_ESTATE, "first deliverers were not tracked in the last call (gsx_prop_set_tracking)");
    if (n_words != ps.n_words) return fail(e, GSX_EINVAL, "n_words must be the last call's words (ceil(m / 64))");
    ps.n_rows = e->prop.rows_valid;
    const size_t cells = (size_t)e->E * ps.n_words;
    if (cells == 0) return GSX_OK;
    uint64_t* d = nullptr;
    if (int rc = dalloc(e, &d, cells)) return rc;
    HIPCHK(e, gsx::launch_prop_dup_rows(ps, d, e->stream));
    HIPCHK(e, hipMemcpyAsync(rows, d, 8 * cells, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    (void)hipFree(d);
    return GSX_OK;
}

int gsx_shard_counts(gsx_engine* e, uint64_t* n_send, uint64_t* n_recv) {
    if (!e) return GSX_EINVAL;
    if (n_send) *n_send = e->n_send;
    if (n_recv) *n_recv = e->n_recv;
    return GSX_OK;
}

// DefaultGossipSubParams, gossipsub.go:230-260
int gsx_default_gossipsub_params(gsx_gossipsub_params* p) {
    if (!p) return GSX_EINVAL;
    std::memset(p, 0, sizeof(*p));
    p->d = 6;
    p->d_lo = 5;
    p->d_hi = 12;
    p->d_score = 4;
    p->d_out = 2;
    p->opportunistic_graft_peers = 2;
    p->opportunistic_graft_ticks = 60;
    p->prune_backoff_ns = 60LL * 1000000000LL;
    p->graft_flood_threshold_ns = 10LL * 1000000000LL;
    p->d_lazy = 6;
    p->history_length = 5;
    p->history_gossip = 5;
    p->max_ihave_length = 5000;
    p->gossip_factor = 0.25;
    p->max_ihave_messages = 10;
    p->gossip_retransmission = 3;
    p->iwant_followup_ns = 3LL * 1000000000LL;
    p->gossip_exchange = 1;  // the reference always handles IHAVE/IWANT (gossipsub.go:615-720)
    p->fanout_ttl_ns = 60LL * 1000000000LL;
    p->do_px = 0;           // WithPeerExchange is opt-in (:325-333)
    p->prune_peers = 16;    // GossipSubPrunePeers
    return GSX_OK;
}

// The reference takes GossipSubParams unchecked; the mesh lanes index their
// peer lists with D / Dscore, so negative or inverted degrees are refused.
int gsx_set_gossipsub_params(gsx_engine* e, const gsx_gossipsub_params* p) {
    if (!e || !p) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (p->d_lo < 0 || p->d < p->d_lo || p->d_hi < p->d || p->d_score < 0 || p->d_score > p->d_hi || p->d_out < 0 ||
        p->opportunistic_graft_peers < 0 || p->prune_backoff_ns < 0)
        return fail(e, GSX_EINVAL, "need 0 <= Dlo <= D <= Dhi, 0 <= Dscore <= Dhi, Dout, OG peers, backoff >= 0");
    // NewMessageCache panics on gossip > history (mcache.go:24-28)
    if (p->history_length < 1 || p->history_gossip < 0 || p->history_gossip > p->history_length ||
        p->d_lazy < 0 || p->max_ihave_length < 0 || !(p->gossip_factor >= 0))
        return fail(e, GSX_EINVAL, "need 0 <= HistoryGossip <= HistoryLength, HistoryLength >= 1, Dlazy, "
                                   "MaxIHaveLength, GossipFactor >= 0");
    if (p->gossip_exchange && (p->max_ihave_messages < 0 || p->gossip_retransmission < 0 || p->iwant_followup_ns < 0))
        return fail(e, GSX_EINVAL, "need MaxIHaveMessages, GossipRetransmission, IWantFollowupTime >= 0");
    if (p->do_px && p->prune_peers < 0) return fail(e, GSX_EINVAL, "need PrunePeers >= 0");
    if (p->do_px != e->gp.do_px) e->hb_clean = false;  // PX reads every (A) PRUNE word: start from zeros
    e->gp = *p;
    return GSX_OK;
}

namespace {
// The gossip exchange's per-pair state, allocated when it is first enabled:
// IHAVE counters, the promises (prom_slots per pair), the receiver-side IHAVE
// topic bits (and truncated ones), the error / occupancy words.
// The round's touch bits (HbState::gx_touch) after the 8 flag words of d_gxflag.
size_t gx_touch_words(const gsx_engine* e) { return ((size_t)e->n_nodes + 63) / 64; }
int gx_alloc(gsx_engine* e) {
    if (e->d_prom_e) return GSX_OK;
    int rc = 0;
    const size_t E = std::max<size_t>(e->E, 1);
    const uint32_t S = gsx::GX_PROMISE_SLOTS0;
    if ((rc = dalloc(e, &e->d_gxreq, E)) ||
        (rc = dalloc(e, &e->d_prom_h, E * S)) || (rc = dalloc(e, &e->d_prom_e, E * S)) ||
        (rc = dalloc(e, &e->d_prom_any, E)) || (rc = dalloc(e, &e->d_prom_cnt, 1)) ||
        (rc = dalloc(e, &e->d_ihave_bits, 2 * E)) ||
        (rc = dalloc(e, &e->d_gxflag, 8 + 2 * gx_touch_words(e))) ||
        (rc = dalloc(e, &e->d_gx_nodes, std::max<size_t>(e->n_nodes, 1))) ||
        (rc = dalloc(e, &e->d_sub_cnt, std::max<size_t>(e->T, 1))) ||
        (rc = dalloc(e, &e->d_gsubs, std::max<size_t>(e->T, 1))))
        return rc;
    e->prom_slots = S;
    HIPCHK(e, hipMemsetAsync(e->d_prom_e, 0, 8 * E * S, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_prom_any, 0, E, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_gxreq, 0, 4 * E, e->stream));
    e->subp.assign(e->T, gsx_engine::SubPool{});
    e->gsub_host.assign(e->T, gsx::GxSub{});
    return GSX_OK;
}

// Doubles the promise slots of every pair (kept promises stay in order).
int gx_prom_grow(gsx_engine* e) {
    const size_t E = std::max<size_t>(e->E, 1);
    const uint32_t S = e->prom_slots, S2 = 2 * S;
    uint64_t* nh = nullptr;
    int64_t* ne = nullptr;
    if (int rc = dalloc(e, &nh, E * S2)) return rc;
    if (int rc = dalloc(e, &ne, E * S2)) {
        (void)hipFree(nh);
        return rc;
    }
    HIPCHK(e, gsx::launch_gx_prom_grow(e->d_prom_h, e->d_prom_e, S, nh, ne, S2, E, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    (void)hipFree(e->d_prom_h);
    (void)hipFree(e->d_prom_e);
    e->d_prom_h = nh;
    e->d_prom_e = ne;
    e->prom_slots = S2;
    return GSX_OK;
}

// The rows of this round's truncated IHAVE lists: a topic whose gossip window
// can exceed MaxIHaveLength gets rows for every target the round can pick
// (the sum over nodes of min(degree, max(Dlazy, GossipFactor * degree)): a
// node picks at most that many from its eligible peers), tw words each.
void gx_target_bound(gsx_engine* e) {
    if (e->tgt_dlazy != e->gp.d_lazy || e->tgt_gf != e->gp.gossip_factor) {
        uint64_t b = 0;
        for (uint32_t v = 0; v < e->n_nodes; ++v) {
            const int64_t deg = e->row_ptr[v + 1] - e->row_ptr[v];
            int64_t tg = e->gp.d_lazy;
            const int64_t f = (int64_t)(e->gp.gossip_factor * (double)deg);
            if (f > tg) tg = f;
            b += (uint64_t)std::min<int64_t>(tg, deg);
        }
        e->tgt_bound = b * (e->members_on ? 2 : 1);  // (a fanout pass gossips too)
        e->tgt_dlazy = e->gp.d_lazy;
        e->tgt_gf = e->gp.gossip_factor;
    }
}
int gx_sub_prepare(gsx_engine* e, const std::vector<uint32_t>& max_ids, const std::vector<uint32_t>& tw) {
    gx_target_bound(e);
    const size_t E = std::max<size_t>(e->E, 1);
    for (uint32_t t = 0; t < e->T; ++t) {
        gsx::GxSub& g = e->gsub_host[t];
        g = gsx::GxSub{};
        if (max_ids[t] <= (uint32_t)std::max(e->gp.max_ihave_length, 0) || e->tgt_bound == 0) continue;
        gsx_engine::SubPool& sp = e->subp[t];
        if (sp.rows < e->tgt_bound || sp.tw < tw[t]) {
            // (doubled at least: the advertised windows widen over a run's first
            // rounds, and a multi-GB free + malloc stalls the round)
            const size_t tw_a = std::max<size_t>(std::max<size_t>(tw[t], 2 * sp.tw), 64);
            if (sp.pool) (void)hipFree(sp.pool);
            sp.pool = nullptr;
            sp.rows = sp.tw = 0;
            if (int rc = dalloc(e, &sp.pool, (size_t)e->tgt_bound * tw_a)) return rc;
            sp.rows = e->tgt_bound;
            sp.tw = tw_a;
        }
        if (!sp.idx)
            if (int rc = dalloc(e, &sp.idx, E)) return rc;
        g.pool = sp.pool;
        g.idx = sp.idx;
        g.cnt = e->d_sub_cnt + t;
        g.tw = tw[t];
        g.cap = (uint32_t)std::min<size_t>(sp.rows, 0xFFFFFFFFu);
    }
    HIPCHK(e, hipMemsetAsync(e->d_sub_cnt, 0, 4 * std::max<size_t>(e->T, 1), e->stream));
    HIPCHK(e, hipMemcpyAsync(e->d_gsubs, e->gsub_host.data(), sizeof(gsx::GxSub) * e->T, hipMemcpyHostToDevice,
                             e->stream));
    return GSX_OK;
}

// The heartbeat round in three steps, so that a range shard can exchange the
// control words of its cross-shard pairs between them (gsx.h):
//   hb_begin  (A) maintenance + emitGossip of every (node, topic), GRAFT/PRUNE bits per pair;
//   hb_recv   (B) handleGraft / handlePrune at the receivers (remote senders' bits from halo_ctl);
//   hb_end    (C) the senders handle the PRUNE answers (remote answers from halo_resp), counters,
//             mcache.Shift.
// state_only: the round's buffers and kernel state (e->hb) without
// maintenance, gossip or the promise penalties (Join / Leave use it)
static int dbg_sync_mask() {
    static int m = -1;
    if (m < 0) {
        const char* s = getenv("GSX_DBG_SYNC");
        m = s ? atoi(s) : 0;
    }
    return m;
}
#define DBG_SYNC(bit) \
    if (dbg_sync_mask() & (bit)) HIPCHK(e, hipStreamSynchronize(e->stream))
// GSX_DBG_HOST: host microseconds between checkpoints of a heartbeat (stderr)
static void dbg_host(const char* what) {
    static const bool on = getenv("GSX_DBG_HOST") != nullptr;
    if (!on) return;
    static auto last = std::chrono::steady_clock::now();
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[host] %-14s %8.1f us\n", what,
            std::chrono::duration<double, std::micro>(now - last).count());
    last = now;
}
int hb_begin_state(gsx_engine* e, uint64_t tick, int64_t now, uint64_t seed, bool state_only) {
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (int rc = fold_deferred(e)) return rc;  // (the round reads every record)
    DBG_SYNC(1);
    dbg_host("hb start");
    e->state_changed();
    if (e->sharded() && (e->n_ranks > 1 ? !e->d_send_pair : true))
        return fail(e, GSX_ESTATE, "heartbeat on a range shard needs its shard plan (gsx_shard_*_plan)");
    if (e->max_deg > gsx::HB_HUB_MAX)
        return fail(e, GSX_ERANGE, "heartbeat supports at most " + std::to_string(gsx::HB_HUB_MAX) + " peers per node");
    if (!e->d_hbstats)
        if (int rc = hb_alloc(e)) return rc;
    const bool gx_on = e->gp.gossip_exchange != 0;
    if (gx_on && e->sharded() && e->n_ranks > 1 && !e->d_dest_halo_base)
        return fail(e, GSX_ESTATE, "gossip exchange on a shard: gsx_shard_set_halo_bases first");
    if (gx_on)
        if (int rc = gx_alloc(e)) return rc;
    ZeroBatch za(e);
    if (int rc = za.add(e->d_hbstats, sizeof(unsigned long long) * gsx::HB_STAT_WORDS)) return rc;
    uint8_t* pen_mask = nullptr;
    if (e->d_prom_e && !state_only) {
        // clearIHaveCounters (:1566-1576): nothing to clear, the exchange's gate
        // reads the counters' values at a heartbeat's one RPC per pair (gx_gate);
        // applyIwantPenalties (:1578-1583): promises expired before now are
        // broken, AddPenalty (P7) on their pairs
        const size_t E = std::max<size_t>(e->E, 1);
        pen_mask = e->d_dirty + 3 * e->E;
        if (int rc = za.add(pen_mask, E)) return rc;
        if (int rc = za.flush()) return rc;
        gsx::HbState hp{};
        hp.n_pairs = e->E;
        hp.now = now;
        hp.prom_h = e->d_prom_h;
        hp.prom_e = e->d_prom_e;
        hp.prom_any = e->d_prom_any;
        hp.prom_slots = e->prom_slots;
        hp.stats = e->d_hbstats;
        hp.dirty = pen_mask;
        HIPCHK(e, gsx::launch_gx_promises(dev_state(e), hp, e->stream));
    }
    if (int rc = za.flush()) return rc;
    // the scores of the heartbeat start (gossipsub.go:1333-1341)
    if (int rc = ensure_scores(e)) return rc;
    // (pen_mask holds exactly the pairs of the broken promises k_gx_promises counted)
    if (pen_mask)
        HIPCHK(e, rescore_subset(e, dev_state(e), kern_params(e), pen_mask, nullptr,
                                 e->d_hbstats + gsx::HB_BROKEN_PROMISES));
    gsx::HbState h{};
    h.row_ptr = e->d_row_ptr;
    h.rev = e->d_rev;
    h.eflags = e->d_eflags;
    h.backoff = e->d_backoff;
    h.bo8 = e->d_bo8;
    h.ctl = e->d_ctl;
    h.resp = e->d_resp;
    h.dirty = e->d_dirty;
    h.inbox = e->d_dirty + e->E;
    h.answer = e->d_dirty + 2 * e->E;
    h.long_nodes = e->d_long;
    h.n_long = e->d_nlong;
    h.stats = e->d_hbstats;
    h.n_pairs = e->E;
    h.n_nodes = e->n_nodes;
    h.node_lo = e->node_lo;
    h.tick = tick;
    h.now = now;
    h.seed = seed;
    h.og_threshold = e->th.opportunistic_graft_threshold;
    h.graylist = e->th.graylist_threshold;
    h.gossip_threshold = e->th.gossip_threshold;
    h.rngk = e->d_rngk;
    h.work = e->d_work;
    h.tcnt = e->d_tcnt;
    h.mcount = e->d_mcount;
    h.publish_threshold = e->th.publish_threshold;
    h.col = e->d_col;  // (the truncated lists' draw streams are keyed by the peer)
    member_fill(e, h);
    if (e->hb_tracing) {
        if (!e->d_tr_acc) {
            if (int rc = dalloc(e, &e->d_tr_acc, std::max<size_t>(e->E, 1))) return rc;
            if (int rc = dalloc(e, &e->d_tr_hp, std::max<size_t>(e->E, 1))) return rc;
        }
        if (int rc = za.add(e->d_tr_acc, 8 * std::max<size_t>(e->E, 1))) return rc;
        if (int rc = za.add(e->d_tr_hp, 8 * std::max<size_t>(e->E, 1))) return rc;
        h.tr_acc = e->d_tr_acc;
        h.tr_hp = e->d_tr_hp;
        h.keep_ctl = true;
    }
    h.n_tiles64 = 64 * (((uint64_t)e->n_nodes + 63) / 64);
    h.hub_work = e->d_hubwork;
    h.n_hub = e->d_nwork + e->T;
    h.hubs = e->d_hubs;
    h.n_hubs = (uint32_t)e->hubs_host.size();
    h.pp = dev_peer_params(e);
    h.gp = gsx::DevGossipParams{e->gp.d,
                                e->gp.d_lo,
                                e->gp.d_hi,
                                e->gp.d_score,
                                e->gp.d_out,
                                e->gp.opportunistic_graft_peers,
                                e->gp.opportunistic_graft_ticks,
                                e->gp.prune_backoff_ns,
                                e->gp.graft_flood_threshold_ns,
                                e->gp.d_lazy,
                                e->gp.max_ihave_length,
                                e->gp.gossip_factor,
                                e->gp.max_ihave_messages,
                                e->gp.gossip_retransmission,
                                e->gp.iwant_followup_ns,
                                e->gp.fanout_ttl_ns,
                                e->gp.do_px,
                                e->gp.prune_peers};
    const gsx::DevState ds = dev_state(e);
    if (int rc = za.add(e->d_nwork, 8 * (size_t)e->T)) return rc;
    // (per topic and gossip pass, mesh then fanout: k_hb_gossip's long-list counts)
    if (int rc = za.add(e->d_nlong, 8 * (size_t)e->T)) return rc;
    if (gx_on) {
        h.ihave_bits = e->d_ihave_bits;
        h.ihave_tr = e->d_ihave_bits + std::max<size_t>(e->E, 1);
        h.gx_err = e->d_gxflag;
        h.gx_nodes = e->d_gx_nodes;
        h.prom_occ = e->d_gxflag + 4;
        h.gx_req = e->d_gxreq;
        h.prom_h = e->d_prom_h;
        h.prom_e = e->d_prom_e;
        h.prom_any = e->d_prom_any;
        h.prom_slots = e->prom_slots;
        h.gsubs = e->d_gsubs;
        // the IHAVE topic bits of the last round (one bulk clear: cheaper than the
        // exchange clearing the pairs it read one by one)
        // (the truncated-list bits only after a round that could set them: gx_sub_prepare)
        if (int rc = za.add(e->d_ihave_bits, (e->ihave_tr_dirty ? 16 : 8) * std::max<size_t>(e->E, 1))) return rc;
        if (int rc = za.add(e->d_gxflag, 32 + 8 * gx_touch_words(e))) return rc;  // flags, touch bits
        h.gx_touch = reinterpret_cast<uint64_t*>(e->d_gxflag + 8);
        if (e->sharded()) {  // the IHAVEs of cross-shard pairs, sender side (gsx_gx_pack_ihave)
            const size_t E = std::max<size_t>(e->E, 1);
            if (!e->d_gxs_out) {
                int rc = 0;
                if ((rc = dalloc(e, &e->d_gxs_out, 2 * E)) || (rc = dalloc(e, &e->d_gxs_rans, E)) ||
                    (rc = dalloc(e, &e->d_gxs_hidx, E)) || (rc = dalloc(e, &e->d_gxs_cnt, (size_t)gsx::MAX_RANKS)) ||
                    (rc = dalloc(e, &e->d_gxs_off, (size_t)gsx::MAX_RANKS)))
                    return rc;
            }
            if (int rc = za.add(e->d_gxs_out, 16 * E)) return rc;  // gxs_out, gxs_tro
            h.gxs_out = e->d_gxs_out;
            h.gxs_tro = e->d_gxs_out + E;
            h.gxs_rans = e->d_gxs_rans;
            h.gxs_hidx = e->d_gxs_hidx;
        }
    }
    if (e->gp.do_px) {  // peer exchange on the round's PRUNEs (gsx.h; heartbeats and Join / Leave rounds)
        if (e->sharded() && e->n_ranks > 1 && !e->d_dest_halo_base)
            return fail(e, GSX_ESTATE, "peer exchange on a shard: gsx_shard_set_halo_bases first");
        const size_t E = std::max<size_t>(e->E, 1);
        if (!e->d_pxno)
            if (int rc = dalloc(e, &e->d_pxno, E)) return rc;
        if (!e->members_on && !e->d_pxscratch)
            if (int rc = dalloc(e, &e->d_pxscratch, E)) return rc;
        if (!e->d_pxbase)
            if (int rc = dalloc(e, &e->d_pxbase, E)) return rc;
        if (e->px_cap > e->pxlog_alloc) {
            if (e->d_pxlog) (void)hipFree(e->d_pxlog);
            e->d_pxlog = nullptr;
            e->pxlog_alloc = 0;
            if (int rc = dalloc(e, &e->d_pxlog, 4 * e->px_cap)) return rc;
            e->pxlog_alloc = e->px_cap;
        }
        if (int rc = za.add(e->d_pxno, E)) return rc;
        h.pxno = e->d_pxno;
        h.px_log = e->px_cap ? e->d_pxlog : nullptr;
        h.px_cap = e->px_cap;
        h.accept_px = e->th.accept_px_threshold;
        h.col = e->d_col;
        if (!e->members_on) h.mscratch = e->d_pxscratch;
        h.pxbase = e->d_pxbase;
        if (e->sharded()) {  // PX lists of cross-shard PRUNEs travel (gsx_hb_px_*)
            if (!e->d_pxs_cnt) {
                if (int rc = dalloc(e, &e->d_pxs_cnt, (size_t)gsx::MAX_RANKS)) return rc;
                if (int rc = dalloc(e, &e->d_pxs_off, (size_t)gsx::MAX_RANKS)) return rc;
            }
            h.send_slot = e->d_send_slot;
            h.send_dest = e->d_send_dest;
            h.send_base = e->d_send_base;
            h.dest_halo_base = e->d_dest_halo_base;
            h.halo_pair = e->d_halo_pair;
            h.pair_obs = e->d_pair_obs;
            h.pxs_cnt = e->d_pxs_cnt;
            h.pxs_off = e->d_pxs_off;
            h.pxs_w = 3u + (uint32_t)std::max(e->gp.prune_peers, 0);
        }
    }
    e->pxs_packed[0] = e->pxs_packed[1] = false;
    const size_t E8 = 8 * (e->E ? e->E : 1);
    // Unsharded, (B) and (C) clear the control words, answers and marks they
    // read, and nothing else is ever set: after one cleared round they stay
    // clean.  Shards pack them for the exchange and clear them here.
    if (e->sharded() || !e->hb_clean) {
        if (int rc = za.add(e->d_ctl, 2 * E8)) return rc;
        if (int rc = za.add(e->d_resp, E8)) return rc;
        if (int rc = za.add(e->d_dirty, 3 * (e->E ? e->E : 1))) return rc;
    } else {
        if (int rc = za.add(e->d_dirty, e->E ? e->E : 1)) return rc;
    }
    if (int rc = za.flush()) return rc;
    e->hb_clean = false;  // until this round's (C) has run
    if (state_only) {
        e->hb = h;
        return GSX_OK;
    }
    dbg_host("hb memsets");
    if (tick % 15 == 0) HIPCHK(e, gsx::launch_hb_clear_backoff(h, e->T, e->stream));  // :1585-1604
    // GetGossipIDs inputs: per topic, the batches of windows [0, HistoryGossip) in order.
    // Cache slots are word-aligned: message k of a batch is slot 64 * (the
    // batch's first word over all topics) + k, and bit (row_off * 64 + k) of
    // the topic's gossip rows (the truncated lists' layout, GxSub)
    e->gb_host.clear();
    e->mc_digest_host.clear();
    std::vector<uint32_t> gb_off(e->T + 1, 0), max_ids(e->T, 0), tw(e->T, 0);
    std::vector<uint64_t> wdig;  // per batch word: the digest sum of all its messages (a full word's digest)
    const size_t n_win = std::min<size_t>((size_t)std::max(e->gp.history_gossip, 0), e->mc.size());
    for (uint32_t t = 0; t < e->T; ++t) {
        gb_off[t] = (uint32_t)e->gb_host.size();
        for (size_t w = 0; w < n_win; ++w)
            for (const auto& b : e->mc[w]) {
                if (b.topic != t) continue;
                e->gb_host.push_back(gsx::GossipBatch{b.d_seen, b.d_dig, b.d_cnt, b.n_words,
                                                      (uint32_t)e->mc_digest_host.size(), (uint32_t)wdig.size(),
                                                      b.n_msgs, tw[t]});
                for (size_t k = 0; k < (size_t)b.n_words * 64; ++k) {
                    const uint64_t d = k < b.ids.size() ? id_digest(b.ids[k]) : 0;
                    e->mc_digest_host.push_back(d);
                    if (k % 64 == 0) wdig.push_back(0);
                    wdig.back() += d;
                }
                max_ids[t] += b.n_msgs;
                tw[t] += b.n_words;
            }
        if (tw[t] > gsx::HB_GOSSIP_MAX_WORDS)
            return fail(e, GSX_ERANGE, "gossip window of topic " + std::to_string(t) + " spans " +
                                           std::to_string(tw[t]) + " words, more than " +
                                           std::to_string(gsx::HB_GOSSIP_MAX_WORDS) + " (shift the cache more often)");
    }
    gb_off[e->T] = (uint32_t)e->gb_host.size();
    for (auto& g : e->gb_host) g.wdig_base += (uint32_t)e->mc_digest_host.size();  // word digests follow the slots
    e->mc_digest_host.insert(e->mc_digest_host.end(), wdig.begin(), wdig.end());
    if (e->gb_host.size() > e->gb_cap) {
        if (e->d_gb) (void)hipFree(e->d_gb);
        e->d_gb = nullptr;
        e->gb_cap = std::max<size_t>(e->gb_host.size(), 2 * e->gb_cap);
        if (int rc = dalloc(e, &e->d_gb, e->gb_cap)) return rc;
    }
    if (e->mc_digest_host.size() > e->ids_cap) {
        if (e->d_mc_digest) (void)hipFree(e->d_mc_digest);
        e->d_mc_digest = nullptr;
        e->ids_cap = std::max<size_t>(e->mc_digest_host.size(), 2 * e->ids_cap);
        if (int rc = dalloc(e, &e->d_mc_digest, e->ids_cap)) return rc;
    }
    if (!e->gb_host.empty()) {
        HIPCHK(e, hipMemcpyAsync(e->d_gb, e->gb_host.data(), sizeof(gsx::GossipBatch) * e->gb_host.size(),
                                 hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->d_mc_digest, e->mc_digest_host.data(), 8 * e->mc_digest_host.size(),
                                 hipMemcpyHostToDevice, e->stream));
    }
    h.mc_digest = e->d_mc_digest;
    dbg_host("hb gb lists");
    DBG_SYNC(2);
    // the truncated IHAVE lists' rows (exchange on, a window longer than MaxIHaveLength)
    if (gx_on) {
        if (int rc = gx_sub_prepare(e, max_ids, tw)) return rc;
        bool pool = false;  // (only a topic with rows can truncate a list: k_hb_gossip_long sets ihave_tr)
        for (uint32_t t = 0; t < e->T; ++t) pool = pool || e->gsub_host[t].pool != nullptr;
        e->ihave_tr_dirty = pool;
    }
    // IHAVE slots: this round's are written under its tag (k_hb_gossip); every
    // other slot reads as empty, so nothing is cleared (but at the tag's wrap)
    if (++e->ihave_round == 0) {
        HIPCHK(e, hipMemsetAsync(e->d_ihave_slot, 0, sizeof(gsx::IhaveSlot) * (size_t)e->T * e->E, e->stream));
        e->ihave_round = 1;
    }
    // the targets' byte tags cycle 1..IHAVE_TAG_MAX: a stale byte equal to this
    // round's can only be 127 rounds old, so the array is cleared as the cycle restarts
    const uint32_t cur8 = (e->ihave_round - 1) % gsx::IHAVE_TAG_MAX + 1;
    if (cur8 == 1 && e->ihave_round > 1)
        HIPCHK(e, hipMemsetAsync(e->d_ihave_tag, 0, (size_t)e->T * e->E, e->stream));
    h.ihave_slot = e->d_ihave_slot;
    h.ihave_unit = e->d_ihave_unit;
    h.ihave_tag = e->d_ihave_tag;
    h.ihave_cur = e->ihave_round;
    h.ihave_cur8 = cur8;
    h.gelig = e->d_gelig;
    e->have_gossip = !e->gb_host.empty();
    // (A) the scan of every unit, then per topic, ascending: maintenance, then
    // emitGossip.  A unit changes only its own topic's records, backoff entries
    // and control bits, so the maintenance of a run of topics is one launch; a
    // topic's gossip reads the live scores maintenance left (gossipsub.go:1514), so it goes
    // after its own topic's run and before the next
    dbg_host("hb sub/ihave");
    if (e->have_gossip) HIPCHK(e, gsx::launch_hb_gelig(ds, h, e->stream));  // (emitGossip's per-pair byte)
    HIPCHK(e, gsx::launch_hb_scan(ds, h, e->stream));
    for (uint32_t t = 0, tb = 0; t < e->T; ++t) {
        const bool g = gb_off[t + 1] > gb_off[t] && max_ids[t] > 0;
        if (!g && t + 1 < e->T) continue;
        HIPCHK(e, gsx::launch_hb_maintain(ds, h, tb, t + 1 - tb, e->max_deg, e->stream));
        tb = t + 1;
        gsx::HbState ht = h;
        ht.n_long = e->d_nlong + t;
        if (gx_on) ht.gsub = e->gsub_host[t];
        DBG_SYNC(4);
        HIPCHK(e, gsx::launch_hb_gossip(ds, ht, t, e->d_gb + gb_off[t], gb_off[t + 1] - gb_off[t],
                                        max_ids[t] ? tw[t] : 0, e->max_deg, e->stream));
    }
    if (e->members_on) {  // the fanout of topics published to but not joined (:1517-1554)
        for (uint32_t t = 0; t < e->T; ++t) {
            HIPCHK(e, gsx::launch_hb_fanout(ds, h, t, e->stream));
            gsx::HbState hf = h;
            hf.fan_mode = 1;
            hf.n_long = e->d_nlong + e->T + t;
            if (gx_on) hf.gsub = e->gsub_host[t];
            HIPCHK(e, gsx::launch_hb_gossip(ds, hf, t, e->d_gb + gb_off[t], gb_off[t + 1] - gb_off[t],
                                            max_ids[t] ? tw[t] : 0, e->max_deg, e->stream));
        }
        ++e->mem_gen;
    }
    // the receivers score the senders as the round left them: the pairs (A)
    // touched that (B) reads (marked in the inbox) are re-scored
    // (a shard's (B) reads every pair with remote control: all touched pairs)
    // (with PX every touched pair: the PX lists read the owner's whole row)
    HIPCHK(e, rescore_subset(e, ds, kern_params(e), h.dirty, (!e->sharded() && !h.pxno) ? h.inbox : nullptr,
                             hb_ctl_gate(e)));
    e->hb = h;
    e->hb_active = true;
    dbg_host("hb (A) queued");
    return GSX_OK;
}

int hb_begin(gsx_engine* e, uint64_t tick, int64_t now, uint64_t seed) {
    return hb_begin_state(e, tick, now, seed, false);
}

int hb_recv(gsx_engine* e, const uint64_t* halo_ctl) {
    e->state_changed();
    gsx::HbState h = e->hb;
    h.halo_ctl = halo_ctl;
    const gsx::DevState ds = dev_state(e);
    if (h.pxno && e->sharded() && !e->pxs_packed[0])
        return fail(e, GSX_ESTATE, "peer exchange on a shard: gsx_hb_px_pack(0) before gsx_hb_recv");
    if (!e->sharded()) HIPCHK(e, gsx::launch_hb_px(ds, h, 0, e->stream));  // the (A) PRUNEs' peer exchange (do_px)
    HIPCHK(e, gsx::launch_hb_recv(ds, h, e->stream));
    // the pairs touched so far that (C) reads: those marked with an answer
    // (a shard's (C) reads every pair with a remote answer: all touched pairs;
    // with PX every touched pair: the answers' PX lists read the whole row)
    HIPCHK(e, rescore_subset(e, ds, kern_params(e), h.dirty, (!e->sharded() && !h.pxno) ? h.answer : nullptr,
                             hb_ctl_gate(e)));
    return GSX_OK;
}

// The forwarding of recovered messages (gsx.h (D), GxFwd): state allocated on
// first use; the hop stamps only grow (re-zeroed before they could wrap).
// The receiver-side slot pass (fin): range shards (the remote senders' slots
// arrive as fin bits); one engine gathers fout[rev q] for the senders in the
// frontier instead, in the pull or in the eligible-sender lists the first
// dense hop builds (GSX_GXF_FIN=1: the pass on one engine too, A/B).
bool gxf_fin_pass(const gsx_engine* e) {
    static const bool env = getenv("GSX_GXF_FIN") != nullptr;
    return e->sharded() || env;
}

int gxf_alloc(gsx_engine* e) {
    const size_t n_grp = std::max<size_t>({e->gxr.grp_topic.size(), (size_t)e->T, 1});
    if (e->d_gxf_b0 && n_grp > e->gxf_b0_grps) {  // more set groups than topics this round
        HIPCHK(e, hipStreamSynchronize(e->stream));
        (void)hipFree(e->d_gxf_b0);
        e->d_gxf_b0 = nullptr;
        const size_t grps = std::max(n_grp, 2 * e->gxf_b0_grps);
        e->gxf_b0_grps = 0;  // (a failed allocation leaves none: the next call retries)
        if (int rc = dalloc(e, &e->d_gxf_b0, grps * std::max<size_t>(e->E, 1))) return rc;
        e->gxf_b0_grps = grps;
        HIPCHK(e, hipMemsetAsync(e->d_gxf_bst, 0, 4 * std::max<size_t>(e->E, 1), e->stream));  // (bst0: no stale stamps)
    }
    if (e->d_gxf_bst && !e->d_gxf_b0) {  // a regrowth failed before: allocate the group counts again
        e->gxf_b0_grps = std::max<size_t>(n_grp, 1);
        if (int rc = dalloc(e, &e->d_gxf_b0, e->gxf_b0_grps * std::max<size_t>(e->E, 1))) {
            e->gxf_b0_grps = 0;
            return rc;
        }
        HIPCHK(e, hipMemsetAsync(e->d_gxf_bst, 0, 4 * std::max<size_t>(e->E, 1), e->stream));
    }
    if (gxf_fin_pass(e) && !e->d_gxf_fin)
        if (int rc = dalloc(e, &e->d_gxf_fin, std::max<size_t>(e->E, 1))) return rc;
    if (e->d_gxf_bst) {
        if (e->gxf_stamp < 0xF0000000u) return GSX_OK;
        HIPCHK(e, hipMemsetAsync(e->d_gxf_bst, 0, 4 * 3 * std::max<size_t>(e->E, 1), e->stream));
        if (e->d_gxf_hst) HIPCHK(e, hipMemsetAsync(e->d_gxf_hst, 0, 4 * 2 * std::max<size_t>(e->E, 1), e->stream));
        e->gxf_stamp = 0;
        return GSX_OK;
    }
    const size_t N = std::max<size_t>(e->n_nodes, 1), E = std::max<size_t>(e->E, 1);
    int rc = 0;
    if ((rc = dalloc(e, &e->d_gxf_mask, 4 * N + 2 * ((N + 63) / 64))) || (rc = dalloc(e, &e->d_gxf_list, 3 * N)) ||
        (rc = dalloc(e, &e->d_gxf_cnt, 2 * ((size_t)gsx::GXF_MAX_HOPS + 1))) || (rc = dalloc(e, &e->d_gxf_bst, 3 * E)) ||
        (rc = dalloc(e, &e->d_gxf_b0, n_grp * E)) ||
        (rc = dalloc(e, &e->d_gxf_b, 2 * E * gsx::GXF_SLOTS)) || (rc = dalloc(e, &e->d_gxf_fout, E)) ||
        (rc = dalloc(e, &e->d_gxf_fent, E)) || (rc = dalloc(e, &e->d_gxf_fend, N)))
        return rc;

    e->gxf_b0_grps = n_grp;
    if (e->sharded() && (rc = dalloc(e, &e->d_gxf_hst, 2 * E))) return rc;
    if (e->d_gxf_hst) HIPCHK(e, hipMemsetAsync(e->d_gxf_hst, 0, 4 * 2 * E, e->stream));
    if (!e->h_gxf_cnt) HIPCHK(e, hipHostMalloc((void**)&e->h_gxf_cnt, 64, hipHostMallocDefault));
    HIPCHK(e, hipMemsetAsync(e->d_gxf_bst, 0, 4 * 3 * E, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_gxf_mask + 2 * N, 0, 8 * N, e->stream));  // rmask: kept clear by the pulls
    e->gxf_stamp = 0;
    return GSX_OK;
}

// The forwarding runs over the exchange's sets: up to 64 sets in up to
// GXF_SLOTS set groups each (a group: up to 64 sets / 65,535 messages of one
// topic, gx_prepare; the IWANT back counts are per group), greedily in order.
int gxf_plan(gsx_engine* e, gsx_engine::GxRound& R) {
    R.runs.clear();
    const uint32_t G = (uint32_t)R.grp_topic.size();
    std::vector<std::vector<size_t>> by_grp(G);
    for (size_t i = 0; i < R.sets.size(); ++i) by_grp[R.set_grp[i]].push_back(i);
    size_t n_sets = 0;
    for (uint32_t g = 0; g < G; ++g) {  // (groups are in the sets' order: topics first seen first)
        if (R.runs.empty() || R.runs.back().grps.size() == gsx::GXF_SLOTS || n_sets + by_grp[g].size() > 64) {
            R.runs.emplace_back();
            n_sets = 0;
        }
        R.runs.back().grps.push_back(g);
        for (size_t i : by_grp[g]) R.runs.back().sets.push_back(i);
        n_sets += by_grp[g].size();
    }
    return GSX_OK;
}

// Sets up run k (descriptors, frontier rows, cleared masks and counts) and
// launches its hop 0 (the recovering nodes' accepted receipts) and the
// per-pair forwarding slots.
int gxf_run_begin(gsx_engine* e, gsx_engine::GxRound& R, size_t k) {
    const size_t N = e->n_nodes;
    const auto& run = R.runs[k];
    const size_t ns = run.sets.size();
    if (ns > e->gxf_sets_cap) {
        if (e->d_gxf_sets) (void)hipFree(e->d_gxf_sets);
        e->d_gxf_sets = nullptr;
        e->gxf_sets_cap = std::max<size_t>(std::max<size_t>(ns, 2 * e->gxf_sets_cap), 64);
        if (int rc = dalloc(e, &e->d_gxf_sets, e->gxf_sets_cap)) return rc;
    }
    const size_t stage_bytes = sizeof(gsx::GxFwdSet) * 64;
    // the staging buffer of the run before: its copy done (not the whole
    // stream: the host keeps queueing the run behind the round's kernels)
    if (e->gxf_stage_queued) HIPCHK(e, hipEventSynchronize(e->ev_gxf_stage));
    e->gxf_stage_queued = false;
    if (e->h_gxf_stage_bytes < stage_bytes) {
        if (e->h_gxf_stage) (void)hipHostFree(e->h_gxf_stage);
        e->h_gxf_stage = nullptr;
        e->h_gxf_stage_bytes = 0;
        HIPCHK(e, hipHostMalloc(&e->h_gxf_stage, stage_bytes, hipHostMallocDefault));
        e->h_gxf_stage_bytes = stage_bytes;
    }
    auto* stage = static_cast<gsx::GxFwdSet*>(e->h_gxf_stage);
    gsx::GxFwd f{};
    f.sets = e->d_gxf_sets;
    f.n_slots = (uint32_t)run.grps.size();
    uint32_t n_src = 0, rw = 0;
    for (size_t ts = 0; ts < run.grps.size(); ++ts) {
        const uint32_t t = R.grp_topic[run.grps[ts]];
        f.slot_topic[ts] = t;
        f.slot_grp[ts] = run.grps[ts];
        for (size_t i : run.sets) {
            const gsx_engine::MsgSet* ms = R.sets[i];
            if (R.set_grp[i] != run.grps[ts]) continue;
            const size_t words = (size_t)ms->n_words * N;
            gsx::GxFwdSet S{};
            S.all = ms->d_all;
            S.x = R.xs[i];
            S.acc = ms->d_acc;
            S.src = ms->d_src;
            for (int z = 0; z < 2; ++z) {
                S.fr[z] = seen_acquire(e, std::max<size_t>(words, 1));
                if (!S.fr[z]) return fail(e, GSX_ENOMEM, "forwarding frontier rows");
                R.scratch.emplace_back(S.fr[z], std::max<size_t>(words, 1));
            }
            S.n_words = ms->n_words;
            S.n_msgs = ms->n_msgs;
            S.topic = t;
            S.slot = (uint32_t)ts;
            S.serial = ms->serial;
            S.woff = rw;
            S.got = e->d_gx_got + i;
            rw += ms->n_words;
            // an old copy: inside the window by its code's validation time (gsx.h (D))
            S.old_in = R.old_in[i];
            S.vc = R.vc[i];
            if (S.old_in == 2) f.mixed = 1;
            f.slot_sets[ts] |= 1ull << f.n_sets;
            stage[f.n_sets] = S;
            ++f.n_sets;
            n_src += ms->n_msgs;
        }
    }
    f.rw = rw;
    HIPCHK(e, hipMemcpyAsync(e->d_gxf_sets, stage, sizeof(gsx::GxFwdSet) * f.n_sets, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipEventRecord(e->ev_gxf_stage, e->stream));
    e->gxf_stage_queued = true;
    f.fmask[0] = e->d_gxf_mask;
    f.fmask[1] = e->d_gxf_mask + N;
    f.rmask = e->d_gxf_mask + 2 * N;
    f.srcm = e->d_gxf_mask + 3 * N;
    f.fbit[0] = e->d_gxf_mask + 4 * N;
    f.fbit[1] = f.fbit[0] + (N + 63) / 64;
    f.flist[0] = e->d_gxf_list;
    f.flist[1] = e->d_gxf_list + N;
    f.rlist = e->d_gxf_list + 2 * N;
    f.fcnt = e->d_gxf_cnt;
    f.rcnt = e->d_gxf_cnt + gsx::GXF_MAX_HOPS + 1;
    const size_t E = std::max<size_t>(e->E, 1);
    f.bst0 = e->d_gxf_bst;
    f.bcnt0 = e->d_gxf_b0;
    f.stamp0 = R.h.gxb_stamp;
    f.bst[0] = e->d_gxf_bst + E;
    f.bst[1] = e->d_gxf_bst + 2 * E;
    f.bcnt[0] = e->d_gxf_b;
    f.bcnt[1] = e->d_gxf_b + E * gsx::GXF_SLOTS;
    f.seq = e->gxf_stamp + 1;
    f.fout = e->d_gxf_fout;
    f.fin = gxf_fin_pass(e) ? e->d_gxf_fin : nullptr;
    static const bool no_compact = getenv("GSX_GXF_NO_COMPACT") != nullptr;  // (A/B)
    if (!no_compact) {
        f.fent = e->d_gxf_fent;
        f.fend = e->d_gxf_fend;
    }
    f.all_sets = f.n_sets >= 64 ? ~0ull : ((1ull << f.n_sets) - 1);
    static const uint32_t fout_div = [] {  // (GSX_GXF_FOUT_DIV: A/B of the fout pass's threshold)
        const char* v = getenv("GSX_GXF_FOUT_DIV");
        return v && atoi(v) > 0 ? (uint32_t)atoi(v) : gsx::GXF_FOUT_DIV;
    }();
    static const uint32_t dense_div = [] {  // (GSX_GXF_DENSE: A/B of the dense-hop threshold)
        const char* v = getenv("GSX_GXF_DENSE");
        return v && atoi(v) > 0 ? (uint32_t)atoi(v) : gsx::GXF_DENSE;
    }();
    f.dense_div = dense_div;
    // (one engine: fout computed once the frontier grows, before the first dense hop)
    static const uint32_t fout_max = [] {
        const char* v = getenv("GSX_GXF_FOUT_MAX");
        return v && atoi(v) > 0 ? (uint32_t)atoi(v) : gsx::GXF_FOUT_MAX;
    }();
    {
        const uint32_t n = (uint32_t)e->n_nodes;
        const uint32_t thr = std::min({n / std::max(fout_div, 1u), fout_max, n / std::max(f.dense_div, 1u)});
        f.fout_lazy = (!f.fin && f.fent) ? std::max(thr, 1u) : 0u;
    }
    if (e->d_gxf_hst) {
        f.hstamp = e->d_gxf_hst;
        f.hidx = e->d_gxf_hst + E;
    }
    {
        ZeroBatch zb(e);
        if (int rc = zb.add(e->d_gxf_mask, 8 * 2 * N)) return rc;  // fmask
        if (int rc = zb.add(f.srcm, 8 * N)) return rc;
        if (int rc = zb.add(f.fbit[0], 8 * 2 * ((N + 63) / 64))) return rc;
        if (int rc = zb.add(e->d_gxf_cnt, 4 * 2 * ((size_t)gsx::GXF_MAX_HOPS + 1))) return rc;
        if (int rc = zb.flush()) return rc;
    }
    HIPCHK(e, gsx::launch_gxf_init(dev_state(e), R.h, f, n_src, e->stream));
    R.f = f;
    R.hops = 0;
    R.fwd_active = true;
    return GSX_OK;
}

int gxf_run_end(gsx_engine* e, gsx_engine::GxRound& R) {
    e->gxf_stamp = R.f.seq + R.hops + 1;
    R.fwd_active = false;
    return GSX_OK;
}

// The forwarding on one engine: every run, its hops launched in chunks with
// one host check of the last hop's frontier size per chunk.
int gx_forward(gsx_engine* e, gsx_engine::GxRound& R) {
    if (R.sets.empty() || e->n_nodes == 0) return GSX_OK;
    if (int rc = gxf_plan(e, R)) return rc;
    const gsx::DevState ds = dev_state(e);
    for (size_t k = 0; k < R.runs.size(); ++k) {
        if (int rc = gxf_run_begin(e, R, k)) return rc;
        uint32_t hop = 1;
        for (;;) {
            // (a steady round's runs end after two hops: a first chunk of three reads
            // their empty frontier at once; long runs check every eight hops)
            const uint32_t chunk = hop == 1 ? 3 : 8;
            if (hop + chunk > gsx::GXF_MAX_HOPS)
                return fail(e, GSX_ERANGE, "forwarding of recovered messages: more than " +
                                               std::to_string(gsx::GXF_MAX_HOPS) + " hops");
            for (uint32_t z = 0; z < chunk; ++z) HIPCHK(e, gsx::launch_gxf_hop(ds, R.h, R.f, hop + z, e->stream));
            hop += chunk;
            HIPCHK(e, hipMemcpyAsync(e->h_gxf_cnt, e->d_gxf_cnt + hop - 1, 4, hipMemcpyDeviceToHost, e->stream));
            HIPCHK(e, hipStreamSynchronize(e->stream));
            if (*e->h_gxf_cnt == 0) break;
        }
        R.hops = hop;
        if (int rc = gxf_run_end(e, R)) return rc;
    }
    return GSX_OK;
}

// The sets' validation codes this round (gsx.h (D), VcRef): whether each
// set's old copies are all / none / by code inside its topic's P3 window
// (the mixed sets' inside-code bits staged for d_gx_vin), and the code this
// round's recovered copies take (hb_finish drops it again from a set that
// recovered nothing; every rank of a range shard decides alike: got_all).
int gx_vcodes(gsx_engine* e, gsx_engine::GxRound& R) {
    if (int rc = vc_fence(e)) return rc;
    const size_t ns = R.sets.size();
    R.old_in.assign(ns, 0);
    R.vc_code.assign(ns, 0);
    R.vc.assign(ns, gsx::VcRef{});
    R.vin_host.clear();
    std::vector<size_t> vin_off(ns, 0);
    for (size_t i = 0; i < ns; ++i) {
        gsx_engine::MsgSet* ms = R.sets[i];
        if (ms->vtime.empty()) ms->vtime.push_back(ms->t0);
        const int64_t win = e->tp[ms->topic < GSX_MAX_TOPICS ? ms->topic : 0].mesh_message_deliveries_window_ns;
        if (!ms->hops_kept) {  // the hop codes stand as one (code 0): they must all fall on one side
            const size_t nh = std::min<size_t>(ms->n_hop, ms->vtime.size());
            bool hin = false, hout = false;
            for (size_t c = 0; c < nh; ++c) (R.h.now - ms->vtime[c] <= win ? hin : hout) = true;
            if (hin && hout)
                return fail(e, GSX_ESTATE, "a message set cached while the gossip exchange was off keeps no arrival "
                                           "hops, and this round's P3 window splits its copies (gsx.h (D))");
        }
        // the codes in use: code 0 alone without planes, else those the planes can hold
        const size_t nc = ms->d_vc ? std::min<size_t>(ms->vtime.size(), (size_t)1 << ms->vc_p) : 1;
        bool any_in = false, any_out = false;
        for (size_t c = 0; c < nc; ++c) (R.h.now - ms->vtime[c] <= win ? any_in : any_out) = true;
        R.old_in[i] = any_in && any_out ? 2u : any_in ? 1u : 0u;
        if (R.old_in[i] == 2) {
            vin_off[i] = R.vin_host.size();
            R.vin_host.resize(R.vin_host.size() + (nc + 63) / 64, 0);
            for (size_t c = 0; c < nc; ++c)
                if (R.h.now - ms->vtime[c] <= win) R.vin_host[vin_off[i] + c / 64] |= 1ull << (c % 64);
        }
        const uint32_t code = (uint32_t)ms->vtime.size();  // provisional: this round's recoveries
        if (int rc = vc_grow(e, ms, bit_width32(code))) return rc;
        ms->vtime.push_back(R.h.now);
        R.vc_code[i] = code;
    }
    if (R.vin_host.size() > e->gx_vin_cap) {
        if (e->d_gx_vin) (void)hipFree(e->d_gx_vin);
        e->d_gx_vin = nullptr;
        e->gx_vin_cap = 0;
        const size_t cap = std::max<size_t>(R.vin_host.size(), 64);
        if (int rc = dalloc(e, &e->d_gx_vin, cap)) return rc;
        e->gx_vin_cap = cap;
    }
    if (!R.vin_host.empty())
        HIPCHK(e, hipMemcpyAsync(e->d_gx_vin, R.vin_host.data(), 8 * R.vin_host.size(), hipMemcpyHostToDevice,
                                 e->stream));
    // range shards: the rows entries carry the senders' inside rows when some set is mixed
    R.h.gxs_vin = R.vin_host.empty() ? 0u : 1u;
    R.h.gx_mixed = R.h.gxs_vin;
    for (size_t i = 0; i < ns; ++i) {
        const gsx_engine::MsgSet* ms = R.sets[i];
        R.vc[i] = gsx::VcRef{ms->d_vc, R.old_in[i] == 2 ? e->d_gx_vin + vin_off[i] : nullptr,
                             (uint64_t)ms->n_words * e->n_nodes, ms->vc_p, 0u};
    }
    return GSX_OK;
}

// (D), first part: the advertised batches of hb_begin's windows (per topic,
// cache order), their message sets and receipt rows, the set heads and the
// flat word list; receipt rows zeroed, full bytes and common words (k_gx_setprep).
int gx_prepare(gsx_engine* e, gsx_engine::GxRound& R) {
    const size_t hist = (size_t)std::max(e->gp.history_length, 1);
    std::vector<gsx::GxBatch> gx;
    std::vector<bool> gx_full_new;  // per set: its full bytes are recomputed this round
    std::vector<bool> x_zero;       // per set: its receipt rows are zero already
    std::vector<uint32_t> off(e->T + 1, 0);
    const size_t n_win = std::min<size_t>((size_t)std::max(e->gp.history_gossip, 0), e->mc.size());
    const size_t N = e->n_nodes;
    for (uint32_t t = 0; t < e->T; ++t) {
        off[t] = (uint32_t)gx.size();
        uint32_t row_off = 0;  // the batch's words in the topic's gossip rows (hb_begin's layout)
        for (size_t w = 0; w < n_win; ++w)
            for (auto& b : e->mc[w]) {
                if (b.topic != t) continue;
                const uint32_t ro = row_off;
                row_off += b.n_words;
                if (!b.set) continue;
                size_t i = 0;
                while (i < R.sets.size() && R.sets[i] != b.set) ++i;
                if (i == R.sets.size()) {
                    const size_t words = (size_t)b.set->n_words * N + 2 * N;  // rows + (dig, cnt) tail
                    gsx_engine::MsgSet* ms = b.set;
                    // a receipt buffer the set's last round left untouched is still zero
                    uint64_t* x = ms->xs_spare;
                    x_zero.push_back(x != nullptr);
                    ms->xs_spare = nullptr;
                    if (!x) x = seen_acquire(e, words);  // (rows zeroed by k_gx_setprep)
                    if (!x) return fail(e, GSX_ENOMEM, "gossip exchange receipts");
                    // which nodes have seen the whole set (skipped by the walk): k_gx_setprep
                    gx_full_new.push_back(!ms->full_ok);
                    if (!ms->full_ok) {
                        if (!ms->d_full) {
                            size_t got = 0;
                            ms->d_full = small_acquire(e, N, &got);
                            if (!ms->d_full) return fail(e, GSX_ENOMEM, "message set full bytes");
                            ms->full_bytes = got;
                        }
                        ms->full_ok = true;
                    }
                    ++ms->refs;  // held until the recovered copies are cached (the Shift may drop its batches)
                    R.sets.push_back(b.set);
                    R.xs.push_back(x);
                }
                gx.push_back(gsx::GxBatch{b.d_seen, b.set->d_all, R.xs[i], b.set->d_val, nullptr, b.set->d_full,
                                          b.n_words, b.set->serial, t,
                                          (uint32_t)(e->mc.size() < hist || w + 1 < hist), ro});
                gx.back().got = reinterpret_cast<uint8_t*>(i);  // (index; rebased below)
                gx.back().dense = b.recovered ? 0u : 1u;
                gx.back().cnt = b.d_cnt;
                gx.back().src = b.set->d_src;
            }
    }
    off[e->T] = (uint32_t)gx.size();
    if (int rc = gx_vcodes(e, R)) return rc;
    // the set groups: consecutive sets of one topic, up to 64 sets and 65,535
    // messages each (the u16 back counts of the forwarding)
    R.set_grp.assign(R.sets.size(), 0);
    R.grp_topic.clear();
    {
        uint32_t cnt = 0;
        size_t msgs = 0;
        for (size_t i = 0; i < R.sets.size(); ++i) {
            const gsx_engine::MsgSet* ms = R.sets[i];
            if (ms->n_msgs > GSX_GX_MAX_SET_MSGS)  // (cached before the exchange was turned on)
                return fail(e, GSX_ERANGE, "gossip exchange: a cached message set above GSX_GX_MAX_SET_MSGS messages");
            if (R.grp_topic.empty() || R.grp_topic.back() != ms->topic || cnt == 64 ||
                msgs + ms->n_msgs > GSX_GX_MAX_SET_MSGS) {
                R.grp_topic.push_back(ms->topic);
                cnt = 0;
                msgs = 0;
            }
            R.set_grp[i] = (uint32_t)R.grp_topic.size() - 1;
            ++cnt;
            msgs += ms->n_msgs;
        }
    }
    {  // the flat word list of all advertised batches (k_gx_node's rounds)
        uint32_t fw = 0;
        for (size_t i = 0; i < gx.size(); ++i) {
            gx[i].woff = fw;
            fw += gx[i].n_words;
            const size_t si = reinterpret_cast<size_t>(gx[i].got);  // (got: the set's index yet)
            gx[i].n_msgs = R.sets[si]->n_msgs;
            gx[i].grp = R.set_grp[si];
            gx[i].old_in = R.old_in[si];
            gx[i].vc = R.vc[si];
        }
        for (auto& g : gx) g.vin_off = 1 + fw + g.woff;  // (range shards: after the entry's rows)
    }
    // every set's words in canonical order, (its first batch in cache order,
    // word, topic) (k_gx_node's receipts: a lane per set word walks the set's
    // batches through `nxt`), and the flat word list's batch per word
    std::vector<uint4> sw;
    std::vector<uint32_t> wb;
    {
        std::vector<uint32_t> last(R.sets.size(), ~0u);
        for (uint32_t t = 0; t < e->T; ++t)
            for (uint32_t g = off[t]; g < off[t + 1]; ++g) {
                const size_t si = reinterpret_cast<size_t>(gx[g].got);
                gx[g].nxt = ~0u;
                if (last[si] == ~0u || gx[last[si]].topic != t) {
                    for (uint32_t w = 0; w < gx[g].n_words; ++w) sw.push_back(make_uint4(g, w, t, 0u));
                } else {
                    gx[last[si]].nxt = g;
                }
                last[si] = g;
            }
        for (uint32_t g = 0; g < gx.size(); ++g) wb.insert(wb.end(), gx[g].n_words, g);  // (woff order)
    }
    dbg_host("gx sets");
    static const bool dbg = getenv("GSX_DBG_GX") != nullptr;
    if (dbg) {
        HIPCHK(e, hipStreamSynchronize(e->stream));
        std::vector<uint8_t> fb(N);
        fprintf(stderr, "[gx] not full per set:");
        for (auto* ms : R.sets) {
            HIPCHK(e, hipMemcpy(fb.data(), ms->d_full, N, hipMemcpyDeviceToHost));
            size_t nf = 0;
            for (uint8_t x : fb) nf += x == 0;
            fprintf(stderr, " s%u:%zu", ms->serial, nf);
        }
        fprintf(stderr, "\n[gx] sets=%zu batches=%zu:", R.sets.size(), gx.size());
        for (const auto& g : gx) fprintf(stderr, " (t%u w%u s%u a%u)", g.topic, g.n_words, g.serial, g.avail);
        fprintf(stderr, "\n");
    }
    if (std::max(gx.size(), R.sets.size()) > e->gx_cap || !e->d_gx_got) {  // (per set: got, chg)
        if (e->d_gx_got) (void)hipFree(e->d_gx_got);
        e->d_gx_got = nullptr;
        // (doubling, 64 at least: a free here waits for every queued kernel)
        e->gx_cap = std::max<size_t>(std::max<size_t>(std::max(gx.size(), R.sets.size()), 2 * e->gx_cap), 64);
        if (int rc = dalloc(e, &e->d_gx_got, 2 * e->gx_cap)) return rc;  // got, then chg
        e->d_gx_chg = e->d_gx_got + e->gx_cap;
    }
    // per set, the messages every node had seen as the exchange began (a
    // set wider than 64 words keeps none: its rows are filtered by emptiness)
    if (R.sets.size() > e->gx_common_cap || !e->d_gx_rhm) {
        if (e->d_gx_common) (void)hipFree(e->d_gx_common);
        e->d_gx_common = nullptr;
        e->gx_common_cap = std::max<size_t>(std::max<size_t>(R.sets.size(), 2 * e->gx_common_cap), 32);
        if (int rc = dalloc(e, &e->d_gx_common, 64 * e->gx_common_cap)) return rc;
        if (!e->d_gx_rhm)
            if (int rc = dalloc(e, &e->d_gx_rhm, N)) return rc;
    }
    // per set what the prep pass has to do: zero the receipt rows, recompute
    // the full bytes, AND the common words; a set with none of it is skipped
    // (one engine keeps each set's common words while its seen rows stand;
    // a range shard ANDs them over the ranks every round)
    std::vector<gsx::GxSetPrep> sprep;
    std::vector<uint64_t*> common_of(R.sets.size(), nullptr);
    for (size_t i = 0; i < R.sets.size(); ++i) {
        gsx_engine::MsgSet* ms = R.sets[i];
        uint64_t* common = nullptr;
        bool redo_common = false;
        if (ms->n_words <= 64) {
            if (e->sharded()) {
                common = e->d_gx_common + 64 * i;
                redo_common = true;
            } else {
                if (!ms->d_common) {  // (the common words, then common2: GxBatch::common2)
                    ms->d_common = reinterpret_cast<uint64_t*>(small_acquire(e, 8 * 128, &ms->common_bytes));
                    if (!ms->d_common) return fail(e, GSX_ENOMEM, "message set common words");
                    ms->common_ok = false;
                }
                common = ms->d_common;
                redo_common = !ms->common_ok;
                if (redo_common) HIPCHK(e, hipMemsetAsync(common, 0xff, 8 * 128, e->stream));
                ms->common_ok = true;  // (hb_finish drops it when a receipt changes the rows)
            }
        }
        common_of[i] = common;
        gsx::GxSetPrep p{ms->d_all, x_zero[i] ? nullptr : R.xs[i], gx_full_new[i] ? ms->d_full : nullptr,
                         redo_common ? common : nullptr, ms->n_words, ms->n_msgs};
        // (common2 on one engine for sets of up to eight words: k_gx_setprep's register
        // path; wider sets keep the all-node words, cached, and are walked unfiltered)
        p.common2 = (redo_common && !e->sharded() && ms->n_words <= 8) ? common + 64 : nullptr;
        if (p.x || p.full || p.common) sprep.push_back(p);
    }
    std::vector<gsx::GxSetMerge> smerge(R.sets.size());
    for (size_t i = 0; i < R.sets.size(); ++i) {
        const gsx_engine::MsgSet* ms = R.sets[i];
        const size_t W = ms->n_words;
        smerge[i] = gsx::GxSetMerge{ms->d_all, R.xs[i], ms->d_acc, ms->d_dg, R.xs[i] + W * N,
                                    reinterpret_cast<uint32_t*>(R.xs[i] + W * N + N), ms->n_words, ms->n_msgs,
                                    ms->d_vc, (uint64_t)W * N, ms->vc_p, R.vc_code[i], e->d_gx_chg + i,
                                    R.h.gx_touch, e->sharded() ? nullptr : ms->d_full};
    }
    if (e->sharded()) HIPCHK(e, hipMemsetAsync(e->d_gx_common, 0xff, 8 * 64 * R.sets.size(), e->stream));
    for (auto& g : gx) {
        const size_t si = reinterpret_cast<size_t>(g.got);
        g.common = common_of[si];
        g.common2 = (common_of[si] && !e->sharded() && R.sets[si]->n_words <= 8) ? common_of[si] + 64 : nullptr;
        g.got = e->d_gx_got + si;
    }
    HIPCHK(e, hipMemsetAsync(e->d_gx_got, 0, 2 * e->gx_cap, e->stream));  // got, chg
    {  // the batch list, offsets, word and set-word lists, prep and merge lists: one pinned
        // staging buffer, one async copy into the device arena d_gxa (the host
        // keeps queueing; the last round's copy drained at its end)
        const auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
        const size_t b_gx = sizeof(gsx::GxBatch) * gx.size(), b_off = 4 * off.size(), b_wb = 4 * wb.size(),
                     b_sw = sizeof(uint4) * sw.size(), b_sp = sizeof(gsx::GxSetPrep) * sprep.size(),
                     b_mg = sizeof(gsx::GxSetMerge) * smerge.size();
        const size_t a_off = al(b_gx), a_wb = al(a_off + b_off), a_sw = al(a_wb + b_wb), a_sp = al(a_sw + b_sw),
                     a_mg = al(a_sp + b_sp);
        const size_t need = a_mg + b_mg;
        if (e->h_gxstage_bytes < need) {
            if (e->h_gxstage) (void)hipHostFree(e->h_gxstage);
            e->h_gxstage = nullptr;
            e->h_gxstage_bytes = 0;
            HIPCHK(e, hipHostMalloc(&e->h_gxstage, 2 * need, hipHostMallocDefault));
            e->h_gxstage_bytes = 2 * need;
        }
        if (e->gxa_bytes < need) {  // (a free here waits for every queued kernel)
            if (e->d_gxa) (void)hipFree(e->d_gxa);
            e->d_gxa = nullptr;
            e->gxa_bytes = 0;
            const size_t bytes = std::max<size_t>(2 * need, 64 << 10);
            if (int rc = dalloc(e, &e->d_gxa, bytes)) return rc;
            e->gxa_bytes = bytes;
        }
        char* hs = static_cast<char*>(e->h_gxstage);
        std::memcpy(hs, gx.data(), b_gx);
        std::memcpy(hs + a_off, off.data(), b_off);
        if (b_wb) std::memcpy(hs + a_wb, wb.data(), b_wb);
        if (b_sw) std::memcpy(hs + a_sw, sw.data(), b_sw);
        if (b_sp) std::memcpy(hs + a_sp, sprep.data(), b_sp);
        if (b_mg) std::memcpy(hs + a_mg, smerge.data(), b_mg);
        HIPCHK(e, hipMemcpyAsync(e->d_gxa, hs, need, hipMemcpyHostToDevice, e->stream));
        e->d_gx = reinterpret_cast<gsx::GxBatch*>(e->d_gxa);
        e->d_gx_off = reinterpret_cast<uint32_t*>(e->d_gxa + a_off);
        e->d_gx_wb = reinterpret_cast<uint32_t*>(e->d_gxa + a_wb);
        e->d_gx_sw = reinterpret_cast<uint4*>(e->d_gxa + a_sw);
        e->d_gx_sp = reinterpret_cast<gsx::GxSetPrep*>(e->d_gxa + a_sp);
        e->d_gx_mg = reinterpret_cast<gsx::GxSetMerge*>(e->d_gxa + a_mg);
        // receipt rows zeroed, full bytes, common words: every set that needs any, in one pass
        HIPCHK(e, gsx::launch_gx_setprep(e->d_gx_sp, (uint32_t)sprep.size(), (uint32_t)N, e->stream));
    }
    R.h.gx_sw = e->d_gx_sw;
    R.h.gx_nsw = (uint32_t)sw.size();
    R.h.gx_wb = e->d_gx_wb;
    R.h.gx = e->d_gx;
    R.h.gx_off = e->d_gx_off;
    R.n_gx = (uint32_t)gx.size();
    R.fw = gx.empty() ? 0u : gx.back().woff + gx.back().n_words;
    R.h.gx_fw = R.fw;
    return GSX_OK;
}

// (D), second part: the uncommon-row masks (k_gx_rhm, over the common words of
// every rank on a shard), the answered-pair mask and the round's back-count stamp.
int gx_ready(gsx_engine* e, gsx_engine::GxRound& R) {
    gsx::HbState& h = R.h;
    HIPCHK(e, gsx::launch_gx_rhm(e->d_gx, R.n_gx, (uint32_t)e->n_nodes, e->d_gx_rhm, e->stream));
    h.gx_rhm = e->d_gx_rhm;
    h.gx_poor = e->sharded() ? 0u : 1u;  // (one engine: gx_rhm over common2)
    h.gsubs = e->d_gsubs;
    // the answered pairs' records take the receipts' credits: re-scored after
    // (the rest stays exact), when the scores were exact before
    R.exact = e->scores_valid;
    if (R.exact) {
        h.gx_mark = e->d_dirty + 3 * e->E;  // (the broken-promise mask of hb_begin, read by then)
        HIPCHK(e, hipMemsetAsync(h.gx_mark, 0, std::max<size_t>(e->E, 1), e->stream));
    }
    if (int rc = gxf_alloc(e)) return rc;
    h.gxb_st0 = e->d_gxf_bst;
    h.gxb_cnt0 = e->d_gxf_b0;
    h.gxb_ngrp = (uint32_t)R.grp_topic.size();
    h.gxb_stamp = ++e->gxf_stamp;
    dbg_host("gx prepared");
    return GSX_OK;
}

// (D), last part: receipts merged into the sets, the recovered rows'
// summaries written (every set, one pass); the credited pairs re-scored.
int gx_merge(gsx_engine* e, gsx_engine::GxRound& R) {
    HIPCHK(e, gsx::launch_gx_merge_sets(e->d_gx_mg, (uint32_t)R.sets.size(), (uint32_t)e->n_nodes, e->stream));
    if (R.exact) {  // the receipts credited P2 / P3 / P4 of the answered pairs
        HIPCHK(e, rescore_subset(e, dev_state(e), kern_params(e), R.h.gx_mark));
    } else {
        e->invalidate_scores();
    }
    ++e->score_gen;
    return GSX_OK;
}

// The round's end: counters, mcache.Shift, the recovered copies Put (one
// batch per message set some node received in: got_all, every rank's on a
// shard; null: this engine's), promise slots kept free.
#ifdef GSX_GX_PROF
extern "C" void gx_prof_dump();  // (gsx_gossip.hip, diagnostic build)
#endif
int hb_finish(gsx_engine* e, gsx_engine::GxRound& R, gsx_heartbeat_out* out, const uint8_t* got_all) {
#ifdef GSX_GX_PROF
    gx_prof_dump();
#endif
    const gsx::HbState& h = R.h;
    const bool gx_run = R.run;
    const size_t hist = (size_t)std::max(e->gp.history_length, 1);
    auto& gx_sets = R.sets;
    auto& gx_x = R.xs;
    unsigned long long st[gsx::HB_STAT_WORDS];
    uint32_t gflag[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    std::vector<uint8_t> got(gx_sets.size(), 0), chg(gx_sets.size(), 1);
    // the round's counters, flags and per-set bytes read back through one pinned
    // buffer (async copies queued together; one drain)
    const size_t nset = gx_run ? gx_sets.size() : 0;
    const size_t rb_bytes = sizeof(st) + sizeof(gflag) + 2 * (gx_run ? e->gx_cap : 0);
    if (e->h_hbrb_bytes < rb_bytes) {
        if (e->h_hbrb) (void)hipHostFree(e->h_hbrb);  // (the last round's copies drained at its end)
        e->h_hbrb = nullptr;
        e->h_hbrb_bytes = 0;
        HIPCHK(e, hipHostMalloc(&e->h_hbrb, 2 * rb_bytes, hipHostMallocDefault));
        e->h_hbrb_bytes = 2 * rb_bytes;
    }
    uint8_t* rb = static_cast<uint8_t*>(e->h_hbrb);
    HIPCHK(e, hipMemcpyAsync(rb, e->d_hbstats, sizeof(st), hipMemcpyDeviceToHost, e->stream));
    if (gx_run) {
        HIPCHK(e, hipMemcpyAsync(rb + sizeof(st), e->d_gxflag, sizeof(gflag), hipMemcpyDeviceToHost, e->stream));
        if (nset)  // got (this engine's: unless got_all) and chg, d_gx_got's two halves
            HIPCHK(e, hipMemcpyAsync(rb + sizeof(st) + sizeof(gflag), e->d_gx_got, e->gx_cap + nset,
                                     hipMemcpyDeviceToHost, e->stream));
    }
    dbg_host("gx queued");
    HIPCHK(e, hipStreamSynchronize(e->stream));
    std::memcpy(st, rb, sizeof(st));
    if (gx_run) {
        std::memcpy(gflag, rb + sizeof(st), sizeof(gflag));
        if (nset) {
            std::memcpy(got.data(), rb + sizeof(st) + sizeof(gflag), nset);
            std::memcpy(chg.data(), rb + sizeof(st) + sizeof(gflag) + e->gx_cap, nset);
        }
    }
    if (got_all) std::memcpy(got.data(), got_all, got.size());
    for (auto& fr : R.scratch) seen_release(e, fr.first, fr.second);
    R.scratch.clear();
    R.pending = false;
    R.stage = 0;
    dbg_host("hb drained");
    static_assert(sizeof(gsx_heartbeat_out) == sizeof(st), "gsx_heartbeat_out mirrors HB_STAT_WORDS");
    std::memcpy(out, st, sizeof(st));
    // a bulk round's (B) left the control words: one clear at the next round's start
    if (gsx::hb_bulk_round(st[gsx::HB_GRAFTS], st[gsx::HB_PRUNES], e->E)) e->hb_clean = false;
    e->px_last = h.pxno ? st[gsx::HB_PX_CONNECT] : 0;
    // mcache.Shift (mcache.go:94-104, gossipsub.go:1563), after the stream drained
    while (e->mc.size() >= hist) {
        for (auto& b : e->mc.back()) batch_release(e, b);
        e->mc.pop_back();
    }
    e->mc.emplace_front();
    // the recovered copies: one batch per message set, Put into the new window 0
    // in ascending set serial (the sets' creation order: gsx.h)
    const size_t N = e->n_nodes;
    std::vector<size_t> by_serial(gx_sets.size());
    for (size_t i = 0; i < by_serial.size(); ++i) by_serial[i] = i;
    std::sort(by_serial.begin(), by_serial.end(),
              [&](size_t a, size_t b) { return gx_sets[a]->serial < gx_sets[b]->serial; });
    for (size_t i : by_serial) {
        gsx_engine::MsgSet* ms = gx_sets[i];
        if (!got[i]) {
            if (!chg[i] && !ms->xs_spare) ms->xs_spare = gx_x[i];  // untouched: still zero for the next round
            else seen_release(e, gx_x[i], (size_t)ms->n_words * N + 2 * N);
            // nothing recovered: no copy took this round's code (k_gx_merge_sets writes accepted receipts only)
            if (i < R.vc_code.size() && ms->vtime.size() == (size_t)R.vc_code[i] + 1) ms->vtime.pop_back();
            continue;
        }
        gsx_engine::McBatch b;
        b.topic = ms->topic;
        b.n_msgs = ms->n_msgs;
        b.n_words = ms->n_words;
        b.d_seen = gx_x[i];
        b.seen_words = (size_t)ms->n_words * N + 2 * N;
        b.d_dig = gx_x[i] + (size_t)ms->n_words * N;
        b.d_cnt = reinterpret_cast<uint32_t*>(gx_x[i] + (size_t)ms->n_words * N + N);
        b.ids = ms->ids;
        b.set = ms;
        b.recovered = true;
        ++ms->refs;  // (its summary: k_gx_merge_sets)
        e->mc.front().push_back(std::move(b));
    }
    const bool merged = gx_run && st[gsx::HB_GOSSIP_DELIVERED] + st[gsx::HB_GOSSIP_REJECTED] +
                                          st[gsx::HB_FWD_DELIVERED] > 0;
    for (size_t i = 0; i < gx_sets.size(); ++i) {
        gsx_engine::MsgSet* ms = gx_sets[i];
        // the receipts were merged into its seen rows: one engine's merge kept the
        // full bytes exact at the touched nodes (only a range shard recomputes
        // them); the common words would stand as a subset of the new ones, but
        // common2 would not (a node that stopped being poor joins its AND), so
        // a set with common2 recomputes both
        if (merged) {
            if (e->sharded()) ms->full_ok = false;
            if (e->sharded() || ms->n_words <= 8) ms->common_ok = false;  // (sets with common2)
        }
        set_release(e, ms);
    }
    gx_sets.clear();
    gx_x.clear();
    dbg_host("hb shift+put");
    if (gflag[0] || gflag[1])
        return fail(e, GSX_ESTATE, "gossip exchange: internal bound broken (truncated-list rows / promise slots)");
    // every pair keeps a free promise slot for the next exchange (one promise per pair each)
    if (gx_run && gflag[4] >= e->prom_slots)
        if (int rc = gx_prom_grow(e)) return rc;
    return GSX_OK;
}

int hb_end(gsx_engine* e, const uint64_t* halo_resp, gsx_heartbeat_out* out) {
    e->state_changed();
    gsx::HbState h = e->hb;
    h.halo_resp = halo_resp;
    const gsx::DevState ds = dev_state(e);
    e->hb_active = false;
    std::memset(out, 0, sizeof(*out));
    if (h.pxno && e->sharded() && !e->pxs_packed[1])
        return fail(e, GSX_ESTATE, "peer exchange on a shard: gsx_hb_px_pack(1) before gsx_hb_end");
    if (!e->sharded()) HIPCHK(e, gsx::launch_hb_px(ds, h, 1, e->stream));  // the (B) answers' peer exchange (do_px)
    HIPCHK(e, gsx::launch_hb_answer(ds, h, e->stream));
    e->hb_clean = !e->sharded() && !e->hb_tracing;  // (tracing keeps the control words)
    HIPCHK(e, rescore_subset(e, ds, kern_params(e), h.dirty, nullptr, hb_ctl_gate(e)));  // the cache leaves the round exact
    // (D) the gossip exchange over the batches the IHAVEs advertised (the
    // windows of hb_begin's list), answered across the Shift
    gsx_engine::GxRound& R = e->gxr;
    R.run = e->gp.gossip_exchange && h.ihave_bits && e->have_gossip;
    R.pending = false;
    R.stage = 0;
    R.sets.clear();
    R.xs.clear();
    R.scratch.clear();
    R.h = h;
    dbg_host("hb (B)(C)");
    if (R.run) {
        int rc = gx_prepare(e, R);
        if (!rc && e->sharded()) {  // the gsx_gx_* steps carry (D) across the ranks, gsx_gx_end finishes the round
            R.pending = true;
            R.stage = 1;
            return GSX_OK;
        }
        if (!rc) rc = gx_ready(e, R);
        if (!rc) {
            const hipError_t st = gsx::launch_gx_exchange(ds, R.h, e->stream);
            if (st != hipSuccess) rc = fail(e, GSX_EDEVICE, std::string("launch_gx_exchange: ") + hipGetErrorString(st));
        }
        // the recovered messages published on (their forwarded first receipts join the receipt rows)
        if (!rc) rc = gx_forward(e, R);
        if (!rc) rc = gx_merge(e, R);
        if (rc) {  // the sets' references and rows back to the pools (the round is lost)
            const std::string msg = e->err;
            gx_abort(e);
            e->err = msg;
            return rc;
        }
    }
    return hb_finish(e, R, out, nullptr);
}

}  // namespace

// ---- the gossipTracer's promises (gossip_tracer.go:48-185), one router per observer

namespace {
uint64_t host_smix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// Go's Int31n over draws h(seed, tag, a, base | k) (the kernels' Rng, gsx_ops.h)
int32_t host_int31n(uint64_t seed, uint64_t tag, uint64_t a, uint64_t base, int32_t n) {
    uint32_t k = 0;
    auto draw = [&]() {
        const uint64_t x = host_smix(seed + 0x9E3779B97F4A7C15ull *
                                               (1ull + host_smix(tag ^ host_smix(a ^ host_smix(base | k++)))));
        return (int32_t)(x >> 33);
    };
    if ((n & (n - 1)) == 0) return draw() & (n - 1);
    const int32_t mx = (int32_t)((1u << 31) - 1 - (1u << 31) % (uint32_t)n);
    int32_t v = draw();
    while (v > mx) v = draw();
    return v % n;
}
int prom_ready(gsx_engine* e) {
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (e->sharded()) return fail(e, GSX_ESTATE, "promises live on unsharded engines (the gossip exchange)");
    return gx_alloc(e);
}
}  // namespace

int gsx_promise_add(gsx_engine* e, uint64_t pair, const uint64_t* handles, uint32_t n, int64_t expire_ns,
                    uint64_t seed) {
    // (expiry 0 marks a free slot; a promise's expiry is now + IWantFollowupTime, never the zero time)
    if (!e || !handles || n == 0 || n > 0x7FFFFFFFu || expire_ns == 0) return GSX_EINVAL;
    if (int rc = prom_ready(e)) return rc;
    if (pair >= e->E) return fail(e, GSX_ERANGE, "pair out of range");
    const uint64_t handle = handles[host_int31n(seed, gsx::TAG_IWANT, pair, 0, (int32_t)n)];  // :53
    for (;;) {
        const uint32_t S = e->prom_slots;
        std::vector<uint64_t> hs(S);
        std::vector<int64_t> es(S);
        HIPCHK(e, hipMemcpyAsync(hs.data(), e->d_prom_h + pair * S, 8 * S, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipMemcpyAsync(es.data(), e->d_prom_e + pair * S, 8 * S, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        uint32_t used = 0, fr = S;
        for (uint32_t k = 0; k < S; ++k) {
            if (es[k] == 0) {
                if (fr == S) fr = k;
                continue;
            }
            ++used;
            if (hs[k] == handle) return GSX_OK;  // promises[mid][p] exists (:66)
        }
        if (fr == S || used + 1 >= S) {  // keep a free slot on every pair (the next exchange adds one)
            if (int rc = gx_prom_grow(e)) return rc;
            if (fr == S) continue;  // (a free slot keeps its index through the grow)
        }
        const uint32_t S2 = e->prom_slots;
        HIPCHK(e, hipMemcpy(e->d_prom_h + pair * S2 + fr, &handle, 8, hipMemcpyHostToDevice));
        HIPCHK(e, hipMemcpy(e->d_prom_e + pair * S2 + fr, &expire_ns, 8, hipMemcpyHostToDevice));
        const uint8_t one = 1;
        HIPCHK(e, hipMemcpy(e->d_prom_any + pair, &one, 1, hipMemcpyHostToDevice));
        return GSX_OK;
    }
}

int gsx_promise_broken(gsx_engine* e, int64_t now_ns, uint32_t* counts, uint64_t* total) {
    if (!e) return GSX_EINVAL;
    if (int rc = prom_ready(e)) return rc;
    const size_t E = std::max<size_t>(e->E, 1);
    uint32_t* d_cnt = nullptr;
    unsigned long long* d_tot = nullptr;
    if (int rc = dalloc(e, &d_cnt, E)) return rc;
    if (int rc = dalloc(e, &d_tot, gsx::HB_STAT_WORDS)) {
        (void)hipFree(d_cnt);
        return rc;
    }
    gsx::HbState h{};
    h.n_pairs = e->E;
    h.now = now_ns;
    h.prom_h = e->d_prom_h;
    h.prom_e = e->d_prom_e;
    h.prom_any = e->d_prom_any;
    h.prom_slots = e->prom_slots;
    h.stats = d_tot;
    unsigned long long st[gsx::HB_STAT_WORDS];
    hipError_t he = hipMemsetAsync(d_tot, 0, sizeof(st), e->stream);
    if (he == hipSuccess) he = gsx::launch_gx_broken(h, d_cnt, e->stream);
    if (he == hipSuccess && counts)
        he = hipMemcpyAsync(counts, d_cnt, 4 * (size_t)e->E, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(st, d_tot, sizeof(st), hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    (void)hipFree(d_cnt);
    (void)hipFree(d_tot);
    if (he != hipSuccess) return fail(e, GSX_EDEVICE, std::string("gsx_promise_broken: ") + hipGetErrorString(he));
    if (total) *total = st[gsx::HB_BROKEN_PROMISES];
    return GSX_OK;
}

int gsx_promise_fulfill(gsx_engine* e, uint32_t node, uint64_t handle) {
    if (!e) return GSX_EINVAL;
    if (int rc = prom_ready(e)) return rc;
    if (node >= e->n_nodes) return fail(e, GSX_ERANGE, "node out of range");
    const uint32_t S = e->prom_slots;
    const size_t p0 = (size_t)e->row_ptr[node] * S, n = (size_t)(e->row_ptr[node + 1] - e->row_ptr[node]) * S;
    if (n == 0) return GSX_OK;
    std::vector<uint64_t> hs(n);
    std::vector<int64_t> es(n);
    HIPCHK(e, hipMemcpyAsync(hs.data(), e->d_prom_h + p0, 8 * n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(es.data(), e->d_prom_e + p0, 8 * n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    bool any = false;
    for (size_t i = 0; i < n; ++i)
        if (es[i] != 0 && hs[i] == handle) {  // delete(gt.promises, mid): every peer's promise for it (:119-126)
            es[i] = 0;
            any = true;
        }
    if (any) HIPCHK(e, hipMemcpy(e->d_prom_e + p0, es.data(), 8 * n, hipMemcpyHostToDevice));
    return GSX_OK;
}

int gsx_promise_throttle(gsx_engine* e, uint64_t pair) {
    if (!e) return GSX_EINVAL;
    if (int rc = prom_ready(e)) return rc;
    if (pair >= e->E) return fail(e, GSX_ERANGE, "pair out of range");
    HIPCHK(e, hipMemsetAsync(e->d_prom_e + pair * e->prom_slots, 0, 8 * (size_t)e->prom_slots, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_promise_count(gsx_engine* e, uint64_t* n) {
    if (!e || !n) return GSX_EINVAL;
    *n = 0;
    if (!e->d_prom_e) return GSX_OK;
    // counted on the device, ordered on the engine's stream; one u64 comes back
    gsx::HbState h{};
    h.n_pairs = e->E;
    h.prom_e = e->d_prom_e;
    h.prom_any = e->d_prom_any;
    h.prom_slots = e->prom_slots;
    HIPCHK(e, hipMemsetAsync(e->d_prom_cnt, 0, 8, e->stream));
    HIPCHK(e, gsx::launch_gx_count(h, e->d_prom_cnt, e->stream));
    unsigned long long c = 0;
    HIPCHK(e, hipMemcpyAsync(&c, e->d_prom_cnt, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    *n = c;
    return GSX_OK;
}

int gsx_heartbeat(gsx_engine* e, uint64_t tick, int64_t now, uint64_t seed, gsx_heartbeat_out* out) {
    if (!e || !out) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (e->loaded && e->sharded()) return fail(e, GSX_ESTATE, "sharded engine: drive the round with gsx_hb_*");
    if (e->hb_active) return fail(e, GSX_ESTATE, "a stepped heartbeat is in flight");
    if (int rc = hb_begin(e, tick, now, seed)) return rc;
    if (int rc = hb_recv(e, nullptr)) return rc;
    return hb_end(e, nullptr, out);
}

int gsx_hb_reserve(gsx_engine* e) {
    if (!e) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (e->max_deg > gsx::HB_HUB_MAX) return GSX_OK;  // (gsx_heartbeat refuses this overlay)
    if (!e->d_hbstats)
        if (int rc = hb_alloc(e)) return rc;
    if (e->gp.gossip_exchange) {
        if (int rc = gx_alloc(e)) return rc;
        if (int rc = gxf_alloc(e)) return rc;
        gx_target_bound(e);
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_hb_begin(gsx_engine* e, uint64_t tick, int64_t now, uint64_t seed) {
    if (!e) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (e->hb_active) return fail(e, GSX_ESTATE, "a stepped heartbeat is in flight");
    return hb_begin(e, tick, now, seed);
}

int gsx_hb_pack_ctl(gsx_engine* e, uint64_t* send) {
    if (!e) return GSX_EINVAL;
    if (!e->hb_active) return fail(e, GSX_ESTATE, "gsx_hb_begin first");
    if (e->n_send && !send) return GSX_EINVAL;
    HIPCHK(e, gsx::launch_hb_pack(e->d_send_pair, e->n_send, 2, e->d_ctl, e->d_ctl + 1, send, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_hb_recv(gsx_engine* e, const uint64_t* halo_ctl) {
    if (!e) return GSX_EINVAL;
    if (!e->hb_active) return fail(e, GSX_ESTATE, "gsx_hb_begin first");
    if (e->n_recv && !halo_ctl) return GSX_EINVAL;
    return hb_recv(e, halo_ctl);
}

int gsx_hb_pack_resp(gsx_engine* e, uint64_t* send) {
    if (!e) return GSX_EINVAL;
    if (!e->hb_active) return fail(e, GSX_ESTATE, "gsx_hb_begin first");
    if (e->n_send && !send) return GSX_EINVAL;
    HIPCHK(e, gsx::launch_hb_pack(e->d_send_pair, e->n_send, 1, e->d_resp, nullptr, send, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

// ---- peer exchange across range shards (gsx.h) -------------------------------------

namespace {
int px_shard_ready(gsx_engine* e, uint32_t kind) {
    if (!e->hb_active) return fail(e, GSX_ESTATE, "gsx_hb_begin first");
    if (kind > 1) return fail(e, GSX_EINVAL, "kind is 0 (the (A) PRUNEs) or 1 (the (B) answers)");
    if (!e->hb.pxno) return fail(e, GSX_ESTATE, "peer exchange is off (do_px)");
    if (!e->sharded()) return fail(e, GSX_ESTATE, "unsharded engines run the peer exchange inside the round");
    return GSX_OK;
}
}  // namespace

int gsx_hb_px_entry_words(gsx_engine* e, uint32_t* words) {
    if (!e || !words) return GSX_EINVAL;
    *words = 3u + (uint32_t)std::max(e->gp.prune_peers, 0);
    return GSX_OK;
}

int gsx_hb_px_count(gsx_engine* e, uint32_t kind, uint64_t* counts) {
    if (!e || !counts) return GSX_EINVAL;
    if (int rc = px_shard_ready(e, kind)) return rc;
    gsx::HbState h = e->hb;
    const uint32_t R = std::max<uint32_t>(e->n_ranks, 1);
    HIPCHK(e, hipMemsetAsync(e->d_pxs_cnt, 0, 8 * (size_t)R, e->stream));
    if (e->n_send) HIPCHK(e, gsx::launch_hb_px_count(h, kind, e->stream));
    e->pxs_counts.assign(R, 0);
    HIPCHK(e, hipMemcpyAsync(e->pxs_counts.data(), e->d_pxs_cnt, 8 * (size_t)R, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    std::memcpy(counts, e->pxs_counts.data(), 8 * (size_t)R);
    return GSX_OK;
}

int gsx_hb_px_pack(gsx_engine* e, uint32_t kind, uint32_t* out) {
    if (!e) return GSX_EINVAL;
    if (int rc = px_shard_ready(e, kind)) return rc;
    const uint32_t R = std::max<uint32_t>(e->n_ranks, 1);
    if (e->pxs_counts.size() != R) return fail(e, GSX_ESTATE, "gsx_hb_px_count first");
    uint64_t tot = 0;
    std::vector<uint64_t> off(R);
    for (uint32_t d = 0; d < R; ++d) {
        off[d] = tot;
        tot += e->pxs_counts[d];
    }
    if (tot && !out) return GSX_EINVAL;
    gsx::HbState h = e->hb;
    h.pxs_out = out;
    HIPCHK(e, hipMemcpyAsync(e->d_pxs_off, off.data(), 8 * (size_t)R, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_pxs_cnt, 0, 8 * (size_t)R, e->stream));
    // every PX PRUNE of this rank's nodes: local receivers handled here, the
    // others' lists written out (kind 0 reads the (A) PRUNE words, 1 the (B) answers)
    HIPCHK(e, gsx::launch_hb_px(dev_state(e), h, kind, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));  // `off` is on the host stack
    e->pxs_counts.clear();
    e->pxs_packed[kind] = true;
    return GSX_OK;
}

int gsx_hb_px_recv(gsx_engine* e, uint32_t kind, const uint32_t* entries, uint64_t n) {
    if (!e || (n && !entries)) return GSX_EINVAL;
    if (int rc = px_shard_ready(e, kind)) return rc;
    if (!e->pxs_packed[kind]) return fail(e, GSX_ESTATE, "gsx_hb_px_pack first (the round's own lists)");
    HIPCHK(e, gsx::launch_hb_px_recv(dev_state(e), e->hb, entries, n, e->stream));
    return GSX_OK;
}

int gsx_hb_end(gsx_engine* e, const uint64_t* halo_resp, gsx_heartbeat_out* out) {
    if (!e || !out) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (!e->hb_active) return fail(e, GSX_ESTATE, "gsx_hb_begin first");
    if (e->n_recv && !halo_resp) return GSX_EINVAL;
    return hb_end(e, halo_resp, out);
}

// ---- the gossip exchange across range shards (gsx.h: gsx_gx_*, gsx_gxf_*) ----------

namespace {
int gxs_step(gsx_engine* e, int stage) {
    if (!e->gxr.pending) return fail(e, GSX_ESTATE, "no sharded gossip exchange in flight (gsx_hb_end prepares one)");
    if (stage >= 0 && e->gxr.stage != stage) return fail(e, GSX_ESTATE, "gossip exchange steps out of order");
    return GSX_OK;
}
gsx::GxsPlan gxs_plan(gsx_engine* e) {
    return gsx::GxsPlan{e->d_send_pair, e->d_send_dest, e->d_send_base, e->d_dest_halo_base, e->d_pair_obs, e->n_send};
}
// A count pass, then the pack into the engine's send buffer in destination order.
using GxsLaunch = std::function<hipError_t(unsigned long long*, const uint64_t*, uint64_t*)>;
// out null: the count pass (counts[n_ranks] per destination, kept); else the
// pack of those entries into out, destination by destination.
int gxs_pack(gsx_engine* e, uint64_t* counts, uint64_t* out, const GxsLaunch& launch) {
    const uint32_t R = std::max<uint32_t>(e->n_ranks, 1);
    if (!out) {
        HIPCHK(e, hipMemsetAsync(e->d_gxs_cnt, 0, 8 * (size_t)R, e->stream));
        HIPCHK(e, launch(e->d_gxs_cnt, nullptr, nullptr));
        e->gxs_counts.assign(R, 0);
        HIPCHK(e, hipMemcpyAsync(e->gxs_counts.data(), e->d_gxs_cnt, 8 * (size_t)R, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (counts) std::memcpy(counts, e->gxs_counts.data(), 8 * (size_t)R);
        return GSX_OK;
    }
    if (e->gxs_counts.size() != R) return fail(e, GSX_ESTATE, "the count pass (out null) first");
    std::vector<uint64_t> off(R);
    uint64_t tot = 0;
    for (uint32_t d = 0; d < R; ++d) {
        off[d] = tot;
        tot += e->gxs_counts[d];
    }
    HIPCHK(e, hipMemcpyAsync(e->d_gxs_off, off.data(), 8 * (size_t)R, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_gxs_cnt, 0, 8 * (size_t)R, e->stream));
    if (tot) HIPCHK(e, launch(e->d_gxs_cnt, e->d_gxs_off, out));
    HIPCHK(e, hipStreamSynchronize(e->stream));  // `off` is on the host stack
    e->gxs_counts.clear();
    return GSX_OK;
}
}  // namespace

int gsx_gx_pending(gsx_engine* e, uint32_t* n_sets) {
    if (!e || !n_sets) return GSX_EINVAL;
    *n_sets = e->gxr.pending ? (uint32_t)e->gxr.sets.size() : 0u;
    return e->gxr.pending ? 1 : 0;
}

int gsx_gx_common(gsx_engine* e, uint64_t* common) {
    if (!e || !common) return GSX_EINVAL;
    if (int rc = gxs_step(e, 1)) return rc;
    const size_t n = 64 * e->gxr.sets.size();
    if (n) HIPCHK(e, hipMemcpyAsync(common, e->d_gx_common, 8 * n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_gx_set_common(gsx_engine* e, const uint64_t* common) {
    if (!e || !common) return GSX_EINVAL;
    if (int rc = gxs_step(e, 1)) return rc;
    const size_t n = 64 * e->gxr.sets.size();
    if (n) HIPCHK(e, hipMemcpy(e->d_gx_common, common, 8 * n, hipMemcpyHostToDevice));
    if (int rc = gx_ready(e, e->gxr)) return rc;
    e->gxr.stage = 2;
    return GSX_OK;
}

int gsx_gx_pack_ihave(gsx_engine* e, uint64_t* send) {
    if (!e || (e->n_send && !send)) return GSX_EINVAL;
    if (int rc = gxs_step(e, 2)) return rc;
    HIPCHK(e, gsx::launch_gxs_pack_ihave(dev_state(e), e->gxr.h, gxs_plan(e), send, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_gx_recv_ihave(gsx_engine* e, const uint64_t* recv) {
    if (!e || (e->n_recv && !recv)) return GSX_EINVAL;
    if (int rc = gxs_step(e, 2)) return rc;
    HIPCHK(e, gsx::launch_gxs_recv_ihave(e->gxr.h, recv, e->d_halo_pair, e->n_recv, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->gxr.stage = 3;
    return GSX_OK;
}

int gsx_gx_rows_words(gsx_engine* e, uint32_t* words) {
    if (!e || !words) return GSX_EINVAL;
    if (int rc = gxs_step(e, -1)) return rc;
    *words = 1 + e->gxr.fw * (e->gxr.h.gxs_vin ? 2u : 1u);  // (gxs_ew)
    return GSX_OK;
}

int gsx_gx_rows_pack(gsx_engine* e, uint64_t* counts, uint64_t* out) {
    if (!e || (!counts && !out)) return GSX_EINVAL;
    if (int rc = gxs_step(e, 3)) return rc;
    gsx::HbState h = e->gxr.h;
    h.gxs_fw = e->gxr.fw;
    const gsx::GxsPlan P = gxs_plan(e);
    return gxs_pack(e, counts, out, [&](unsigned long long* c, const uint64_t* off, uint64_t* out) {
        return gsx::launch_gxs_rows(h, P, e->d_gx, e->gxr.n_gx, c, off, out, e->stream);
    });
}

int gsx_gx_rows_recv(gsx_engine* e, const uint64_t* entries, uint64_t n) {
    if (!e || (n && !entries)) return GSX_EINVAL;
    if (int rc = gxs_step(e, 3)) return rc;
    gsx::HbState& h = e->gxr.h;
    h.gxs_rows = entries;
    h.gxs_fw = e->gxr.fw;
    HIPCHK(e, gsx::launch_gxs_rows_recv(h, entries, n, e->d_halo_pair, e->stream));
    e->gxr.stage = 4;
    return GSX_OK;
}

int gsx_gx_exchange(gsx_engine* e, uint32_t* n_runs) {
    if (!e || !n_runs) return GSX_EINVAL;
    if (int rc = gxs_step(e, 4)) return rc;
    HIPCHK(e, gsx::launch_gx_exchange(dev_state(e), e->gxr.h, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));  // (the received rows are read by then)
    e->gxr.h.gxs_rows = nullptr;
    if (int rc = gxf_plan(e, e->gxr)) return rc;
    *n_runs = (uint32_t)e->gxr.runs.size();
    e->gxr.stage = 5;
    return GSX_OK;
}

int gsx_gxf_begin(gsx_engine* e, uint32_t run) {
    if (!e) return GSX_EINVAL;
    if (int rc = gxs_step(e, 5)) return rc;
    if (e->gxr.fwd_active || run >= e->gxr.runs.size()) return fail(e, GSX_ESTATE, "no such forwarding run / one in flight");
    return gxf_run_begin(e, e->gxr, run);
}

int gsx_gxf_entry_words(gsx_engine* e, uint32_t* words) {
    if (!e || !words) return GSX_EINVAL;
    if (!e->gxr.fwd_active) return fail(e, GSX_ESTATE, "gsx_gxf_begin first");
    *words = gsx::GXF_HDR + e->gxr.f.rw;
    return GSX_OK;
}

int gsx_gxf_pack_fout(gsx_engine* e, uint64_t* send) {
    if (!e || (e->n_send && !send)) return GSX_EINVAL;
    if (!e->gxr.fwd_active) return fail(e, GSX_ESTATE, "gsx_gxf_begin first");
    HIPCHK(e, gsx::launch_gxf_pack_fout(e->gxr.f, gxs_plan(e), send, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_gxf_recv_fout(gsx_engine* e, const uint64_t* recv) {
    if (!e || (e->n_recv && !recv)) return GSX_EINVAL;
    if (!e->gxr.fwd_active) return fail(e, GSX_ESTATE, "gsx_gxf_begin first");
    HIPCHK(e, gsx::launch_gxf_recv_fout(e->gxr.f, recv, e->d_halo_pair, e->n_recv, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_gxf_pack(gsx_engine* e, uint32_t hop, uint64_t* counts, uint64_t* out) {
    if (!e || (!counts && !out)) return GSX_EINVAL;
    if (!e->gxr.fwd_active) return fail(e, GSX_ESTATE, "gsx_gxf_begin first");
    if (hop == 0 || hop >= gsx::GXF_MAX_HOPS) return fail(e, GSX_ERANGE, "hop out of range");
    const gsx::GxsPlan P = gxs_plan(e);
    const gsx::GxFwd f = e->gxr.f;
    const gsx::HbState h = e->gxr.h;
    return gxs_pack(e, counts, out, [&](unsigned long long* c, const uint64_t* off, uint64_t* out) {
        return gsx::launch_gxf_halo(h, f, P, hop, c, off, out, e->stream);
    });
}

int gsx_gxf_pack_dev(gsx_engine* e, uint32_t hop, uint64_t* out, int64_t* d_counts) {
    if (!e || !d_counts || (e->n_send && !out)) return GSX_EINVAL;
    if (!e->gxr.fwd_active) return fail(e, GSX_ESTATE, "gsx_gxf_begin first");
    if (hop == 0 || hop >= gsx::GXF_MAX_HOPS) return fail(e, GSX_ERANGE, "hop out of range");
    const uint32_t R = std::max<uint32_t>(e->n_ranks, 1);
    HIPCHK(e, hipMemsetAsync(e->d_gxs_cnt, 0, 8 * (size_t)R, e->stream));
    if (e->n_send)  // destination d's entries from its dense segment's first slot (send_base[d]) on
        HIPCHK(e, gsx::launch_gxf_halo(e->gxr.h, e->gxr.f, gxs_plan(e), hop, e->d_gxs_cnt, e->d_send_base, out,
                                       e->stream));
    HIPCHK(e, gsx::launch_gxf_pack_counts(e->d_gxs_cnt, e->gxr.f.fcnt + hop - 1, R, d_counts, e->stream));
    return GSX_OK;
}

int gsx_gxf_step(gsx_engine* e, uint32_t hop, const uint64_t* entries, uint64_t n, uint64_t* n_front) {
    if (!e || (n && !entries)) return GSX_EINVAL;
    if (!e->gxr.fwd_active) return fail(e, GSX_ESTATE, "gsx_gxf_begin first");
    if (hop == 0 || hop >= gsx::GXF_MAX_HOPS) return fail(e, GSX_ERANGE, "hop out of range");
    gsx::GxFwd& f = e->gxr.f;
    f.hent = entries;
    HIPCHK(e, gsx::launch_gxf_halo_recv(e->gxr.h, f, hop, entries, n, e->d_halo_pair, e->d_halo_node, e->stream));
    HIPCHK(e, gsx::launch_gxf_hop(dev_state(e), e->gxr.h, f, hop, e->stream));
    f.hent = nullptr;  // (the launches hold it; the caller keeps the entries until they ran)
    e->gxr.hops = std::max(e->gxr.hops, hop + 1);
    if (!n_front) return GSX_OK;
    HIPCHK(e, hipMemcpyAsync(e->h_gxf_cnt, e->d_gxf_cnt + hop, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    *n_front = *e->h_gxf_cnt;
    return GSX_OK;
}

int gsx_gxf_end(gsx_engine* e) {
    if (!e) return GSX_EINVAL;
    if (!e->gxr.fwd_active) return fail(e, GSX_ESTATE, "gsx_gxf_begin first");
    return gxf_run_end(e, e->gxr);
}

int gsx_gx_got(gsx_engine* e, uint8_t* got) {
    if (!e || !got) return GSX_EINVAL;
    if (int rc = gxs_step(e, 5)) return rc;
    if (e->gxr.fwd_active) return fail(e, GSX_ESTATE, "a forwarding run is in flight");
    if (!e->gxr.sets.empty())
        HIPCHK(e, hipMemcpyAsync(got, e->d_gx_got, e->gxr.sets.size(), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_gx_end(gsx_engine* e, const uint8_t* got_all, gsx_heartbeat_out* out) {
    if (!e || !out || (!got_all && !e->gxr.sets.empty())) return GSX_EINVAL;
    if (int rc = gxs_step(e, 5)) return rc;
    if (e->gxr.fwd_active) return fail(e, GSX_ESTATE, "a forwarding run is in flight");
    if (int rc = gx_merge(e, e->gxr)) return rc;
    return hb_finish(e, e->gxr, out, got_all);
}

// ---- topic membership API (gsx.h) ------------------------------------------------

int gsx_set_subscriptions(gsx_engine* e, const uint64_t* joined) {
    if (!e || !joined) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (e->hb_active) return fail(e, GSX_ESTATE, "a stepped heartbeat is in flight");
    if (int rc = members_init(e)) return rc;
    const uint64_t all = e->T >= 64 ? ~0ull : ((1ull << e->T) - 1);
    for (uint32_t v = 0; v < e->n_nodes; ++v) e->h_sub[v] = joined[v] & all;
    HIPCHK(e, hipMemcpy(e->d_sub, e->h_sub.data(), 8 * (size_t)e->n_nodes, hipMemcpyHostToDevice));
    HIPCHK(e, gsx::launch_psub(e->d_col, e->d_sub, e->d_psub, e->E, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    ++e->mem_gen;
    return GSX_OK;
}

int gsx_export_membership(gsx_engine* e, uint64_t* joined, uint64_t* fanout, int64_t* lastpub) {
    if (!e) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (!e->members_on) {  // every node joined to every topic, no fanout
        const uint64_t all = e->T >= 64 ? ~0ull : ((1ull << e->T) - 1);
        if (joined)
            for (uint32_t v = 0; v < e->n_nodes; ++v) joined[v] = all;
        if (fanout) std::memset(fanout, 0, 8 * (size_t)e->E);
        if (lastpub) std::memset(lastpub, 0, 8 * (size_t)e->n_nodes * e->T);
        return GSX_OK;
    }
    if (joined) std::memcpy(joined, e->h_sub.data(), 8 * (size_t)e->n_nodes);
    if (fanout && e->E) HIPCHK(e, hipMemcpyAsync(fanout, e->d_fanout, 8 * (size_t)e->E, hipMemcpyDeviceToHost, e->stream));
    if (lastpub && e->n_nodes)
        HIPCHK(e, hipMemcpyAsync(lastpub, e->d_lastpub, 8 * (size_t)e->n_nodes * e->T, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

namespace {
// Join / Leave: the subscriptions are announced first, then each entry's
// mesh change (one launch per rank of the entry within its node, so one
// node's row has one lane per launch), then the peers handle the GRAFTs /
// PRUNEs ((B)) and the joiners the PRUNE answers ((C)), as in a heartbeat.
int member_round(gsx_engine* e, const uint32_t* nodes, const uint32_t* topics, size_t n, int64_t now, uint64_t seed,
                 bool leave, gsx_heartbeat_out* out) {
    if (!e || (!nodes && n) || (!topics && n) || !out) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (e->hb_active) return fail(e, GSX_ESTATE, "a stepped heartbeat is in flight");
    if (e->max_deg > gsx::HB_HUB_MAX)
        return fail(e, GSX_ERANGE, "membership changes support at most " + std::to_string(gsx::HB_HUB_MAX) + " peers per node");
    if (int rc = members_init(e)) return rc;
    for (size_t i = 0; i < n; ++i)
        if (nodes[i] >= e->n_nodes || topics[i] >= e->T) return fail(e, GSX_ERANGE, "node or topic out of range");
    e->state_changed();
    // the entries that change something, announced (a repeated entry finds it done)
    std::vector<std::vector<uint32_t>> rank_nodes, rank_topics;
    std::unordered_map<uint32_t, uint32_t> per_node;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t v = nodes[i], t = topics[i];
        const bool in = (e->h_sub[v] >> t) & 1;
        if (leave ? !in : in) continue;
        e->h_sub[v] = leave ? (e->h_sub[v] & ~(1ull << t)) : (e->h_sub[v] | (1ull << t));
        const uint32_t k = per_node[v]++;
        if (k >= rank_nodes.size()) {
            rank_nodes.emplace_back();
            rank_topics.emplace_back();
        }
        rank_nodes[k].push_back(v);
        rank_topics[k].push_back(t);
    }
    HIPCHK(e, hipMemcpy(e->d_sub, e->h_sub.data(), 8 * (size_t)e->n_nodes, hipMemcpyHostToDevice));
    HIPCHK(e, gsx::launch_psub(e->d_col, e->d_sub, e->d_psub, e->E, e->stream));
    ++e->mem_gen;
    // a heartbeat's buffers and state, without maintenance or gossip
    if (int rc = hb_begin_state(e, 0, now, seed, true)) return rc;
    gsx::HbState h = e->hb;
    const gsx::DevState ds = dev_state(e);
    for (size_t k = 0; k < rank_nodes.size(); ++k) {
        std::vector<uint32_t> lst(rank_nodes[k]);
        lst.insert(lst.end(), rank_topics[k].begin(), rank_topics[k].end());
        if (int rc = member_list(e, lst)) return rc;
        const uint32_t m = (uint32_t)rank_nodes[k].size();
        HIPCHK(e, gsx::launch_join(ds, h, e->d_mlist, e->d_mlist + m, m, leave ? 1 : 0, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));  // `lst` is reused
    }
    // the receivers' mesh sizes (the scan counts every unit) and the scores of the touched pairs
    HIPCHK(e, gsx::launch_hb_scan(ds, h, e->stream));
    HIPCHK(e, rescore_subset(e, ds, kern_params(e), h.dirty));
    e->hb_active = true;
    if (int rc = hb_recv(e, nullptr)) return rc;
    std::memset(out, 0, sizeof(*out));
    e->hb_active = false;
    HIPCHK(e, gsx::launch_hb_px(ds, e->hb, 1, e->stream));  // the answers' peer exchange (do_px)
    HIPCHK(e, gsx::launch_hb_answer(ds, e->hb, e->stream));
    e->hb_clean = !e->hb_tracing;
    HIPCHK(e, rescore_subset(e, ds, kern_params(e), h.dirty));
    unsigned long long st[gsx::HB_STAT_WORDS];
    HIPCHK(e, hipMemcpyAsync(st, e->d_hbstats, sizeof(st), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    std::memcpy(out, st, sizeof(st));
    if (gsx::hb_bulk_round(st[gsx::HB_GRAFTS], st[gsx::HB_PRUNES], e->E)) e->hb_clean = false;
    e->px_last = e->hb.pxno ? st[gsx::HB_PX_CONNECT] : 0;
    return GSX_OK;
}
}  // namespace

int gsx_join(gsx_engine* e, const uint32_t* nodes, const uint32_t* topics, size_t n, int64_t now_ns, uint64_t seed,
             gsx_heartbeat_out* out) {
    return member_round(e, nodes, topics, n, now_ns, seed, false, out);
}

int gsx_leave(gsx_engine* e, const uint32_t* nodes, const uint32_t* topics, size_t n, int64_t now_ns,
              gsx_heartbeat_out* out) {
    return member_round(e, nodes, topics, n, now_ns, 0, true, out);
}

int gsx_hb_set_tracing(gsx_engine* e, uint32_t on) {
    if (!e) return GSX_EINVAL;
    if (e->hb_active) return fail(e, GSX_ESTATE, "a stepped heartbeat is in flight");
    e->hb_tracing = on != 0;
    e->hb_clean = false;
    return GSX_OK;
}

int gsx_hb_trace_words(gsx_engine* e, uint64_t* sent_graft, uint64_t* sent_prune, uint64_t* acc_graft,
                       uint64_t* handled_prune) {
    if (!e) return GSX_EINVAL;
    if (!e->hb_tracing || !e->d_tr_acc) return fail(e, GSX_ESTATE, "no traced heartbeat (gsx_hb_set_tracing)");
    if (e->hb_active) return fail(e, GSX_ESTATE, "a stepped heartbeat is in flight");
    const size_t n = 8 * (size_t)e->E;
    if (n) {
        // (the [pair][2] control words, one column each)
        if (sent_graft)
            HIPCHK(e, hipMemcpy2DAsync(sent_graft, 8, e->d_ctl, 16, 8, e->E, hipMemcpyDeviceToHost, e->stream));
        if (sent_prune)
            HIPCHK(e, hipMemcpy2DAsync(sent_prune, 8, e->d_ctl + 1, 16, 8, e->E, hipMemcpyDeviceToHost, e->stream));
        if (acc_graft) HIPCHK(e, hipMemcpyAsync(acc_graft, e->d_tr_acc, n, hipMemcpyDeviceToHost, e->stream));
        if (handled_prune) HIPCHK(e, hipMemcpyAsync(handled_prune, e->d_tr_hp, n, hipMemcpyDeviceToHost, e->stream));
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_hb_set_px_log(gsx_engine* e, size_t cap) {
    if (!e) return GSX_EINVAL;
    if (e->hb_active) return fail(e, GSX_ESTATE, "a stepped heartbeat is in flight");
    e->px_cap = cap;
    return GSX_OK;
}

int gsx_hb_px_records(gsx_engine* e, uint32_t* out, size_t cap, size_t* n) {
    if (!e || !n || (cap && !out)) return GSX_EINVAL;
    if (e->hb_active) return fail(e, GSX_ESTATE, "a stepped heartbeat is in flight");
    const size_t kept = std::min<size_t>((size_t)e->px_last, std::min(e->px_cap, e->pxlog_alloc));
    *n = kept;
    if (!kept || !cap) return GSX_OK;
    std::vector<std::array<uint32_t, 4>> rec(kept);
    HIPCHK(e, hipMemcpyAsync(rec.data(), e->d_pxlog, 16 * kept, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    std::sort(rec.begin(), rec.end());
    std::memcpy(out, rec.data(), 16 * std::min(kept, cap));
    return GSX_OK;
}

int gsx_gossip_results(gsx_engine* e, uint32_t* ihave_len, uint64_t* ihave_digest) {
    if (!e) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    const size_t TE = (size_t)e->T * e->E;
    if (!e->d_ihave_slot) {  // no heartbeat yet: nothing was sent
        if (ihave_len) std::memset(ihave_len, 0, 4 * TE);
        if (ihave_digest) std::memset(ihave_digest, 0, 8 * TE);
        return GSX_OK;
    }
    // per (topic, pair): this round's byte tag says whether the pair's owner sent
    // an IHAVE and where its (hash, len) is: the unit's record, or (IHAVE_OWN) a
    // truncated list's subset in the pair's own slot
    const size_t TN = 2 * (size_t)e->T * e->n_nodes;  // (the mesh pass's units, then the fanout pass's)
    std::vector<gsx::IhaveSlot> sl(TE), un(TN);
    std::vector<uint8_t> tg(TE);
    if (TE) {
        HIPCHK(e, hipMemcpyAsync(sl.data(), e->d_ihave_slot, sizeof(gsx::IhaveSlot) * TE, hipMemcpyDeviceToHost,
                                 e->stream));
        HIPCHK(e, hipMemcpyAsync(tg.data(), e->d_ihave_tag, TE, hipMemcpyDeviceToHost, e->stream));
    }
    if (TN) HIPCHK(e, hipMemcpyAsync(un.data(), e->d_ihave_unit, sizeof(gsx::IhaveSlot) * TN, hipMemcpyDeviceToHost,
                                     e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const uint32_t cur = e->ihave_round;  // (0: no heartbeat ran, every slot empty)
    const uint8_t cur8 = cur ? (uint8_t)((cur - 1) % gsx::IHAVE_TAG_MAX + 1) : 0;
    for (uint32_t t = 0; t < e->T; ++t)
        for (uint32_t v = 0; v < e->n_nodes; ++v)
            for (int64_t r = e->row_ptr[v]; r < e->row_ptr[v + 1]; ++r) {
                const size_t i = (size_t)t * e->E + (size_t)r;
                const uint8_t b = tg[i];
                const gsx::IhaveSlot* x = nullptr;  // (else a slot of an earlier round)
                if (cur8 && (b & gsx::IHAVE_TAG_MAX) == cur8)
                    x = (b & gsx::IHAVE_OWN) ? &sl[i]
                                             : &un[((b & gsx::IHAVE_FAN) ? (size_t)e->T : 0) * e->n_nodes +
                                                   (size_t)t * e->n_nodes + v];
                if (ihave_len) ihave_len[i] = x ? x->len : 0;
                if (ihave_digest) ihave_digest[i] = x ? x->hash : 0;
            }
    return GSX_OK;
}

int gsx_mcache_ids(gsx_engine* e, uint32_t node, uint32_t topic, uint32_t n_windows, uint64_t* out, size_t cap,
                   size_t* n_out) {
    if (!e || !n_out || (cap && !out)) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (node >= e->n_nodes) return fail(e, GSX_ERANGE, "node out of range");
    HIPCHK(e, hipStreamSynchronize(e->stream));
    size_t n = 0;
    const size_t nw = std::min<size_t>(n_windows, e->mc.size());
    std::vector<uint64_t> words;
    for (size_t w = 0; w < nw; ++w)
        for (const auto& b : e->mc[w]) {
            if (topic != GSX_ANY_TOPIC && b.topic != topic) continue;
            words.resize(b.n_words);
            // row `node` of the [node][word] bitset
            HIPCHK(e, hipMemcpy(words.data(), b.d_seen + (size_t)node * b.n_words, 8 * (size_t)b.n_words,
                                hipMemcpyDeviceToHost));
            for (uint32_t k = 0; k < b.n_msgs; ++k)
                if (words[k / 64] >> (k % 64) & 1) {
                    if (n < cap) out[n] = b.ids[k];
                    ++n;
                }
        }
    *n_out = n;
    return GSX_OK;
}

int gsx_mcache_clear(gsx_engine* e) {
    if (!e) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    mcache_clear(e);
    return GSX_OK;
}

// ---- message-parallel replicas: one batch from its message blocks (gsx.h) ----

namespace {
int mcache_ready(gsx_engine* e) {
    if (int rc = gx_busy(e)) return rc;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    if (e->sharded()) return fail(e, GSX_ESTATE, "block merging runs on unsharded engines (replicas)");
    if (e->prop.active) return fail(e, GSX_ESTATE, "a stepped propagation is in flight");
    return GSX_OK;
}
const gsx_engine::McBatch* mcache_newest(gsx_engine* e) {
    if (e->mc.empty() || e->mc.front().empty()) return nullptr;
    return &e->mc.front().back();
}
}  // namespace

int gsx_mcache_last(gsx_engine* e, uint32_t* n_words, uint32_t* n_msgs) {
    if (!e || !n_words || !n_msgs) return GSX_EINVAL;
    if (int rc = mcache_ready(e)) return rc;
    const auto* b = mcache_newest(e);
    if (!b) return fail(e, GSX_ESTATE, "the current cache window is empty");
    *n_words = b->n_words;
    *n_msgs = b->n_msgs;
    return GSX_OK;
}

int gsx_mcache_copy_last(gsx_engine* e, uint64_t* cache_rows, uint64_t* set_rows, uint64_t* code_rows,
                         uint32_t n_planes) {
    if (!e || !cache_rows || !set_rows || (n_planes && !code_rows)) return GSX_EINVAL;
    if (int rc = mcache_ready(e)) return rc;
    const auto* b = mcache_newest(e);
    if (!b || !b->set) return fail(e, GSX_ESTATE, "no cached gossipsub batch with a message set");
    if (b->set->vc_p > n_planes) return fail(e, GSX_ERANGE, "the set's validation codes need more planes");
    // a set propagated with the gossip exchange off kept no arrival hops: planes of
    // zeros would claim every copy validated at now_ns (the merged set must keep none)
    if (n_planes && !b->set->hops_kept)
        return fail(e, GSX_ESTATE, "the cached set kept no validation codes (gossip exchange off): copy it with 0 planes");
    if (int rc = vc_fence(e)) return rc;
    const size_t words = (size_t)b->n_words * e->n_nodes;
    HIPCHK(e, hipMemcpyAsync(cache_rows, b->d_seen, 8 * words, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(set_rows, b->set->d_all, 8 * words, hipMemcpyDeviceToDevice, e->stream));
    if (n_planes) {
        const uint32_t p = b->set->d_vc ? b->set->vc_p : 0u;
        if (p) HIPCHK(e, hipMemcpyAsync(code_rows, b->set->d_vc, 8 * words * p, hipMemcpyDeviceToDevice, e->stream));
        HIPCHK(e, hipMemsetAsync(code_rows + words * p, 0, 8 * words * (n_planes - p), e->stream));
    }
    return GSX_OK;
}

int gsx_mcache_pop(gsx_engine* e) {
    if (!e) return GSX_EINVAL;
    if (int rc = mcache_ready(e)) return rc;
    if (!mcache_newest(e)) return fail(e, GSX_ESTATE, "the current cache window is empty");
    auto& w = e->mc.front();
    if (w.back().set && w.back().set->serial == e->msg_serial && w.back().set->refs == 1) --e->msg_serial;
    batch_release(e, w.back());  // (the buffers go back to the pool: stream-ordered reuse)
    w.pop_back();
    return GSX_OK;
}

int gsx_mcache_put(gsx_engine* e, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg, uint32_t n_parts,
                   const uint32_t* part_msgs, const uint64_t* const* cache_parts, const uint64_t* const* set_parts,
                   const uint64_t* const* code_parts, uint32_t n_planes) {
    if (!e || !cfg || !msgs || !m || !n_parts || !part_msgs || !cache_parts || !set_parts || (n_planes && !code_parts))
        return GSX_EINVAL;
    if (n_planes > 8) return fail(e, GSX_EINVAL, "a propagated set's codes (arrival hops) take at most 8 planes");
    if (int rc = mcache_ready(e)) return rc;
    if (cfg->router != GSX_ROUTER_GOSSIPSUB) return fail(e, GSX_EINVAL, "only gossipsub batches are cached");
    if (m > 0xFFFFFFFFull) return fail(e, GSX_ERANGE, "batch too large");
    if (e->gp.gossip_exchange && m > GSX_GX_MAX_SET_MSGS)
        return fail(e, GSX_ERANGE, "batch above GSX_GX_MAX_SET_MSGS messages with the gossip exchange on");
    for (size_t k = 0; k < m; ++k) {
        if (msgs[k].source >= e->n_total) return fail(e, GSX_ERANGE, "message source out of range");
        if (msgs[k].validation > GSX_VALIDATION_THROTTLE) return fail(e, GSX_EINVAL, "bad message validation outcome");
    }
    std::vector<gsx::McPart> cp(n_parts), sp(n_parts);
    uint64_t off = 0;
    for (uint32_t k = 0; k < n_parts; ++k) {
        if (part_msgs[k] && (!cache_parts[k] || !set_parts[k])) return fail(e, GSX_EINVAL, "missing block rows");
        cp[k] = gsx::McPart{cache_parts[k], (uint32_t)off, part_msgs[k], prop_words(part_msgs[k])};
        sp[k] = gsx::McPart{set_parts[k], (uint32_t)off, part_msgs[k], prop_words(part_msgs[k])};
        off += part_msgs[k];
    }
    if (off != m) return fail(e, GSX_EINVAL, "the blocks do not add up to the batch");
    if (int rc = fanout_publish(e, msgs, m, cfg)) return rc;
    const uint32_t W = prop_words(m);
    const size_t N = e->n_nodes;
    // the blocks' descriptors (cache, set, then each code plane) on the device
    for (uint32_t b = 0; b < n_planes; ++b)
        for (uint32_t k = 0; k < n_parts; ++k) {
            if (part_msgs[k] && !code_parts[k]) return fail(e, GSX_EINVAL, "missing block codes");
            const size_t pw = (size_t)prop_words(part_msgs[k]) * e->n_nodes;
            cp.push_back(gsx::McPart{part_msgs[k] ? code_parts[k] + b * pw : nullptr, cp[k].off, part_msgs[k],
                                     prop_words(part_msgs[k])});
        }
    const size_t need = (2 + (size_t)n_planes) * (size_t)n_parts * sizeof(gsx::McPart);
    if (need > e->mparts_cap) {
        if (e->d_mparts) (void)hipFree(e->d_mparts);
        e->d_mparts = nullptr;
        e->mparts_cap = 0;
        if (int rc = dalloc(e, &e->d_mparts, need)) return rc;
        e->mparts_cap = need;
    }
    cp.insert(cp.begin() + n_parts, sp.begin(), sp.end());
    auto* dparts = reinterpret_cast<gsx::McPart*>(e->d_mparts);
    HIPCHK(e, hipMemcpyAsync(dparts, cp.data(), need, hipMemcpyHostToDevice, e->stream));
    gsx_engine::MsgSet* set = new gsx_engine::MsgSet;
    set->serial = ++e->msg_serial;
    set->n_msgs = (uint32_t)m;
    set->n_words = W;
    set->topic = cfg->topic;
    set->ids.resize(m);
    for (size_t k = 0; k < m; ++k) set->ids[k] = msgs[k].msg_id;
    set->refs = 1;
    set->all_words = (size_t)W * N;
    set->d_all = seen_acquire(e, set->all_words);
    gsx_engine::McBatch b;
    b.topic = cfg->topic;
    b.n_msgs = (uint32_t)m;
    b.n_words = W;
    b.seen_words = (size_t)W * N + 2 * N;
    b.d_seen = seen_acquire(e, b.seen_words);
    b.ids = set->ids;
    b.set = set;
    if (!set->d_all || !b.d_seen) {
        batch_release(e, b);
        return fail(e, GSX_ENOMEM, "seen rows of the merged batch");
    }
    HIPCHK(e, gsx::launch_mc_merge(dparts, n_parts, b.d_seen, (uint32_t)N, W, e->stream));
    HIPCHK(e, gsx::launch_mc_merge(dparts + n_parts, n_parts, set->d_all, (uint32_t)N, W, e->stream));
    std::vector<uint64_t> acc(W, 0), dg((size_t)W * 64 + W, 0);
    std::vector<uint32_t> vals(m);
    for (size_t k = 0; k < m; ++k) {
        vals[k] = msgs[k].validation;
        if (vals[k] == GSX_VALIDATION_ACCEPT) acc[k / 64] |= 1ull << (k % 64);
        dg[k] = id_digest(msgs[k].msg_id);
        dg[(size_t)W * 64 + k / 64] += dg[k];
    }
    if (!set_small_alloc(e, set, m, W)) {
        batch_release(e, b);
        return fail(e, GSX_ENOMEM, "message set arrays");
    }
    std::vector<uint64_t> srcs;
    set_sources(srcs, msgs, m);
    set->t0 = cfg->now_ns;
    {  // the blocks' validation codes: their arrival hops (as gsx_propagate leaves them)
        const int64_t step = cfg->hop_latency_ns + cfg->validation_delay_ns;
        set->vtime.resize(step > 0 ? (size_t)cfg->max_hops + 1 : 1);
        for (size_t h = 0; h < set->vtime.size(); ++h) set->vtime[h] = cfg->now_ns + (int64_t)h * step;
        set->n_hop = (uint32_t)set->vtime.size();
        set->hops_kept = n_planes > 0 || step <= 0;
        if (n_planes && step > 0) {
            if (int rc = vc_grow(e, set, n_planes)) {
                batch_release(e, b);
                return rc;
            }
            for (uint32_t p = 0; p < n_planes; ++p)
                HIPCHK(e, gsx::launch_mc_merge(dparts + (2 + p) * (size_t)n_parts, n_parts,
                                               set->d_vc + (size_t)p * W * N, (uint32_t)N, W, e->stream));
        }
    }
    HIPCHK(e, hipMemcpyAsync(set->d_val, vals.data(), 4 * m, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(set->d_acc, acc.data(), 8 * (size_t)W, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(set->d_dg, dg.data(), 8 * dg.size(), hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(set->d_src, srcs.data(), 8 * m, hipMemcpyHostToDevice, e->stream));
    b.d_dig = b.d_seen + (size_t)W * N;
    b.d_cnt = reinterpret_cast<uint32_t*>(b.d_seen + (size_t)W * N + N);
    HIPCHK(e, gsx::launch_mc_summary(b.d_seen, (uint32_t)N, W, (uint32_t)m, set->d_dg, set->d_dg + (size_t)W * 64,
                                     b.d_dig, b.d_cnt, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));  // the host vectors above
    if (e->mc.empty()) e->mc.emplace_back();
    e->mc.front().push_back(std::move(b));
    return GSX_OK;
}

int gsx_export_backoff(gsx_engine* e, int64_t* out) {
    if (!e || !out) return GSX_EINVAL;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    const size_t TE = (size_t)e->T * e->E;
    if (TE) HIPCHK(e, hipMemcpyAsync(out, e->d_backoff, 8 * TE, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

int gsx_import_backoff(gsx_engine* e, const int64_t* in) {
    if (!e || !in) return GSX_EINVAL;
    if (int rc = gx_busy(e)) return rc;
    if (!e->loaded) return fail(e, GSX_ESTATE, "no overlay loaded");
    const size_t TE = (size_t)e->T * e->E;
    if (TE) HIPCHK(e, hipMemcpyAsync(e->d_backoff, in, 8 * TE, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, gsx::launch_bo_rebuild(e->d_backoff, e->d_bo8, e->E, e->T, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return GSX_OK;
}

}  // extern "C"
