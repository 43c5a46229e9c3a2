/*
 * gsx_oracle.c — CPU restatement of /root/reference/score.go and
 * score_params.go.  TEST INFRASTRUCTURE ONLY (see gsx_oracle.h).
 *
 * Compile with -ffp-contract=off: every expression below is evaluated as the
 * reference writes it, one IEEE binary64 rounding per operation.
 */
#include "gsx_oracle.h"

#include <math.h>
#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

#define TIME_CACHE_DURATION_NS (120LL * 1000000000LL) /* pubsub.go:30 */
#include <stdio.h>
#include <time.h>
/* ORC_PROF=1: wall time of the heartbeat's phases on stderr (checker tuning only) */
static void orc_prof(const char* what) {
    static int on = -1;
    static double last = 0;
    if (on < 0) on = getenv("ORC_PROF") != NULL;
    if (!on) return;
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    const double t = ts.tv_sec + 1e-9 * ts.tv_nsec;
    if (what) fprintf(stderr, "[orc] %-12s %8.3f s\n", what, t - last);
    last = t;
}

/* topicStats, score.go:37-62 */
typedef struct {
    bool in_mesh;
    int64_t graft_time;
    int64_t mesh_time;
    double first_message_deliveries;
    double mesh_message_deliveries;
    bool mesh_message_deliveries_active;
    double mesh_failure_penalty;
    double invalid_message_deliveries;
} orc_topic_stats;

/* peerStats, score.go:17-35 (topics live in orc_engine.ts[pair*T + t]) */
typedef struct {
    bool present; /* the map entry ps.peerStats[p] exists */
    bool connected;
    int64_t expire;
    double behaviour_penalty;
} orc_peer_stats;

/* deliveryRecord + deliveryEntry, score.go:98-109 */
enum { DELIVERY_UNKNOWN = 0, DELIVERY_VALID, DELIVERY_INVALID, DELIVERY_IGNORED, DELIVERY_THROTTLED };

typedef struct {
    uint32_t obs;
    uint64_t msg;
    int status;
    int64_t first_seen;
    int64_t validated; /* 0 == time.Time{} (IsZero) only before validation */
    bool validated_set;
    int64_t expire;
    uint64_t* peers; /* set of pairs; NULL after `drec.peers = nil` */
    size_t n_peers, cap_peers;
    bool peers_nil;
    bool alive;
    int64_t hnext; /* hash chain */
    int64_t qnext; /* per-observer gc queue */
} orc_record;

/* ps.peerIPs (score.go:73-74) restated as an open-addressing map
 * (observer << 32 | ip) -> number of tracked peers of that observer on ip. */
typedef struct {
    uint64_t* keys;
    uint32_t* vals;
    size_t cap, used;
} ipcount_map;

struct orc_engine;
static int ipcount_init(struct orc_engine* o);

/* The messages of one gsx_propagate call: validation outcome and, per
 * (message, node), whether the node has seen it (first receipt or publish,
 * and receipts through the gossip exchange); shared by the batch that cached
 * them and by the batches of copies recovered later (reference counted). */
typedef struct {
    uint32_t serial, m, n, refs;
    uint32_t* val;
    uint32_t* src; /* [message] the publishing node (the origin, excluded by forwarding) */
    int64_t t0;    /* now_ns of the call that made the set */
    uint8_t* seen;
    /* when each node's copy finished validating (score.go:944-974 keeps
     * drec.validated per (observer, message)): [node * m + k] a code into
     * vtime; the call's copies have code = arrival hop (validated at t0 + hop
     * * (hop_latency + validation_delay), the source at t0), every exchange
     * round that recovered copies of the set appends the code of its `now` */
    uint16_t* vcode;
    int64_t* vtime;
    uint32_t n_vtime;
} orc_msgset;
typedef struct {
    uint32_t topic, m, n;
    uint64_t* ids;
    uint8_t* has; /* [k * n + v]: in v's cache (mcache membership) */
    orc_msgset* set;
} orc_mc_batch;
typedef struct {
    uint64_t q, handle; /* the asker's pair (u -> v); message set serial << 32 | index */
    int64_t expire;
    uint64_t used; /* slot occupied (open addressing, backward-shift deletion) */
} orc_promise;
typedef struct orc_mc_window {
    orc_mc_batch* b;
    size_t nb, cap;
} orc_mc_window;
#define ORC_MC_MAX 64

struct orc_engine {
    uint32_t T;
    ipcount_map ipc;
    int64_t last_refresh; /* now of the last refreshScores() (state view only) */
    gsx_thresholds th;
    uint8_t* eflags; /* GSX_EDGE_* per pair */
    int64_t* backoff; /* gs.backoff[topic][peer] per [t][pair], 0 = no entry (gossipsub.go:436) */
    /* mcache (mcache.go): window w holds the gossipsub batches Put while it was
     * window 0; node v has message k of a batch iff has[v * m + k] (node-major) */
    struct orc_mc_window* mc;
    uint32_t mc_n; /* windows alive (history[0..mc_n-1]) */
    uint32_t* ihave_len;   /* [t][pair] of the last heartbeat */
    uint64_t* ihave_hash;
    /* the last heartbeat's tracer Graft / Prune calls, topic bits per pair
     * (gsx_hb_trace_words): sent GRAFT, sent PRUNE, accepted GRAFT, handled PRUNE */
    uint64_t *tr_sg, *tr_sp, *tr_ag, *tr_hp;
    /* gossip exchange state: peerhave / iasked per pair (gossipsub.go:414-415),
     * the promises of gossipTracer (gossip_tracer.go:24-27) and mcache.peertx
     * (mcache.go:40) as (responder pair, handle) -> count */
    uint32_t *peerhave, *iasked;
    orc_promise* prom; /* hash table keyed (pair, handle): promises[mid][p] of one router per observer */
    size_t n_prom, cap_prom;
    uint32_t* prom_node; /* [node]: promises its router keeps (fulfillPromise skips nodes with none) */
    /* the truncated IHAVE lists of the last heartbeat (gsx.h, emitGossip): per
     * topic, the row of each (topic, pair) sent one (sub_idx[t][pair], UINT32_MAX
     * none; allocated on first use) in a pool of sub_tw[t]-word bitmasks over the
     * topic's gossip positions (the windows' batches in GetGossipIDs order) */
    uint32_t* sub_idx[GSX_MAX_TOPICS];
    uint64_t* sub_rows[GSX_MAX_TOPICS];
    size_t sub_n[GSX_MAX_TOPICS], sub_cap[GSX_MAX_TOPICS]; /* rows handed out; words allocated */
    uint32_t sub_tw[GSX_MAX_TOPICS];
    uint64_t* ptx_key; /* (pair << 0) ^ handle mixed; open addressing */
    uint64_t* ptx_pair;
    uint32_t* ptx_cnt;
    size_t ptx_cap, ptx_n;
    uint32_t msg_serial;
    /* topic membership (A13): joined topics per node (gs.mesh[topic] exists;
     * its neighbours know it: gs.p.topics), fanout (gs.fanout, gs.lastpub) */
    uint64_t* sub;     /* [node] */
    uint64_t* fanout;  /* [pair]: topics whose fanout holds the peer */
    uint64_t* fan_has; /* [node]: topics with a fanout entry */
    int64_t* lastpub;  /* [node][topic] */
    /* peer exchange (do_px) during orc_heartbeat: per pair bit 0 = (A) pruned it
     * without PX, bit 1 = its (B) answers go without PX (NULL otherwise); the
     * round's connection candidates (receiver, candidate, pruner, topic | kind << 8) */
    uint8_t* pxno;
    uint32_t* pxlog;
    size_t n_px, cap_px;
    uint64_t px_tick, px_seed;
    gsx_gossipsub_params gp; /* for Publish / Join (D, fanout) */
    gsx_peer_score_params pp;
    gsx_topic_score_params tp[GSX_MAX_TOPICS];
    bool scored[GSX_MAX_TOPICS]; /* ps.params.Topics[topic] exists */

    uint32_t n_nodes;
    uint64_t E;
    int64_t* row_ptr;
    int32_t* col;
    uint32_t* node_ips;
    uint32_t* pair_ip; /* [pair][2]: the IP list the observer holds for the peer (peerStats.ips) */
    uint32_t* pair_obs;

    orc_peer_stats* ps;
    orc_topic_stats* ts;
    double* app;

    uint32_t* whitelist;
    size_t n_whitelist;

    /* delivery records */
    orc_record* recs;
    size_t n_recs, cap_recs;
    int64_t* buckets;
    size_t n_buckets;
    int64_t* q_head;
    int64_t* q_tail;
    uint64_t n_alive;

    /* duplicate receipts of the last propagation (orc_prop_set_dup_tracking):
     * [pair (u -> v)][word] bit per message v sent u after u had it */
    bool dup_track;
    uint64_t* dup_rows;
    size_t dup_words;
    uint64_t dup_E;
};

/* ------------------------------------------------------------------------ */
/* score_params.go                                                          */

/* isInvalidNumber, score_params.go:291-293 */
static bool invalid_number(double x) { return isnan(x) || isinf(x); }

/* PeerScoreThresholds.validate, score_params.go:34-51 */
int orc_validate_thresholds(const gsx_thresholds* p) {
    if (p->gossip_threshold > 0 || invalid_number(p->gossip_threshold)) return GSX_EINVAL;
    if (p->publish_threshold > 0 || p->publish_threshold > p->gossip_threshold ||
        invalid_number(p->publish_threshold))
        return GSX_EINVAL;
    if (p->graylist_threshold > 0 || p->graylist_threshold > p->publish_threshold ||
        invalid_number(p->graylist_threshold))
        return GSX_EINVAL;
    if (p->accept_px_threshold < 0 || invalid_number(p->accept_px_threshold)) return GSX_EINVAL;
    if (p->opportunistic_graft_threshold < 0 || invalid_number(p->opportunistic_graft_threshold))
        return GSX_EINVAL;
    return 0;
}

/* PeerScoreParams.validate, score_params.go:151-198 (topic loop 152-157 is
 * orc_validate_topic_params per topic, done by the caller). */
int orc_validate_peer_params(const gsx_peer_score_params* p) {
    if (p->topic_score_cap < 0 || invalid_number(p->topic_score_cap)) return GSX_EINVAL;
    if (!p->app_specific_score_set) return GSX_EINVAL;
    if (p->ip_colocation_factor_weight > 0 || invalid_number(p->ip_colocation_factor_weight)) return GSX_EINVAL;
    if (p->ip_colocation_factor_weight != 0 && p->ip_colocation_factor_threshold < 1) return GSX_EINVAL;
    if (p->behaviour_penalty_weight > 0 || invalid_number(p->behaviour_penalty_weight)) return GSX_EINVAL;
    if (p->behaviour_penalty_weight != 0 &&
        (p->behaviour_penalty_decay <= 0 || p->behaviour_penalty_decay >= 1 ||
         invalid_number(p->behaviour_penalty_decay)))
        return GSX_EINVAL;
    if (p->behaviour_penalty_threshold < 0 || invalid_number(p->behaviour_penalty_threshold)) return GSX_EINVAL;
    if (p->decay_interval_ns < 1000000000LL) return GSX_EINVAL;
    if (p->decay_to_zero <= 0 || p->decay_to_zero >= 1 || invalid_number(p->decay_to_zero)) return GSX_EINVAL;
    return 0;
}

/* TopicScoreParams.validate, score_params.go:200-268 */
int orc_validate_topic_params(const gsx_topic_score_params* p) {
    if (p->topic_weight < 0 || invalid_number(p->topic_weight)) return GSX_EINVAL;
    /* P1 */
    if (p->time_in_mesh_quantum_ns == 0) return GSX_EINVAL;
    if (p->time_in_mesh_weight < 0 || invalid_number(p->time_in_mesh_weight)) return GSX_EINVAL;
    if (p->time_in_mesh_weight != 0 && p->time_in_mesh_quantum_ns <= 0) return GSX_EINVAL;
    if (p->time_in_mesh_weight != 0 && (p->time_in_mesh_cap <= 0 || invalid_number(p->time_in_mesh_cap)))
        return GSX_EINVAL;
    /* P2 */
    if (p->first_message_deliveries_weight < 0 || invalid_number(p->first_message_deliveries_weight))
        return GSX_EINVAL;
    if (p->first_message_deliveries_weight != 0 &&
        (p->first_message_deliveries_decay <= 0 || p->first_message_deliveries_decay >= 1 ||
         invalid_number(p->first_message_deliveries_decay)))
        return GSX_EINVAL;
    if (p->first_message_deliveries_weight != 0 &&
        (p->first_message_deliveries_cap <= 0 || invalid_number(p->first_message_deliveries_cap)))
        return GSX_EINVAL;
    /* P3 */
    if (p->mesh_message_deliveries_weight > 0 || invalid_number(p->mesh_message_deliveries_weight))
        return GSX_EINVAL;
    if (p->mesh_message_deliveries_weight != 0 &&
        (p->mesh_message_deliveries_decay <= 0 || p->mesh_message_deliveries_decay >= 1 ||
         invalid_number(p->mesh_message_deliveries_decay)))
        return GSX_EINVAL;
    if (p->mesh_message_deliveries_weight != 0 &&
        (p->mesh_message_deliveries_cap <= 0 || invalid_number(p->mesh_message_deliveries_cap)))
        return GSX_EINVAL;
    if (p->mesh_message_deliveries_weight != 0 &&
        (p->mesh_message_deliveries_threshold <= 0 || invalid_number(p->mesh_message_deliveries_threshold)))
        return GSX_EINVAL;
    if (p->mesh_message_deliveries_window_ns < 0) return GSX_EINVAL;
    if (p->mesh_message_deliveries_weight != 0 && p->mesh_message_deliveries_activation_ns < 1000000000LL)
        return GSX_EINVAL;
    /* P3b */
    if (p->mesh_failure_penalty_weight > 0 || invalid_number(p->mesh_failure_penalty_weight)) return GSX_EINVAL;
    if (p->mesh_failure_penalty_weight != 0 &&
        (invalid_number(p->mesh_failure_penalty_decay) || p->mesh_failure_penalty_decay <= 0 ||
         p->mesh_failure_penalty_decay >= 1))
        return GSX_EINVAL;
    /* P4 */
    if (p->invalid_message_deliveries_weight > 0 || invalid_number(p->invalid_message_deliveries_weight))
        return GSX_EINVAL;
    if (p->invalid_message_deliveries_decay <= 0 || p->invalid_message_deliveries_decay >= 1 ||
        invalid_number(p->invalid_message_deliveries_decay))
        return GSX_EINVAL;
    return 0;
}

/* ScoreParameterDecayWithBase, score_params.go:282-287: `decay / base` is a
 * Duration (int64) division, truncating. */
double orc_score_parameter_decay_with_base(int64_t decay_ns, int64_t base_ns, double decay_to_zero) {
    double ticks = (double)(decay_ns / base_ns);
    return pow(decay_to_zero, 1 / ticks);
}

/* ScoreParameterDecay, score_params.go:277-279 (DefaultDecayInterval 1s,
 * DefaultDecayToZero 0.01, :270-273) */
double orc_score_parameter_decay(int64_t decay_ns) {
    return orc_score_parameter_decay_with_base(decay_ns, 1000000000LL, 0.01);
}

/* ------------------------------------------------------------------------ */
/* engine                                                                   */

orc_engine* orc_create(uint32_t n_topics) {
    if (n_topics == 0 || n_topics > GSX_MAX_TOPICS) return NULL;
    orc_engine* o = (orc_engine*)calloc(1, sizeof(orc_engine));
    if (!o) return NULL;
    o->T = n_topics;
    orc_default_gossipsub_params(&o->gp);
    return o;
}

static void free_records(orc_engine* o) {
    for (size_t i = 0; i < o->n_recs; i++) free(o->recs[i].peers);
    free(o->recs);
    free(o->buckets);
    free(o->q_head);
    free(o->q_tail);
    o->recs = NULL;
    o->buckets = NULL;
    o->q_head = o->q_tail = NULL;
    o->n_recs = o->cap_recs = 0;
    o->n_alive = 0;
}

static void batch_free(orc_mc_batch* b) {
    free(b->ids);
    free(b->has);
    if (b->set && --b->set->refs == 0) {
        free(b->set->val);
        free(b->set->src);
        free(b->set->seen);
        free(b->set->vcode);
        free(b->set->vtime);
        free(b->set);
    }
    b->set = NULL;
}

int orc_mcache_clear(orc_engine* o) {
    for (uint32_t w = 0; w < o->mc_n; w++) {
        for (size_t i = 0; i < o->mc[w].nb; i++) batch_free(&o->mc[w].b[i]);
        free(o->mc[w].b);
        memset(&o->mc[w], 0, sizeof(orc_mc_window));
    }
    o->mc_n = o->mc ? 1 : 0; /* history[0] exists, empty */
    return 0;
}

void orc_destroy(orc_engine* o) {
    if (!o) return;
    free(o->row_ptr);
    free(o->col);
    free(o->node_ips);
    free(o->pair_ip);
    free(o->pair_obs);
    free(o->ps);
    free(o->ts);
    free(o->app);
    free(o->whitelist);
    free(o->eflags);
    free(o->backoff);
    free(o->dup_rows);
    orc_mcache_clear(o);
    free(o->mc);
    free(o->ihave_len);
    free(o->ihave_hash);
    free(o->tr_sg);
    free(o->tr_sp);
    free(o->tr_ag);
    free(o->tr_hp);
    free(o->peerhave);
    free(o->iasked);
    free(o->sub);
    free(o->fanout);
    free(o->fan_has);
    free(o->lastpub);
    free(o->pxlog);
    free(o->prom);
    free(o->prom_node);
    for (int t = 0; t < GSX_MAX_TOPICS; t++) {
        free(o->sub_idx[t]);
        free(o->sub_rows[t]);
    }
    free(o->ptx_key);
    free(o->ptx_pair);
    free(o->ptx_cnt);
    free(o->ipc.keys);
    free(o->ipc.vals);
    free_records(o);
    free(o);
}

uint64_t orc_num_pairs(orc_engine* o) { return o->E; }

int orc_set_peer_params(orc_engine* o, const gsx_peer_score_params* p) {
    o->pp = *p;
    return 0;
}

/* SetTopicScoreParams, score.go:194-234 */
int orc_set_topic_params(orc_engine* o, uint32_t topic, const gsx_topic_score_params* p) {
    if (topic >= o->T) return GSX_ERANGE;
    bool exist = o->scored[topic];
    gsx_topic_score_params old = o->tp[topic];
    o->tp[topic] = *p;
    o->scored[topic] = true;
    if (!exist) return 0;
    bool recap = false;
    if (p->first_message_deliveries_cap < old.first_message_deliveries_cap) recap = true;
    if (p->mesh_message_deliveries_cap < old.mesh_message_deliveries_cap) recap = true;
    if (!recap) return 0;
    for (uint64_t q = 0; q < o->E; q++) {
        if (!o->ps[q].present) continue;
        orc_topic_stats* t = &o->ts[q * o->T + topic];
        if (t->first_message_deliveries > p->first_message_deliveries_cap)
            t->first_message_deliveries = p->first_message_deliveries_cap;
        if (t->mesh_message_deliveries > p->mesh_message_deliveries_cap)
            t->mesh_message_deliveries = p->mesh_message_deliveries_cap;
    }
    return 0;
}

int orc_load_overlay(orc_engine* o, uint32_t n_nodes, const int64_t* row_ptr, const int32_t* col,
                     const uint8_t* edge_flags, const uint32_t* node_ips) {
    uint64_t E = (uint64_t)row_ptr[n_nodes];
    free(o->eflags);
    o->eflags = (uint8_t*)calloc(E ? E : 1, 1);
    if (!o->eflags) return GSX_ENOMEM;
    free(o->backoff);
    o->backoff = (int64_t*)calloc((size_t)o->T * (E ? E : 1), sizeof(int64_t));
    if (!o->backoff) return GSX_ENOMEM;
    free(o->ihave_len);
    free(o->ihave_hash);
    o->ihave_len = (uint32_t*)calloc((size_t)o->T * (E ? E : 1), sizeof(uint32_t));
    o->ihave_hash = (uint64_t*)calloc((size_t)o->T * (E ? E : 1), sizeof(uint64_t));
    if (!o->ihave_len || !o->ihave_hash) return GSX_ENOMEM;
    free(o->peerhave);
    free(o->iasked);
    free(o->sub);
    free(o->fanout);
    free(o->fan_has);
    free(o->lastpub);
    o->sub = (uint64_t*)malloc(sizeof(uint64_t) * (n_nodes ? n_nodes : 1));
    o->fanout = (uint64_t*)calloc(E ? E : 1, sizeof(uint64_t));
    o->fan_has = (uint64_t*)calloc(n_nodes ? n_nodes : 1, sizeof(uint64_t));
    o->lastpub = (int64_t*)calloc((size_t)(n_nodes ? n_nodes : 1) * o->T, sizeof(int64_t));
    if (!o->sub || !o->fanout || !o->fan_has || !o->lastpub) return GSX_ENOMEM;
    for (uint32_t v = 0; v < n_nodes; v++) o->sub[v] = o->T >= 64 ? ~0ull : ((1ull << o->T) - 1); /* all joined */
    o->peerhave = (uint32_t*)calloc(E ? E : 1, sizeof(uint32_t));
    o->iasked = (uint32_t*)calloc(E ? E : 1, sizeof(uint32_t));
    if (!o->peerhave || !o->iasked) return GSX_ENOMEM;
    o->n_prom = 0;
    if (o->prom) memset(o->prom, 0, sizeof(orc_promise) * o->cap_prom);
    free(o->prom_node);
    o->prom_node = (uint32_t*)calloc(n_nodes ? n_nodes : 1, sizeof(uint32_t));
    if (!o->prom_node) return GSX_ENOMEM;
    for (int t = 0; t < GSX_MAX_TOPICS; t++) { /* per-pair rows: sized by the new overlay on first use */
        free(o->sub_idx[t]);
        o->sub_idx[t] = NULL;
        o->sub_n[t] = 0;
    }
    /* the GetForPeer counts start empty: a slot is occupied iff its count is
     * nonzero, so the counts (and keys) of the last overlay are dropped whole */
    free(o->ptx_key);
    free(o->ptx_pair);
    free(o->ptx_cnt);
    o->ptx_key = o->ptx_pair = NULL;
    o->ptx_cnt = NULL;
    o->ptx_cap = o->ptx_n = 0;
    uint64_t** tw[4] = {&o->tr_sg, &o->tr_sp, &o->tr_ag, &o->tr_hp};
    for (int i = 0; i < 4; i++) {
        free(*tw[i]);
        *tw[i] = (uint64_t*)calloc(E ? E : 1, sizeof(uint64_t));
        if (!*tw[i]) return GSX_ENOMEM;
    }
    if (!o->mc) o->mc = (orc_mc_window*)calloc(ORC_MC_MAX, sizeof(orc_mc_window));
    if (!o->mc) return GSX_ENOMEM;
    orc_mcache_clear(o);
    if (edge_flags && E) memcpy(o->eflags, edge_flags, E);
    free(o->row_ptr);
    free(o->col);
    free(o->node_ips);
    free(o->pair_obs);
    free(o->ps);
    free(o->ts);
    free(o->app);
    free_records(o);
    o->n_nodes = n_nodes;
    o->E = E;
    o->row_ptr = (int64_t*)malloc(sizeof(int64_t) * (n_nodes + 1));
    o->col = (int32_t*)malloc(sizeof(int32_t) * (E ? E : 1));
    o->node_ips = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (n_nodes ? n_nodes : 1));
    free(o->pair_ip);
    o->pair_ip = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (E ? E : 1));
    o->pair_obs = (uint32_t*)malloc(sizeof(uint32_t) * (E ? E : 1));
    o->ps = (orc_peer_stats*)calloc(E ? E : 1, sizeof(orc_peer_stats));
    o->ts = (orc_topic_stats*)calloc((E ? E : 1) * o->T, sizeof(orc_topic_stats));
    o->app = (double*)calloc(E ? E : 1, sizeof(double));
    o->q_head = (int64_t*)malloc(sizeof(int64_t) * (n_nodes ? n_nodes : 1));
    o->q_tail = (int64_t*)malloc(sizeof(int64_t) * (n_nodes ? n_nodes : 1));
    if (!o->row_ptr || !o->col || !o->node_ips || !o->pair_ip || !o->pair_obs || !o->ps || !o->ts || !o->app ||
        !o->q_head || !o->q_tail)
        return GSX_ENOMEM;
    memcpy(o->row_ptr, row_ptr, sizeof(int64_t) * (n_nodes + 1));
    if (E) memcpy(o->col, col, sizeof(int32_t) * E);
    for (uint32_t i = 0; i < n_nodes; i++) {
        o->node_ips[2 * i] = node_ips ? node_ips[2 * i] : GSX_NO_IP;
        o->node_ips[2 * i + 1] = node_ips ? node_ips[2 * i + 1] : GSX_NO_IP;
        o->q_head[i] = o->q_tail[i] = -1;
        for (int64_t p = row_ptr[i]; p < row_ptr[i + 1]; p++) o->pair_obs[p] = i;
    }
    for (uint64_t p = 0; p < E; p++)
        for (int k = 0; k < 2; k++)
            o->pair_ip[2 * p + k] = node_ips ? node_ips[2 * (size_t)col[p] + k] : GSX_NO_IP;
    if (ipcount_init(o)) return GSX_ENOMEM;
    o->n_buckets = 1024;
    o->buckets = (int64_t*)malloc(sizeof(int64_t) * o->n_buckets);
    for (size_t i = 0; i < o->n_buckets; i++) o->buckets[i] = -1;
    return 0;
}

int orc_set_ip_whitelist(orc_engine* o, const uint32_t* ip_ids, size_t n) {
    free(o->whitelist);
    o->whitelist = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    if (n) memcpy(o->whitelist, ip_ids, sizeof(uint32_t) * n);
    o->n_whitelist = n;
    return 0;
}

int orc_set_app_scores(orc_engine* o, const double* app, size_t n_pairs) {
    if (n_pairs != o->E) return GSX_EINVAL;
    memcpy(o->app, app, sizeof(double) * n_pairs);
    return 0;
}

static bool whitelisted(const orc_engine* o, uint32_t ip) {
    for (size_t i = 0; i < o->n_whitelist; i++)
        if (o->whitelist[i] == ip) return true;
    return false;
}

/* the IP list of the peer behind pair q (peerStats.ips; getIPs score.go:977-1017):
 * its node's addresses at load, or what orc_set_pair_ips set since */
static int pair_ips(const orc_engine* o, uint64_t q, uint32_t out[2]) {
    int n = 0;
    for (int k = 0; k < 2; k++) {
        uint32_t ip = o->pair_ip[2 * q + k];
        if (ip != GSX_NO_IP) out[n++] = ip;
    }
    return n;
}

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

static uint32_t* ipcount_slot(ipcount_map* m, uint64_t key, bool insert) {
    size_t i = (size_t)(mix64(key) & (m->cap - 1));
    for (;;) {
        if (m->keys[i] == key) return &m->vals[i];
        if (m->keys[i] == UINT64_MAX) {
            if (!insert) return NULL;
            m->keys[i] = key;
            m->vals[i] = 0;
            m->used++;
            return &m->vals[i];
        }
        i = (i + 1) & (m->cap - 1);
    }
}

static int ipcount_init(orc_engine* o) {
    ipcount_map* m = &o->ipc;
    free(m->keys);
    free(m->vals);
    size_t need = 2 * (size_t)o->E + 16, cap = 16;
    while (cap < 2 * need) cap <<= 1;
    m->cap = cap;
    m->used = 0;
    m->keys = (uint64_t*)malloc(sizeof(uint64_t) * cap);
    m->vals = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    if (!m->keys || !m->vals) return GSX_ENOMEM;
    memset(m->keys, 0xff, sizeof(uint64_t) * cap);
    return 0;
}

/* setIPs / removeIPs (score.go:1021-1074) for the whole IP list of pair q:
 * the peer joins (+1) or leaves (-1) each of its IPs' sets once. */
static void ipcount_add(orc_engine* o, uint64_t q, int delta) {
    uint32_t ips[2];
    int k = pair_ips(o, q, ips);
    for (int j = 0; j < k; j++) {
        if (j == 1 && ips[1] == ips[0]) continue; /* a set: the peer counts once */
        uint64_t key = ((uint64_t)o->pair_obs[q] << 32) | ips[j];
        *ipcount_slot(&o->ipc, key, true) += (uint32_t)delta;
    }
}

/* room for `more` new keys at a load factor <= 1/2 (rehash into a larger table) */
static int ipcount_reserve(orc_engine* o, size_t more) {
    ipcount_map* m = &o->ipc;
    if (2 * (m->used + more) <= m->cap) return 0;
    ipcount_map old = *m;
    size_t cap = m->cap;
    while (2 * (m->used + more) > cap) cap <<= 1;
    m->keys = (uint64_t*)malloc(sizeof(uint64_t) * cap);
    m->vals = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    if (!m->keys || !m->vals) return GSX_ENOMEM;
    memset(m->keys, 0xff, sizeof(uint64_t) * cap);
    m->cap = cap;
    m->used = 0;
    for (size_t i = 0; i < old.cap; i++)
        if (old.keys[i] != UINT64_MAX) *ipcount_slot(m, old.keys[i], true) = old.vals[i];
    free(old.keys);
    free(old.vals);
    return 0;
}

/* setIPs (score.go:1021-1059) for pairs whose peer now has other addresses
 * (refreshIPs, score.go:560-586): a present peer leaves the sets of its old
 * IPs and joins those of the new list; an absent one only records it. */
int orc_set_pair_ips(orc_engine* o, const uint64_t* pairs, const uint32_t* ips, size_t n) {
    for (size_t i = 0; i < n; i++)
        if (pairs[i] >= o->E) return GSX_ERANGE;
    if (ipcount_reserve(o, 2 * n)) return GSX_ENOMEM;
    for (size_t i = 0; i < n; i++) {
        const uint64_t q = pairs[i];
        if (o->ps[q].present) ipcount_add(o, q, -1);
        o->pair_ip[2 * q] = ips[2 * i];
        o->pair_ip[2 * q + 1] = ips[2 * i + 1];
        if (o->ps[q].present) ipcount_add(o, q, +1);
    }
    return 0;
}

/* PeerScoreSnapshot.IPColocationFactor of every pair (inspectScoresExtended, score.go:487) */
int orc_ip_colocation_factors(orc_engine* o, double* out);

static void ipcount_rebuild(orc_engine* o) {
    memset(o->ipc.vals, 0, sizeof(uint32_t) * o->ipc.cap);
    for (uint64_t q = 0; q < o->E; q++)
        if (o->ps[q].present) ipcount_add(o, q, +1);
}

/* ipColocationFactor, score.go:337-381 */
static double ip_colocation_factor(const orc_engine* o, uint64_t p) {
    if (!o->ps[p].present) return 0;
    double result = 0;
    uint32_t ips[2];
    int k = pair_ips(o, p, ips);
    uint32_t obs = o->pair_obs[p];
    for (int j = 0; j < k; j++) {
        uint32_t ip = ips[j];
        if (o->n_whitelist > 0 && whitelisted(o, ip)) continue; /* :346-367 */
        uint32_t* v = ipcount_slot((ipcount_map*)&o->ipc, ((uint64_t)obs << 32) | ip, false);
        uint32_t peers_in_ip = v ? *v : 0; /* len(ps.peerIPs[ip]) */
        if ((int64_t)peers_in_ip > (int64_t)o->pp.ip_colocation_factor_threshold) {
            double surpluss = (double)((int64_t)peers_in_ip - (int64_t)o->pp.ip_colocation_factor_threshold);
            result += surpluss * surpluss;
        }
    }
    return result;
}

int orc_ip_colocation_factors(orc_engine* o, double* out) {
    for (uint64_t p = 0; p < o->E; p++) out[p] = ip_colocation_factor(o, p);
    return 0;
}

/* score(), score.go:258-335; topics in ascending index order */
static double score_pair(const orc_engine* o, uint64_t p) {
    const orc_peer_stats* pstats = &o->ps[p];
    if (!pstats->present) return 0;
    double score = 0;
    for (uint32_t t = 0; t < o->T; t++) {
        if (!o->scored[t]) continue; /* :269-273 */
        const gsx_topic_score_params* tp = &o->tp[t];
        const orc_topic_stats* ts = &o->ts[p * o->T + t];
        double topic_score = 0;
        /* P1 :279-285 — integer Duration division */
        if (ts->in_mesh) {
            double p1 = (double)(ts->mesh_time / tp->time_in_mesh_quantum_ns);
            if (p1 > tp->time_in_mesh_cap) p1 = tp->time_in_mesh_cap;
            topic_score += p1 * tp->time_in_mesh_weight;
        }
        /* P2 :288-289 */
        double p2 = ts->first_message_deliveries;
        topic_score += p2 * tp->first_message_deliveries_weight;
        /* P3 :292-298 */
        if (ts->mesh_message_deliveries_active) {
            if (ts->mesh_message_deliveries < tp->mesh_message_deliveries_threshold) {
                double deficit = tp->mesh_message_deliveries_threshold - ts->mesh_message_deliveries;
                double p3 = deficit * deficit;
                topic_score += p3 * tp->mesh_message_deliveries_weight;
            }
        }
        /* P3b :302-303 */
        double p3b = ts->mesh_failure_penalty;
        topic_score += p3b * tp->mesh_failure_penalty_weight;
        /* P4 :307-308 */
        double p4 = (ts->invalid_message_deliveries * ts->invalid_message_deliveries);
        topic_score += p4 * tp->invalid_message_deliveries_weight;
        /* :311 */
        score += topic_score * tp->topic_weight;
    }
    /* :315-317 */
    if (o->pp.topic_score_cap > 0 && score > o->pp.topic_score_cap) score = o->pp.topic_score_cap;
    /* P5 :320-321 */
    double p5 = o->app[p];
    score += p5 * o->pp.app_specific_weight;
    /* P6 :324-325 */
    double p6 = ip_colocation_factor(o, p);
    score += p6 * o->pp.ip_colocation_factor_weight;
    /* P7 :328-332 */
    if (pstats->behaviour_penalty > o->pp.behaviour_penalty_threshold) {
        double excess = pstats->behaviour_penalty - o->pp.behaviour_penalty_threshold;
        double p7 = excess * excess;
        score += p7 * o->pp.behaviour_penalty_weight;
    }
    return score;
}

double orc_score(orc_engine* o, uint64_t pair) {
    if (pair >= o->E) return 0;
    return score_pair(o, pair);
}

int orc_scores(orc_engine* o, double* out, size_t n_pairs) {
    if (n_pairs != o->E) return GSX_EINVAL;
    for (uint64_t p = 0; p < o->E; p++) out[p] = score_pair(o, p);
    return 0;
}

/* one pair's share of refreshScores, score.go:502-557 (purge handled by caller) */
static void refresh_pair(orc_engine* o, uint64_t p, int64_t now) {
    orc_peer_stats* pstats = &o->ps[p];
    for (uint32_t t = 0; t < o->T; t++) {
        if (!o->scored[t]) continue; /* :520-524 */
        const gsx_topic_score_params* tp = &o->tp[t];
        orc_topic_stats* ts = &o->ts[p * o->T + t];
        /* :527-542 */
        ts->first_message_deliveries *= tp->first_message_deliveries_decay;
        if (ts->first_message_deliveries < o->pp.decay_to_zero) ts->first_message_deliveries = 0;
        ts->mesh_message_deliveries *= tp->mesh_message_deliveries_decay;
        if (ts->mesh_message_deliveries < o->pp.decay_to_zero) ts->mesh_message_deliveries = 0;
        ts->mesh_failure_penalty *= tp->mesh_failure_penalty_decay;
        if (ts->mesh_failure_penalty < o->pp.decay_to_zero) ts->mesh_failure_penalty = 0;
        ts->invalid_message_deliveries *= tp->invalid_message_deliveries_decay;
        if (ts->invalid_message_deliveries < o->pp.decay_to_zero) ts->invalid_message_deliveries = 0;
        /* :544-549 */
        if (ts->in_mesh) {
            ts->mesh_time = now - ts->graft_time;
            if (ts->mesh_time > tp->mesh_message_deliveries_activation_ns) ts->mesh_message_deliveries_active = true;
        }
    }
    /* :553-556 */
    pstats->behaviour_penalty *= o->pp.behaviour_penalty_decay;
    if (pstats->behaviour_penalty < o->pp.decay_to_zero) pstats->behaviour_penalty = 0;
}

/* refreshScores, score.go:497-558 */
int orc_refresh(orc_engine* o, int64_t now) {
    o->last_refresh = now;
    for (uint64_t p = 0; p < o->E; p++) {
        orc_peer_stats* pstats = &o->ps[p];
        if (!pstats->present) continue;
        if (!pstats->connected) {
            /* :503-516 — `now.After(expire)`: removeIPs + delete */
            if (now > pstats->expire) {
                ipcount_add(o, p, -1);
                pstats->present = false;
            }
            continue;
        }
        refresh_pair(o, p, now);
    }
    return 0;
}

int orc_refresh_scores_range(orc_engine* o, int64_t now, uint64_t p0, uint64_t p1, double* out) {
    o->last_refresh = now;
    if (p1 > o->E) p1 = o->E;
    for (uint64_t p = p0; p < p1; p++) {
        orc_peer_stats* pstats = &o->ps[p];
        if (!pstats->present) continue;
        if (!pstats->connected) {
            if (now > pstats->expire) {
                ipcount_add(o, p, -1);
                pstats->present = false;
            }
            continue;
        }
        refresh_pair(o, p, now);
    }
    for (uint64_t p = p0; p < p1; p++) out[p - p0] = score_pair(o, p);
    return 0;
}

/* refreshScores + score() over every pair with n_threads OpenMP threads (the
 * bench's multi-core CPU baseline).  The purge (removeIPs changes the shared
 * per-observer IP counts) runs first and serially; then every connected pair
 * decays its own counters and is scored, independently of the others (the
 * IP counts are only read).  Same results as orc_refresh + orc_scores. */
int orc_refresh_scores_parallel(orc_engine* o, int64_t now, double* out, int n_threads) {
    o->last_refresh = now;
    for (uint64_t p = 0; p < o->E; p++) {
        orc_peer_stats* pstats = &o->ps[p];
        if (pstats->present && !pstats->connected && now > pstats->expire) {
            ipcount_add(o, p, -1);
            pstats->present = false;
        }
    }
    const int64_t E = (int64_t)o->E;
#pragma omp parallel for num_threads(n_threads) schedule(static, 4096)
    for (int64_t p = 0; p < E; p++) {
        if (o->ps[p].present && o->ps[p].connected) refresh_pair(o, (uint64_t)p, now);
        out[p] = score_pair(o, (uint64_t)p);
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* tracer events, score.go:588-974                                          */

/* getTopicStats, score.go:875-890: records of scored topics always exist in
 * this dense model; an unscored topic has none. */
static orc_topic_stats* topic_stats(orc_engine* o, uint64_t p, uint32_t topic) {
    if (topic >= o->T || !o->scored[topic]) return NULL;
    return &o->ts[p * o->T + topic];
}

/* AddPeer, score.go:588-602 */
static void add_peer(orc_engine* o, uint64_t p) {
    orc_peer_stats* pstats = &o->ps[p];
    if (!pstats->present) {
        memset(pstats, 0, sizeof(*pstats));
        memset(&o->ts[p * o->T], 0, sizeof(orc_topic_stats) * o->T);
        pstats->present = true;
        ipcount_add(o, p, +1); /* setIPs: the IPs now count for this observer */
    }
    pstats->connected = true;
}

/* RemovePeer, score.go:604-637 */
static void remove_peer(orc_engine* o, uint64_t p, int64_t now) {
    orc_peer_stats* pstats = &o->ps[p];
    if (!pstats->present) return;
    if (score_pair(o, p) > 0) { /* :615-619 */
        ipcount_add(o, p, -1);         /* removeIPs */
        pstats->present = false;       /* delete(ps.peerStats, p): the entry is gone, */
        pstats->connected = false;     /* connected with it */
        return;
    }
    for (uint32_t t = 0; t < o->T; t++) { /* :623-633 */
        orc_topic_stats* ts = topic_stats(o, p, t);
        if (!ts) continue;
        ts->first_message_deliveries = 0;
        double threshold = o->tp[t].mesh_message_deliveries_threshold;
        if (ts->in_mesh && ts->mesh_message_deliveries_active && ts->mesh_message_deliveries < threshold) {
            double deficit = threshold - ts->mesh_message_deliveries;
            ts->mesh_failure_penalty += deficit * deficit;
        }
        ts->in_mesh = false;
    }
    pstats->connected = false;
    pstats->expire = now + o->pp.retain_score_ns;
}

/* Graft, score.go:642-660 */
static void graft(orc_engine* o, uint64_t p, uint32_t topic, int64_t now) {
    if (!o->ps[p].present) return;
    orc_topic_stats* ts = topic_stats(o, p, topic);
    if (!ts) return;
    ts->in_mesh = true;
    ts->graft_time = now;
    ts->mesh_time = 0;
    ts->mesh_message_deliveries_active = false;
}

/* Prune, score.go:662-684 */
static void prune(orc_engine* o, uint64_t p, uint32_t topic) {
    if (!o->ps[p].present) return;
    orc_topic_stats* ts = topic_stats(o, p, topic);
    if (!ts) return;
    double threshold = o->tp[topic].mesh_message_deliveries_threshold;
    if (ts->mesh_message_deliveries_active && ts->mesh_message_deliveries < threshold) {
        double deficit = threshold - ts->mesh_message_deliveries;
        ts->mesh_failure_penalty += deficit * deficit;
    }
    ts->in_mesh = false;
}

/* markInvalidMessageDelivery, score.go:894-907 */
static void mark_invalid(orc_engine* o, uint64_t p, uint32_t topic) {
    if (!o->ps[p].present) return;
    orc_topic_stats* ts = topic_stats(o, p, topic);
    if (!ts) return;
    ts->invalid_message_deliveries += 1;
}

/* markFirstMessageDelivery, score.go:912-939 */
static void mark_first(orc_engine* o, uint64_t p, uint32_t topic) {
    if (!o->ps[p].present) return;
    orc_topic_stats* ts = topic_stats(o, p, topic);
    if (!ts) return;
    double cap = o->tp[topic].first_message_deliveries_cap;
    ts->first_message_deliveries += 1;
    if (ts->first_message_deliveries > cap) ts->first_message_deliveries = cap;
    if (!ts->in_mesh) return;
    cap = o->tp[topic].mesh_message_deliveries_cap;
    ts->mesh_message_deliveries += 1;
    if (ts->mesh_message_deliveries > cap) ts->mesh_message_deliveries = cap;
}

/* markDuplicateMessageDelivery, score.go:944-974.  validated_set=false is
 * time.Time{} (always inside the window). */
static void mark_duplicate(orc_engine* o, uint64_t p, uint32_t topic, bool validated_set, int64_t validated,
                           int64_t now) {
    if (!o->ps[p].present) return;
    orc_topic_stats* ts = topic_stats(o, p, topic);
    if (!ts) return;
    if (!ts->in_mesh) return;
    const gsx_topic_score_params* tp = &o->tp[topic];
    if (validated_set && (now - validated) > tp->mesh_message_deliveries_window_ns) return;
    double cap = tp->mesh_message_deliveries_cap;
    ts->mesh_message_deliveries += 1;
    if (ts->mesh_message_deliveries > cap) ts->mesh_message_deliveries = cap;
}

/* AddPenalty, score.go:384-398 */
static void add_penalty(orc_engine* o, uint64_t p, int64_t count) {
    if (!o->ps[p].present) return;
    o->ps[p].behaviour_penalty += (double)count;
}

int orc_apply_events(orc_engine* o, const gsx_event* ev, size_t n) {
    for (size_t i = 0; i < n; i++) {
        const gsx_event* e = &ev[i];
        if (e->pair >= o->E) return GSX_ERANGE;
        switch (e->kind) {
        case GSX_EV_ADD_PEER: add_peer(o, e->pair); break;
        case GSX_EV_REMOVE_PEER: remove_peer(o, e->pair, e->now_ns); break;
        case GSX_EV_GRAFT: graft(o, e->pair, e->topic, e->now_ns); break;
        case GSX_EV_PRUNE: prune(o, e->pair, e->topic); break;
        case GSX_EV_FIRST_DELIVERY: mark_first(o, e->pair, e->topic); break;
        case GSX_EV_MESH_DELIVERY: mark_duplicate(o, e->pair, e->topic, false, 0, e->now_ns); break;
        case GSX_EV_INVALID_DELIVERY: mark_invalid(o, e->pair, e->topic); break;
        case GSX_EV_PENALTY: add_penalty(o, e->pair, e->arg); break;
        case GSX_EV_APP_SCORE: memcpy(&o->app[e->pair], &e->arg, sizeof(double)); break; /* score.go:320 */
        default: return GSX_EINVAL;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* delivery records, score.go:686-870                                       */

static size_t rec_bucket(const orc_engine* o, uint32_t obs, uint64_t msg) {
    return (size_t)(mix64(((uint64_t)obs * 0x9E3779B97F4A7C15ULL) ^ msg) & (o->n_buckets - 1));
}

static void rehash(orc_engine* o) {
    size_t nb = o->n_buckets * 2;
    int64_t* b = (int64_t*)malloc(sizeof(int64_t) * nb);
    for (size_t i = 0; i < nb; i++) b[i] = -1;
    free(o->buckets);
    o->buckets = b;
    o->n_buckets = nb;
    for (size_t i = 0; i < o->n_recs; i++) {
        orc_record* r = &o->recs[i];
        if (!r->alive) continue;
        size_t h = rec_bucket(o, r->obs, r->msg);
        r->hnext = o->buckets[h];
        o->buckets[h] = (int64_t)i;
    }
}

/* messageDeliveries.getRecord, score.go:833-854 */
static orc_record* get_record(orc_engine* o, uint32_t obs, uint64_t msg, int64_t now) {
    size_t h = rec_bucket(o, obs, msg);
    for (int64_t i = o->buckets[h]; i >= 0; i = o->recs[i].hnext)
        if (o->recs[i].obs == obs && o->recs[i].msg == msg) return &o->recs[i];
    if (o->n_recs == o->cap_recs) {
        size_t nc = o->cap_recs ? 2 * o->cap_recs : 256;
        orc_record* nr = (orc_record*)realloc(o->recs, sizeof(orc_record) * nc);
        if (!nr) return NULL;
        o->recs = nr;
        o->cap_recs = nc;
    }
    if (o->n_alive * 2 > o->n_buckets) {
        rehash(o);
        h = rec_bucket(o, obs, msg);
    }
    int64_t idx = (int64_t)o->n_recs++;
    orc_record* r = &o->recs[idx];
    memset(r, 0, sizeof(*r));
    r->obs = obs;
    r->msg = msg;
    r->status = DELIVERY_UNKNOWN;
    r->first_seen = now;
    r->expire = now + TIME_CACHE_DURATION_NS;
    r->alive = true;
    r->hnext = o->buckets[h];
    o->buckets[h] = idx;
    r->qnext = -1;
    if (o->q_tail[obs] >= 0)
        o->recs[o->q_tail[obs]].qnext = idx;
    else
        o->q_head[obs] = idx;
    o->q_tail[obs] = idx;
    o->n_alive++;
    return r;
}

static bool rec_has_peer(const orc_record* r, uint64_t p) {
    for (size_t i = 0; i < r->n_peers; i++)
        if (r->peers[i] == p) return true;
    return false;
}

static void rec_add_peer(orc_record* r, uint64_t p) {
    if (r->peers_nil || rec_has_peer(r, p)) return;
    if (r->n_peers == r->cap_peers) {
        size_t nc = r->cap_peers ? 2 * r->cap_peers : 4;
        r->peers = (uint64_t*)realloc(r->peers, sizeof(uint64_t) * nc);
        r->cap_peers = nc;
    }
    r->peers[r->n_peers++] = p;
}

static void rec_nil_peers(orc_record* r) {
    free(r->peers);
    r->peers = NULL;
    r->n_peers = r->cap_peers = 0;
    r->peers_nil = true;
}

/* ValidateMessage, score.go:686-693 */
int orc_trace_validate(orc_engine* o, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now) {
    (void)topic;
    if (pair >= o->E) return GSX_ERANGE;
    return get_record(o, o->pair_obs[pair], msg_id, now) ? 0 : GSX_ENOMEM;
}

/* DeliverMessage, score.go:695-719 */
int orc_trace_deliver(orc_engine* o, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now) {
    if (pair >= o->E) return GSX_ERANGE;
    mark_first(o, pair, topic);
    orc_record* r = get_record(o, o->pair_obs[pair], msg_id, now);
    if (!r) return GSX_ENOMEM;
    if (r->status != DELIVERY_UNKNOWN) return 0;
    r->status = DELIVERY_VALID;
    r->validated = now;
    r->validated_set = true;
    for (size_t i = 0; i < r->n_peers; i++)
        if (r->peers[i] != pair) mark_duplicate(o, r->peers[i], topic, false, 0, now);
    return 0;
}

/* RejectMessage, score.go:721-786 */
int orc_trace_reject(orc_engine* o, uint64_t pair, uint64_t msg_id, uint32_t topic, int32_t reason, int64_t now) {
    if (pair >= o->E) return GSX_ERANGE;
    switch (reason) {
    case GSX_REJECT_MISSING_SIGNATURE:
    case GSX_REJECT_INVALID_SIGNATURE:
    case GSX_REJECT_UNEXPECTED_SIGNATURE:
    case GSX_REJECT_UNEXPECTED_AUTH_INFO:
    case GSX_REJECT_SELF_ORIGIN: mark_invalid(o, pair, topic); return 0;
    case GSX_REJECT_BLACKLISTED_PEER:
    case GSX_REJECT_BLACKLISTED_SOURCE:
    case GSX_REJECT_VALIDATION_QUEUE_FULL: return 0;
    default: break;
    }
    orc_record* r = get_record(o, o->pair_obs[pair], msg_id, now);
    if (!r) return GSX_ENOMEM;
    if (r->status != DELIVERY_UNKNOWN) return 0;
    switch (reason) {
    case GSX_REJECT_VALIDATION_THROTTLED:
        r->status = DELIVERY_THROTTLED;
        rec_nil_peers(r);
        return 0;
    case GSX_REJECT_VALIDATION_IGNORED:
        r->status = DELIVERY_IGNORED;
        rec_nil_peers(r);
        return 0;
    default: break;
    }
    r->status = DELIVERY_INVALID;
    mark_invalid(o, pair, topic);
    for (size_t i = 0; i < r->n_peers; i++) mark_invalid(o, r->peers[i], topic);
    rec_nil_peers(r);
    return 0;
}

/* DuplicateMessage, score.go:788-820 */
int orc_trace_duplicate(orc_engine* o, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now) {
    if (pair >= o->E) return GSX_ERANGE;
    orc_record* r = get_record(o, o->pair_obs[pair], msg_id, now);
    if (!r) return GSX_ENOMEM;
    if (!r->peers_nil && rec_has_peer(r, pair)) return 0;
    switch (r->status) {
    case DELIVERY_UNKNOWN: rec_add_peer(r, pair); break;
    case DELIVERY_VALID:
        rec_add_peer(r, pair);
        mark_duplicate(o, pair, topic, r->validated_set, r->validated, now);
        break;
    case DELIVERY_INVALID: mark_invalid(o, pair, topic); break;
    default: break; /* throttled / ignored */
    }
    return 0;
}

/* messageDeliveries.gc, score.go:856-870 (one queue per observer, as each
 * router owns its own peerScore) */
int orc_gc_deliveries(orc_engine* o, int64_t now) {
    for (uint32_t obs = 0; obs < o->n_nodes; obs++) {
        while (o->q_head[obs] >= 0 && now > o->recs[o->q_head[obs]].expire) {
            int64_t idx = o->q_head[obs];
            orc_record* r = &o->recs[idx];
            size_t h = rec_bucket(o, r->obs, r->msg);
            int64_t* link = &o->buckets[h];
            while (*link != idx) link = &o->recs[*link].hnext;
            *link = r->hnext;
            r->alive = false;
            free(r->peers);
            r->peers = NULL;
            o->n_alive--;
            o->q_head[obs] = r->qnext;
        }
        if (o->q_head[obs] < 0) o->q_tail[obs] = -1;
    }
    return 0;
}

uint64_t orc_num_delivery_records(orc_engine* o) { return o->n_alive; }

/* ------------------------------------------------------------------------ */
/* state view                                                               */

/* ------------------------------------------------------------------------ */
/* propagation: floodsub.go:76-100, gossipsub.go:943-1013, randomsub.go:99-160 */

int orc_set_thresholds(orc_engine* o, const gsx_thresholds* t) {
    o->th = *t;
    return 0;
}

/* p in ps.topics[topic] / ps.peers: connected and tracked */
/* the peer of pair r is in gs.p.topics[t] (subscribed, and known: present, connected) */
static bool in_topic(const orc_engine* o, uint64_t r, uint32_t t) {
    return o->ps[r].present && o->ps[r].connected && t < 64 && (o->sub[o->col[r]] >> t & 1);
}
static bool joined(const orc_engine* o, uint32_t v, uint32_t t) { return t < 64 && (o->sub[v] >> t & 1); }

/* the pair (u -> v) given the pair (v -> u); -1 if u does not track v */
static int64_t reverse_pair(const orc_engine* o, uint64_t r) {
    uint32_t v = o->pair_obs[r];
    uint32_t u = (uint32_t)o->col[r];
    for (int64_t q = o->row_ptr[u]; q < o->row_ptr[u + 1]; q++)
        if ((uint32_t)o->col[q] == v) return q;
    return -1;
}

/* Go's rand.Intn(n) = Int31n (math/rand), with Int31 draws taken from the
 * counter hash h(seed, 7, vertex, msg_id << 16 | k): the canonical RNG of
 * SURVEY.md §7 in place of the global math/rand source. */
static uint64_t splitmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static uint64_t h4(uint64_t seed, uint64_t tag, uint64_t a, uint64_t b) {
    uint64_t inner = splitmix(tag ^ splitmix(a ^ splitmix(b)));
    return splitmix(seed + 0x9E3779B97F4A7C15ULL * (1 + inner));
}
typedef struct {
    uint64_t seed, tag, vertex, base;
    uint32_t k;
} orc_rng;
static int32_t rng_int31(orc_rng* g) { return (int32_t)(h4(g->seed, g->tag, g->vertex, g->base | g->k++) >> 33); }
static int32_t rng_int31n(orc_rng* g, int32_t n) {
    if ((n & (n - 1)) == 0) return rng_int31(g) & (n - 1);
    int32_t max = (int32_t)((1u << 31) - 1 - (1u << 31) % (uint32_t)n);
    int32_t v = rng_int31(g);
    while (v > max) v = rng_int31(g);
    return v % n;
}
/* shufflePeers, gossipsub.go:1890-1895 */
static void shuffle_pairs(uint64_t* a, int n, orc_rng* g) {
    for (int i = 0; i < n; i++) {
        int j = rng_int31n(g, i + 1);
        uint64_t t = a[i];
        a[i] = a[j];
        a[j] = t;
    }
}

#define RANDOMSUB_D 6 /* randomsub.go:16-18 */

/* The pairs (v -> u) a vertex sends message m to: rt.Publish with
 * msg.ReceivedFrom = from (-1 when v published it) and GetFrom() = origin.
 * Returns the count; `out` has room for deg(v). */
static int router_targets(orc_engine* o, const gsx_prop_config* cfg, uint32_t v, uint32_t origin, int64_t from,
                          uint64_t msg_id, uint64_t* out, uint64_t* scratch, const double* score0) {
    int n = 0;
    const int64_t r0 = o->row_ptr[v], r1 = o->row_ptr[v + 1];
    if (cfg->router == GSX_ROUTER_FLOODSUB) { /* floodsub.go:81-90 */
        for (int64_t r = r0; r < r1; r++) {
            uint32_t u = (uint32_t)o->col[r];
            if (!in_topic(o, r, cfg->topic)) continue;
            if ((int64_t)u == from || u == origin) continue;
            out[n++] = (uint64_t)r;
        }
        return n;
    }
    if (cfg->router == GSX_ROUTER_RANDOMSUB) { /* randomsub.go:99-160 */
        int nrs = 0;
        for (int64_t r = r0; r < r1; r++) {
            uint32_t u = (uint32_t)o->col[r];
            if (!in_topic(o, r, cfg->topic)) continue;
            if ((int64_t)u == from || u == origin) continue;
            if (o->eflags[r] & GSX_EDGE_FLOODSUB) out[n++] = (uint64_t)r; /* rs.peers[p] == FloodSubID */
            else scratch[nrs++] = (uint64_t)r;
        }
        if (nrs > RANDOMSUB_D) {
            int target = RANDOMSUB_D;
            int sq = (int)ceil(sqrt((double)cfg->randomsub_size));
            if (sq > target) target = sq;
            if (target > nrs) target = nrs;
            orc_rng g = {cfg->seed, 7, v, msg_id << 16, 0};
            shuffle_pairs(scratch, nrs, &g); /* candidates in ascending neighbour order, then shuffled */
            nrs = target;
        }
        for (int i = 0; i < nrs; i++) out[n++] = scratch[i];
        return n;
    }
    /* gossipsub.go:943-1013 */
    const uint32_t topic = cfg->topic;
    const double thr = o->th.publish_threshold;
    for (int64_t r = r0; r < r1; r++) {
        if (!in_topic(o, r, cfg->topic)) continue; /* tmap */
        const uint8_t ef = o->eflags[r];
        const bool direct = (ef & GSX_EDGE_DIRECT) != 0;
        bool send;
        if (cfg->flood_publish && from < 0) { /* :953-960 */
            send = direct || score0[r] >= thr;
        } else {
            const bool mesh_peer = (ef & GSX_EDGE_GOSSIPSUB) != 0; /* gs.feature(GossipSubFeatureMesh, ...) */
            send = direct;                                          /* :962-968 */
            if (!send && !mesh_peer) send = score0[r] >= thr; /* :970-975 */
            if (!send && topic < o->T) /* gs.mesh[topic], or the fanout when not joined (:977-999) */
                send = joined(o, v, topic) ? o->ts[(uint64_t)r * o->T + topic].in_mesh : (o->fanout[r] >> topic & 1);
        }
        if (!send) continue;
        uint32_t u = (uint32_t)o->col[r];
        if ((int64_t)u == from || u == origin) continue; /* :1006-1009 */
        out[n++] = (uint64_t)r;
    }
    return n;
}

typedef struct {
    uint32_t u, v;
    uint64_t r; /* the sending pair (v -> u) */
} orc_arrival;

static int arrival_cmp(const void* a, const void* b) {
    const orc_arrival* x = (const orc_arrival*)a;
    const orc_arrival* y = (const orc_arrival*)b;
    if (x->u != y->u) return x->u < y->u ? -1 : 1;
    if (x->v != y->v) return x->v < y->v ? -1 : 1;
    return 0;
}

/* Time of a copy arriving at hop h (h >= 1): every hop is hop_latency_ns of
 * transit, and a receiver forwards only after validating for
 * validation_delay_ns (validation.go:230-351). */
static int64_t arrival_time(const gsx_prop_config* cfg, uint32_t h) {
    return cfg->now_ns + (int64_t)h * cfg->hop_latency_ns + (h ? (int64_t)(h - 1) * cfg->validation_delay_ns : 0);
}

/* Publish at a source that has not joined the topic (gossipsub.go:981-998):
 * its fanout, picked when empty (getPeers(D) of non-direct peers with
 * score >= PublishThreshold, draws h(seed, 10, source, topic << 24 | k)),
 * and lastpub = now; once per source at the call start.  score0: the scores
 * the call starts from (NULL: the current ones). */
static void fanout_publish(orc_engine* o, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg,
                           const double* score0) {
    if (!(cfg->router == GSX_ROUTER_GOSSIPSUB && !cfg->flood_publish && cfg->topic < o->T)) return;
    const uint32_t N = o->n_nodes;
    const uint32_t t = cfg->topic;
    uint64_t max_deg = 0;
    for (uint32_t i = 0; i < N; i++)
        if ((uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]) > max_deg) max_deg = (uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]);
    uint64_t* tg = (uint64_t*)malloc(sizeof(uint64_t) * (max_deg ? max_deg : 1));
    uint8_t* done = (uint8_t*)calloc(N ? N : 1, 1);
    for (size_t k = 0; k < m; k++) {
        const uint32_t src = msgs[k].source;
        if (src >= N || done[src] || joined(o, src, t)) continue;
        done[src] = 1;
        bool empty = true;
        for (int64_t r = o->row_ptr[src]; r < o->row_ptr[src + 1] && empty; r++)
            if (o->fanout[r] >> t & 1) empty = false;
        if (empty) {
            int n = 0;
            for (int64_t r = o->row_ptr[src]; r < o->row_ptr[src + 1]; r++) {
                const uint8_t ef = o->eflags[r];
                if (!in_topic(o, (uint64_t)r, t) || !(ef & GSX_EDGE_GOSSIPSUB) || (ef & GSX_EDGE_DIRECT)) continue;
                const double sc = score0 ? score0[r] : score_pair(o, (uint64_t)r);
                if (!(sc >= o->th.publish_threshold)) continue;
                tg[n++] = (uint64_t)r;
            }
            orc_rng g = {cfg->seed, 10, src, (uint64_t)t << 24, 0};
            shuffle_pairs(tg, n, &g);
            if (n > o->gp.d) n = o->gp.d;
            for (int i = 0; i < n; i++) o->fanout[tg[i]] |= 1ull << t;
            if (n > 0) o->fan_has[src] |= 1ull << t;
        }
        o->lastpub[(size_t)src * o->T + t] = cfg->now_ns;
    }
    free(done);
    free(tg);
}

int orc_propagate(orc_engine* o, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg, gsx_prop_out* out,
                  uint8_t* hop_out, int32_t* from_out) {
    if (cfg->max_hops > GSX_MAX_HOPS || cfg->validation_delay_ns < 0) return GSX_EINVAL;
    for (size_t k = 0; k < m; k++)
        if (msgs[k].validation > GSX_VALIDATION_THROTTLE) return GSX_EINVAL;
    memset(out, 0, sizeof(*out));
    const uint32_t N = o->n_nodes;
    free(o->dup_rows);
    o->dup_rows = NULL;
    o->dup_words = (m + 63) / 64;
    o->dup_E = o->E;
    if (o->dup_track) o->dup_rows = (uint64_t*)calloc(o->E * o->dup_words + 1, sizeof(uint64_t));
    uint8_t* hop = (uint8_t*)malloc(N ? N : 1);
    int32_t* from = (int32_t*)malloc(sizeof(int32_t) * (N ? N : 1));
    uint32_t* frontier = (uint32_t*)malloc(sizeof(uint32_t) * (N ? N : 1));
    uint32_t* next = (uint32_t*)malloc(sizeof(uint32_t) * (N ? N : 1));
    uint64_t max_deg = 0;
    for (uint32_t i = 0; i < N; i++)
        if ((uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]) > max_deg) max_deg = (uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]);
    uint64_t* tg = (uint64_t*)malloc(sizeof(uint64_t) * (max_deg ? max_deg : 1));
    uint64_t* scratch = (uint64_t*)malloc(sizeof(uint64_t) * (max_deg ? max_deg : 1));
    size_t cap_arr = 1024, n_arr = 0;
    orc_arrival* arr = (orc_arrival*)malloc(sizeof(orc_arrival) * cap_arr);
    const bool credit = cfg->credit_scores && cfg->topic < o->T && o->scored[cfg->topic];
    const bool gate = cfg->router == GSX_ROUTER_GOSSIPSUB; /* floodsub / randomsub: AcceptAll */
    /* The synchronous contract (gsx.h): the graylist and publishThreshold
     * tests of one call read the scores as they stand when it starts; the
     * call's own credits (P2/P3, and P4 of rejected messages) land at its end. */
    double* score0 = (double*)malloc(sizeof(double) * (o->E ? o->E : 1));
    for (uint64_t r = 0; r < o->E; r++) score0[r] = score_pair(o, r);
    fanout_publish(o, msgs, m, cfg, score0);
    /* gossipsub's Publish Puts every message a node processes into its
     * mcache (gossipsub.go:944); one batch entry in window 0 */
    orc_mc_batch* mcb = NULL;
    if (cfg->router == GSX_ROUTER_GOSSIPSUB && m > 0 && o->mc) {
        orc_mc_window* w0 = &o->mc[0];
        if (w0->nb == w0->cap) {
            w0->cap = w0->cap ? 2 * w0->cap : 4;
            w0->b = (orc_mc_batch*)realloc(w0->b, sizeof(orc_mc_batch) * w0->cap);
        }
        mcb = &w0->b[w0->nb++];
        mcb->topic = cfg->topic;
        mcb->m = (uint32_t)m;
        mcb->n = N;
        mcb->ids = (uint64_t*)malloc(sizeof(uint64_t) * m);
        mcb->has = (uint8_t*)calloc(m * (size_t)(N ? N : 1), 1);
        for (size_t k = 0; k < m; k++) mcb->ids[k] = msgs[k].msg_id;
        mcb->set = (orc_msgset*)calloc(1, sizeof(orc_msgset));
        mcb->set->serial = ++o->msg_serial;
        mcb->set->m = (uint32_t)m;
        mcb->set->n = N;
        mcb->set->refs = 1;
        mcb->set->val = (uint32_t*)malloc(sizeof(uint32_t) * m);
        mcb->set->src = (uint32_t*)malloc(sizeof(uint32_t) * m);
        mcb->set->t0 = cfg->now_ns;
        mcb->set->seen = (uint8_t*)calloc(m * (size_t)(N ? N : 1), 1);
        mcb->set->vcode = (uint16_t*)calloc(m * (size_t)(N ? N : 1), sizeof(uint16_t));
        mcb->set->n_vtime = cfg->max_hops + 1;
        mcb->set->vtime = (int64_t*)malloc(sizeof(int64_t) * mcb->set->n_vtime);
        for (uint32_t h = 0; h <= cfg->max_hops; h++)
            mcb->set->vtime[h] = cfg->now_ns + (int64_t)h * (cfg->hop_latency_ns + cfg->validation_delay_ns);
        for (size_t k = 0; k < m; k++) {
            mcb->set->val[k] = msgs[k].validation;
            mcb->set->src[k] = msgs[k].source;
        }
    }
    for (size_t k = 0; k < m; k++) {
        const uint32_t src = msgs[k].source;
        if (src >= N) return GSX_ERANGE;
        /* not accepted: seen, but neither delivered nor forwarded (pushMsg ->
         * validation -> RejectMessage, pubsub.go:1046-1090, score.go:721-786) */
        const uint32_t val = msgs[k].validation;
        const bool dropped = val != GSX_VALIDATION_ACCEPT;
        memset(hop, 0xFF, N);
        for (uint32_t i = 0; i < N; i++) from[i] = -1;
        hop[src] = 0; /* the local publish */
        uint32_t nf = 1, nn;
        frontier[0] = src;
        for (uint32_t h = 1; h <= cfg->max_hops && nf > 0; h++) {
            n_arr = 0;
            for (uint32_t i = 0; i < nf; i++) {
                const uint32_t v = frontier[i];
                int nt = router_targets(o, cfg, v, src, from[v], msgs[k].msg_id, tg, scratch, score0);
                for (int j = 0; j < nt; j++) {
                    if (n_arr == cap_arr) {
                        cap_arr *= 2;
                        arr = (orc_arrival*)realloc(arr, sizeof(orc_arrival) * cap_arr);
                    }
                    arr[n_arr].u = (uint32_t)o->col[tg[j]];
                    arr[n_arr].v = v;
                    arr[n_arr].r = tg[j];
                    n_arr++;
                }
            }
            /* each receiver handles its copies lowest sender first (pushMsg, pubsub.go:1046-1090) */
            qsort(arr, n_arr, sizeof(orc_arrival), arrival_cmp);
            nn = 0;
            for (size_t a = 0; a < n_arr; a++) {
                const uint32_t u = arr[a].u, v = arr[a].v;
                out->transmissions++;
                const int64_t qr = (credit || gate) ? reverse_pair(o, arr[a].r) : -1; /* u's peerStats for v */
                /* handleIncomingRPC asks the router first (pubsub.go:1014-1017):
                 * gossipsub's AcceptFrom (gossipsub.go:583-594) returns AcceptNone
                 * for a non-direct sender scoring below GraylistThreshold, and the
                 * RPC is dropped whole: no seen mark, no trace, no credit.  A
                 * sender u keeps no peerStats for scores 0 (score.go:247-256). */
                if (gate && qr >= 0 && !(o->eflags[qr] & GSX_EDGE_DIRECT) &&
                    score0[qr] < o->th.graylist_threshold) {
                    out->graylisted++;
                    continue;
                }
                const int64_t q = credit ? qr : -1;
                if (hop[u] == 0xFF) { /* first receipt: markSeen, then validation */
                    hop[u] = (uint8_t)h;
                    from[u] = (int32_t)v;
                    if (!dropped) { /* DeliverMessage, then Publish forwards it */
                        next[nn++] = u;
                        out->deliveries++;
                        out->hop_deliveries[h]++;
                        if (q >= 0) mark_first(o, (uint64_t)q, cfg->topic);
                    } else if (val == GSX_VALIDATION_REJECT) { /* RejectMessage(ValidationFailed) */
                        out->rejected++;
                        if (q >= 0) mark_invalid(o, (uint64_t)q, cfg->topic);
                    } else { /* RejectMessage(ValidationIgnored / Throttled): no penalty */
                        out->ignored++;
                    }
                } else { /* seenMessage -> DuplicateMessage, validated when the first copy's validation ended */
                    out->duplicates++;
                    if (o->dup_rows) { /* tracer.DuplicateMessage (pubsub.go:1052-1056, trace.go:136-164) */
                        const int64_t qd = qr >= 0 ? qr : reverse_pair(o, arr[a].r);
                        if (qd >= 0) o->dup_rows[(size_t)qd * o->dup_words + k / 64] |= 1ull << (k % 64);
                    }
                    if (q >= 0 && !dropped)
                        mark_duplicate(o, (uint64_t)q, cfg->topic, true,
                                       arrival_time(cfg, hop[u]) + (hop[u] ? cfg->validation_delay_ns : 0),
                                       arrival_time(cfg, h));
                    else if (q >= 0 && val == GSX_VALIDATION_REJECT)
                        mark_invalid(o, (uint64_t)q, cfg->topic); /* deliveryInvalid, score.go:811-813 */
                }
            }
            if (nn > 0 && h > out->hops) out->hops = h;
            memcpy(frontier, next, sizeof(uint32_t) * nn); /* already ascending: arrivals sorted by u */
            nf = nn;
        }
        if (hop_out) memcpy(hop_out + k * (size_t)N, hop, N);
        if (from_out) memcpy(from_out + k * (size_t)N, from, sizeof(int32_t) * N);
        if (mcb) /* Publish Puts what a node processes: a dropped message only at its source */
            for (uint32_t i = 0; i < N; i++) {
                mcb->has[(size_t)i * m + k] = hop[i] != 0xFF && (!dropped || i == src);
                mcb->set->seen[(size_t)i * m + k] = hop[i] != 0xFF;
                mcb->set->vcode[(size_t)i * m + k] = hop[i] != 0xFF ? hop[i] : 0;
            }
    }
    free(hop);
    free(from);
    free(frontier);
    free(next);
    free(tg);
    free(scratch);
    free(arr);
    free(score0);
    return 0;
}

int orc_prop_set_dup_tracking(orc_engine* o, int on) {
    o->dup_track = on != 0;
    return 0;
}

int orc_prop_duplicates(orc_engine* o, uint64_t* rows, size_t n_words) {
    if (!o->dup_rows || o->dup_E != o->E) return GSX_ESTATE;
    if (n_words != o->dup_words) return GSX_EINVAL;
    memcpy(rows, o->dup_rows, sizeof(uint64_t) * o->E * n_words);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* heartbeat: gossipsub.go:1303-1604, 718-859                               */

int orc_default_gossipsub_params(gsx_gossipsub_params* p) { /* DefaultGossipSubParams, gossipsub.go:230-260 */
    memset(p, 0, sizeof(*p));
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
    p->history_gossip = 5; /* HistoryGossip: GossipSubHistoryLength (:238) */
    p->max_ihave_length = 5000;
    p->gossip_factor = 0.25;
    p->max_ihave_messages = 10;
    p->gossip_retransmission = 3;
    p->iwant_followup_ns = 3LL * 1000000000LL;
    p->gossip_exchange = 1; /* handleIHave / handleIWant always run in the reference (gossipsub.go:615-720) */
    p->fanout_ttl_ns = 60LL * 1000000000LL;
    p->do_px = 0;
    p->prune_peers = 16; /* GossipSubPrunePeers, :46 */
    return 0;
}

#define HEARTBEAT_INTERVAL_NS (1000000000LL) /* GossipSubHeartbeatInterval, clearBackoff's slack (:1596) */

typedef struct {
    orc_engine* o;
    const gsx_gossipsub_params* gp;
    const double* cache; /* per pair: scores at the heartbeat start */
    uint8_t* ctl;        /* [t][pair (v -> u)] 1 GRAFT, 2 PRUNE sent by v */
    uint64_t tick;
    int64_t now;
    gsx_heartbeat_out* out;
    uint64_t seed;
    uint64_t* mids; /* emitGossip scratch: ids, gossip positions, Floyd marks */
    uint32_t* mpos;
    uint8_t* msel;
    size_t mcap;
} hb_ctx;

static bool hb_in_mesh(const orc_engine* o, uint64_t r, uint32_t t) {
    return o->ps[r].present && o->ts[r * o->T + t].in_mesh;
}
static int64_t* hb_backoff(orc_engine* o, uint64_t r, uint32_t t) { return &o->backoff[(size_t)t * o->E + r]; }

/* addBackoff / doAddBackoff, gossipsub.go:845-859 */
static void add_backoff(orc_engine* o, uint64_t r, uint32_t t, int64_t now, int64_t interval) {
    int64_t expire = now + interval;
    int64_t* b = hb_backoff(o, r, t);
    if (*b == 0 || *b < expire) *b = expire; /* backoff[p].Before(expire) (zero time is before everything) */
}

/* getPeers, gossipsub.go:1852-1872: topic peers with the mesh feature that
 * pass the filter, in ascending order, shuffled, truncated to count. */
enum { F_NOT_MESH = 1, F_NO_BACKOFF = 2, F_NOT_DIRECT = 4, F_OUTBOUND = 8, F_NOT_FANOUT = 16 };
static int get_peers(hb_ctx* c, uint32_t v, uint32_t t, int count, int filter, int score_cmp, double score_ref,
                     uint64_t* out, orc_rng* g) {
    orc_engine* o = c->o;
    int n = 0;
    for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) {
        if (!in_topic(o, (uint64_t)r, t)) continue;
        const uint8_t ef = o->eflags[r];
        if (!(ef & GSX_EDGE_GOSSIPSUB)) continue; /* gs.feature(GossipSubFeatureMesh, ...) */
        if ((filter & F_NOT_MESH) && hb_in_mesh(o, (uint64_t)r, t)) continue;
        if ((filter & F_NO_BACKOFF) && *hb_backoff(o, (uint64_t)r, t) != 0) continue; /* map presence (:1377) */
        if ((filter & F_NOT_DIRECT) && (ef & GSX_EDGE_DIRECT)) continue;
        if ((filter & F_OUTBOUND) && !(ef & GSX_EDGE_OUTBOUND)) continue;
        if ((filter & F_NOT_FANOUT) && (o->fanout[r] >> t & 1)) continue;
        const double s = c->cache[r];
        if (score_cmp == 0 && !(s >= score_ref)) continue;
        if (score_cmp == 1 && !(s > score_ref)) continue;
        out[n++] = (uint64_t)r;
    }
    shuffle_pairs(out, n, g);
    if (count > 0 && n > count) n = count;
    return n;
}

static void hb_graft(hb_ctx* c, uint64_t r, uint32_t t) { /* graftPeer, :1353-1359 */
    graft(c->o, r, t, c->now);
    c->ctl[(size_t)t * c->o->E + r] = 1;
    c->o->tr_sg[r] |= 1ull << t; /* tracer.Graft, :1355 */
    c->out->grafts++;
}

static void hb_prune(hb_ctx* c, uint64_t r, uint32_t t) { /* prunePeer, :1345-1351 */
    prune(c->o, r, t);
    add_backoff(c->o, r, t, c->now, c->gp->prune_backoff_ns);
    c->ctl[(size_t)t * c->o->E + r] = 2;
    c->o->tr_sp[r] |= 1ull << t; /* tracer.Prune, :1346 */
    c->out->prunes++;
}

static int mesh_list(const orc_engine* o, uint32_t v, uint32_t t, uint64_t* out) {
    int n = 0;
    for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++)
        if (hb_in_mesh(o, (uint64_t)r, t)) out[n++] = (uint64_t)r;
    return n;
}

/* stable sort of pairs by cached score; desc = 1 for descending */
static void sort_by_score(const double* cache, uint64_t* a, int n, int desc) {
    for (int i = 1; i < n; i++) { /* insertion sort: stable */
        uint64_t x = a[i];
        int j = i - 1;
        while (j >= 0 && (desc ? cache[a[j]] < cache[x] : cache[a[j]] > cache[x])) {
            a[j + 1] = a[j];
            j--;
        }
        a[j + 1] = x;
    }
}

/* the mesh maintenance of one (node, topic), gossipsub.go:1344-1510 */
static void hb_unit(hb_ctx* c, uint32_t v, uint32_t t, orc_rng* gr, uint64_t* plst, uint64_t* tmp) {
    orc_engine* o = c->o;
    const gsx_gossipsub_params* gp = c->gp;
#define g (*gr)
    /* drop all peers with negative score, without PX (:1361-1368) */
    int n = mesh_list(o, v, t, plst);
    for (int i = 0; i < n; i++)
        if (c->cache[plst[i]] < 0) {
            hb_prune(c, plst[i], t);
            if (o->pxno) o->pxno[plst[i]] |= 1; /* noPX[p] = true */
        }
    /* do we have enough peers? (:1370-1385) */
    n = mesh_list(o, v, t, plst);
    if (n < gp->d_lo) {
        int ineed = gp->d - n;
        int k = get_peers(c, v, t, ineed, F_NOT_MESH | F_NO_BACKOFF | F_NOT_DIRECT, 0, 0.0, tmp, &g);
        for (int i = 0; i < k; i++) hb_graft(c, tmp[i], t);
    }
    /* do we have too many peers? (:1387-1448) */
    n = mesh_list(o, v, t, plst);
    if (n > gp->d_hi) {
        shuffle_pairs(plst, n, &g);
        sort_by_score(c->cache, plst, n, 1);
        shuffle_pairs(plst + gp->d_score, n - gp->d_score, &g);
        int outbound = 0;
        for (int i = 0; i < gp->d; i++)
            if (o->eflags[plst[i]] & GSX_EDGE_OUTBOUND) outbound++;
        if (outbound < gp->d_out) {
            /* rotate(i): move plst[i] to the front (:1411-1418) */
#define ROTATE(i)                                   \
    do {                                            \
        uint64_t p_ = plst[(i)];                    \
        for (int j_ = (i); j_ > 0; j_--) plst[j_] = plst[j_ - 1]; \
        plst[0] = p_;                               \
    } while (0)
            if (outbound > 0) {
                int ihave = outbound;
                for (int i = 1; i < gp->d && ihave > 0; i++)
                    if (o->eflags[plst[i]] & GSX_EDGE_OUTBOUND) {
                        ROTATE(i);
                        ihave--;
                    }
            }
            int ineed = gp->d_out - outbound;
            for (int i = gp->d; i < n && ineed > 0; i++)
                if (o->eflags[plst[i]] & GSX_EDGE_OUTBOUND) {
                    ROTATE(i);
                    ineed--;
                }
#undef ROTATE
        }
        for (int i = gp->d; i < n; i++) hb_prune(c, plst[i], t);
    }
    /* do we have enough outbound peers? (:1450-1476) */
    n = mesh_list(o, v, t, plst);
    if (n >= gp->d_lo) {
        int outbound = 0;
        for (int i = 0; i < n; i++)
            if (o->eflags[plst[i]] & GSX_EDGE_OUTBOUND) outbound++;
        if (outbound < gp->d_out) {
            int ineed = gp->d_out - outbound;
            int k = get_peers(c, v, t, ineed, F_NOT_MESH | F_NO_BACKOFF | F_NOT_DIRECT | F_OUTBOUND, 0, 0.0, tmp, &g);
            for (int i = 0; i < k; i++) hb_graft(c, tmp[i], t);
        }
    }
    /* opportunistic grafting (:1478-1510) */
    n = mesh_list(o, v, t, plst);
    if (gp->opportunistic_graft_ticks && c->tick % gp->opportunistic_graft_ticks == 0 && n > 1) {
        sort_by_score(c->cache, plst, n, 0);
        double median = c->cache[plst[n / 2]];
        if (median < o->th.opportunistic_graft_threshold) {
            int k = get_peers(c, v, t, gp->opportunistic_graft_peers, F_NOT_MESH | F_NO_BACKOFF | F_NOT_DIRECT, 1,
                              median, tmp, &g);
            for (int i = 0; i < k; i++) hb_graft(c, tmp[i], t);
        }
    }
#undef g
}

static uint64_t ihave_digest(const uint64_t* ids, size_t n) { /* gsx.h, gsx_gossip_results */
    uint64_t d = 0;
    for (size_t i = 0; i < n; i++) d += splitmix(ids[i] + 0x9E3779B97F4A7C15ULL);
    return d;
}

/* Floyd's sampling (gsx.h, truncated IHAVE lists): k distinct positions of
 * [0, L) marked in sel, draws Int31n(j + 1) for j = L - k .. L - 1 */
static void floyd_select(uint8_t* sel, uint32_t L, uint32_t k, orc_rng* g) {
    memset(sel, 0, L);
    for (uint32_t j = L - k; j < L; j++) {
        uint32_t x = (uint32_t)rng_int31n(g, (int32_t)(j + 1));
        if (sel[x]) x = j;
        sel[x] = 1;
    }
}

/* the truncated list's row of (topic, pair), zeroed (allocated on first use) */
static uint64_t* sub_row(orc_engine* o, uint32_t t, uint64_t r) {
    const size_t E = o->E ? o->E : 1, tw = o->sub_tw[t];
    if (!o->sub_idx[t]) {
        o->sub_idx[t] = (uint32_t*)malloc(sizeof(uint32_t) * E);
        memset(o->sub_idx[t], 0xFF, sizeof(uint32_t) * E);
    }
    if ((o->sub_n[t] + 1) * tw > o->sub_cap[t]) { /* capacity in words: tw changes between rounds */
        size_t cap = o->sub_cap[t] ? 2 * o->sub_cap[t] : 1024 * tw;
        while (cap < (o->sub_n[t] + 1) * tw) cap *= 2;
        o->sub_cap[t] = cap;
        o->sub_rows[t] = (uint64_t*)realloc(o->sub_rows[t], sizeof(uint64_t) * cap);
    }
    o->sub_idx[t][r] = (uint32_t)o->sub_n[t];
    uint64_t* row = o->sub_rows[t] + tw * o->sub_n[t]++;
    memset(row, 0, sizeof(uint64_t) * tw);
    return row;
}

/* emitGossip (gossipsub.go:1669-1723) for (v, t) after its maintenance, with
 * mcache.GetGossipIDs (mcache.go:82-92) over the first HistoryGossip windows.
 * The list's own order is never observable (a receiver collects it into a
 * set, :643-650), so it is not shuffled and draws nothing; a list longer than
 * MaxIHaveLength reaches each target as its own uniform MaxIHaveLength-subset
 * (the reference reshuffles the list per target and keeps a prefix,
 * :1712-1720: i.i.d. uniform subsets), drawn by Floyd's sampling of
 * min(MaxIHaveLength, L - MaxIHaveLength) positions with draws h(seed, 13,
 * node << 32 | peer, tick << 32 | topic << 24 | fan << 23 | k): the marked positions when
 * that is MaxIHaveLength, else the unmarked ones.  The subset is kept per
 * (topic, pair) as a bitmask over the topic's gossip positions for the
 * exchange (D). */
static void emit_gossip(hb_ctx* c, uint32_t v, uint32_t t, orc_rng* g, uint64_t* peers, bool fan) {
    orc_engine* o = c->o;
    const gsx_gossipsub_params* gp = c->gp;
    size_t L = 0;
    uint32_t base = 0; /* gossip position of the batch's message 0 */
    const uint32_t nw = (uint32_t)gp->history_gossip < o->mc_n ? (uint32_t)gp->history_gossip : o->mc_n;
    for (uint32_t w = 0; w < nw; w++)
        for (size_t b = 0; b < o->mc[w].nb; b++) {
            const orc_mc_batch* mb = &o->mc[w].b[b];
            if (mb->topic != t) continue;
            const uint8_t* has = mb->has + (size_t)v * mb->m;
            for (uint32_t k = 0; k < mb->m; k++) {
                if (!has[k]) continue;
                if (L == c->mcap) {
                    c->mcap = c->mcap ? 2 * c->mcap : 1024;
                    c->mids = (uint64_t*)realloc(c->mids, sizeof(uint64_t) * c->mcap);
                    c->mpos = (uint32_t*)realloc(c->mpos, sizeof(uint32_t) * c->mcap);
                    c->msel = (uint8_t*)realloc(c->msel, c->mcap);
                }
                c->mids[L] = mb->ids[k];
                c->mpos[L++] = base + k;
            }
            base += mb->m;
        }
    if (L == 0) return;
    int np = 0;
    for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) {
        if (!in_topic(o, (uint64_t)r, t)) continue;
        const uint8_t ef = o->eflags[r];
        /* exclude: the mesh peers, or the fanout peers for a fanout topic (:1514, :1553) */
        const bool excl = fan ? (o->fanout[r] >> t & 1) : hb_in_mesh(o, (uint64_t)r, t);
        if (excl || (ef & GSX_EDGE_DIRECT) || !(ef & GSX_EDGE_GOSSIPSUB)) continue;
        if (!(score_pair(o, (uint64_t)r) >= o->th.gossip_threshold)) continue; /* live score */
        peers[np++] = (uint64_t)r;
    }
    int target = gp->d_lazy;
    const int factor = (int)(gp->gossip_factor * (double)np);
    if (factor > target) target = factor;
    if (target > np) target = np;
    else shuffle_pairs(peers, np, g);
    const size_t maxl = (size_t)(gp->max_ihave_length > 0 ? gp->max_ihave_length : 0);
    uint64_t all = 0;
    if (L <= maxl) all = ihave_digest(c->mids, L);
    for (int i = 0; i < target; i++) {
        const uint64_t r = peers[i];
        const size_t x = (size_t)t * o->E + r;
        size_t len = L;
        uint64_t d = all;
        if (L > maxl) {
            const uint32_t kk = (uint32_t)(maxl < L - maxl ? maxl : L - maxl);
            const bool take = kk == maxl; /* the marked positions are the list, else the unmarked ones */
            orc_rng gs = {c->seed, 13, ((uint64_t)v << 32) | (uint32_t)o->col[r],
                          (c->tick << 32) | ((uint64_t)t << 24) | ((uint64_t)fan << 23), 0};
            floyd_select(c->msel, (uint32_t)L, kk, &gs);
            uint64_t* row = sub_row(o, t, r);
            len = maxl;
            d = 0;
            for (size_t e = 0; e < L; e++)
                if ((c->msel[e] != 0) == take) {
                    d += splitmix(c->mids[e] + 0x9E3779B97F4A7C15ULL);
                    row[c->mpos[e] / 64] |= 1ull << (c->mpos[e] % 64);
                }
        } else if (o->sub_idx[t]) {
            o->sub_idx[t][r] = UINT32_MAX; /* (a fanout pass after a truncated mesh pass) */
        }
        o->ihave_len[x] = (uint32_t)len;
        o->ihave_hash[x] = d;
        c->out->ihave_msgs++;
        c->out->ihave_ids += len;
    }
}

/* mcache.Shift (mcache.go:94-104) */
static void mcache_shift(orc_engine* o, uint32_t history) {
    if (!o->mc) return;
    if (history > ORC_MC_MAX) history = ORC_MC_MAX;
    while (o->mc_n >= history && o->mc_n > 0) { /* drop history[len-1] */
        orc_mc_window* w = &o->mc[o->mc_n - 1];
        for (size_t i = 0; i < w->nb; i++) batch_free(&w->b[i]);
        free(w->b);
        memset(w, 0, sizeof(*w));
        o->mc_n--;
    }
    memmove(&o->mc[1], &o->mc[0], sizeof(orc_mc_window) * o->mc_n);
    memset(&o->mc[0], 0, sizeof(orc_mc_window));
    o->mc_n++;
}

/* handlePrune at u for a PRUNE of topic t from the peer of pair q (u -> v), :811-843 */
static void handle_prune(orc_engine* o, const gsx_gossipsub_params* gp, uint64_t q, uint32_t t, int64_t now,
                         gsx_heartbeat_out* out) {
    prune(o, q, t); /* tracer.Prune, unconditional */
    o->tr_hp[q] |= 1ull << t;
    /* the PRUNE carries PruneBackoff in whole seconds (:1821); 0 means "use our own" (:825-830) */
    const int64_t secs = gp->prune_backoff_ns / 1000000000LL;
    add_backoff(o, q, t, now, secs > 0 ? secs * 1000000000LL : gp->prune_backoff_ns);
    out->prunes_handled++;
}

/* ---- (D) the gossip exchange: handleIHave / handleIWant (gossipsub.go:615-716)
 * and the gossipTracer's promises (gossip_tracer.go:48-153) -------------- */

/* The promises of every router's gossipTracer (gossip_tracer.go:24-27),
 * promises[mid][p] of observer u as one hash table keyed (pair (u -> p),
 * handle): linear probing with backward-shift deletion, no bound on the
 * number outstanding (AddPromise never refuses one, :59-74). */
static size_t prom_home(uint64_t q, uint64_t handle, size_t cap) {
    return (size_t)mix64(q * 0x9E3779B97F4A7C15ULL ^ handle) & (cap - 1);
}
static int64_t prom_find(const orc_engine* o, uint64_t q, uint64_t handle) {
    if (!o->cap_prom) return -1;
    for (size_t j = prom_home(q, handle, o->cap_prom);; j = (j + 1) & (o->cap_prom - 1)) {
        if (!o->prom[j].used) return -1;
        if (o->prom[j].q == q && o->prom[j].handle == handle) return (int64_t)j;
    }
}
static void prom_put(orc_engine* o, uint64_t q, uint64_t handle, int64_t expire) { /* (q, handle) absent */
    if (2 * (o->n_prom + 1) > o->cap_prom) {
        const size_t oc = o->cap_prom, nc = oc ? 2 * oc : 1024;
        orc_promise* old = o->prom;
        o->prom = (orc_promise*)calloc(nc, sizeof(orc_promise));
        o->cap_prom = nc;
        o->n_prom = 0;
        for (size_t i = 0; i < oc; i++)
            if (old[i].used) prom_put(o, old[i].q, old[i].handle, old[i].expire);
        free(old);
    }
    size_t j = prom_home(q, handle, o->cap_prom);
    while (o->prom[j].used) j = (j + 1) & (o->cap_prom - 1);
    o->prom[j].q = q;
    o->prom[j].handle = handle;
    o->prom[j].expire = expire;
    o->prom[j].used = 1;
    o->n_prom++;
}
static void prom_erase(orc_engine* o, size_t i) {
    const size_t m = o->cap_prom - 1;
    for (size_t j = (i + 1) & m; o->prom[j].used; j = (j + 1) & m) {
        const size_t k = prom_home(o->prom[j].q, o->prom[j].handle, o->cap_prom);
        /* the entry at j may fill the hole at i iff its home is not cyclically in (i, j] */
        const bool in = i <= j ? (k > i && k <= j) : (k > i || k <= j);
        if (!in) {
            o->prom[i] = o->prom[j];
            i = j;
        }
    }
    memset(&o->prom[i], 0, sizeof(orc_promise));
    o->n_prom--;
}
/* Keeps the promises keep(entry) accepts, rebuilding the table. */
static void prom_filter(orc_engine* o, bool (*keep)(const orc_promise*, const void*), const void* arg) {
    const size_t oc = o->cap_prom;
    orc_promise* old = o->prom;
    o->prom = oc ? (orc_promise*)calloc(oc, sizeof(orc_promise)) : NULL;
    o->n_prom = 0;
    for (size_t i = 0; i < oc; i++)
        if (old[i].used && keep(&old[i], arg)) prom_put(o, old[i].q, old[i].handle, old[i].expire);
    free(old);
    memset(o->prom_node, 0, sizeof(uint32_t) * (o->n_nodes ? o->n_nodes : 1));
    for (size_t i = 0; i < oc; i++)
        if (o->prom[i].used) o->prom_node[o->pair_obs[o->prom[i].q]]++;
}

static void add_promise(orc_engine* o, uint64_t q, uint64_t handle, int64_t expire) { /* AddPromise :59-74 */
    if (prom_find(o, q, handle) < 0) {
        prom_put(o, q, handle, expire);
        o->prom_node[o->pair_obs[q]]++;
    }
}

static void fulfill_promises(orc_engine* o, uint32_t u, uint64_t handle) { /* fulfillPromise :119-126 */
    if (!o->n_prom || !o->prom_node[u]) return;
    for (int64_t q = o->row_ptr[u]; q < o->row_ptr[u + 1]; q++) {
        const int64_t i = prom_find(o, (uint64_t)q, handle);
        if (i >= 0) {
            prom_erase(o, (size_t)i);
            o->prom_node[u]--;
        }
    }
}

typedef struct {
    int64_t now;
    uint32_t* cnt;
    uint64_t total;
} broken_ctx;
static bool prom_keep_unbroken(const orc_promise* p, const void* arg) {
    broken_ctx* c = (broken_ctx*)arg;
    if (!(p->expire < c->now)) return true;
    c->cnt[p->q]++;
    c->total++;
    return false;
}
/* GetBrokenPromises (:79-115): the promises that expired before now are
 * removed and counted per pair; returns their number */
static uint64_t broken_promises(orc_engine* o, int64_t now, uint32_t* cnt) {
    broken_ctx c = {now, cnt, 0};
    if (o->n_prom) prom_filter(o, prom_keep_unbroken, &c);
    return c.total;
}
static bool prom_keep_other_pair(const orc_promise* p, const void* arg) { return p->q != *(const uint64_t*)arg; }

/* The gossipTracer's methods on one router's promises (gsx.h: the tracer
 * API, gossip_tracer.go:48-185): AddPromise's pick is Int31n(n) with draws
 * h(seed, 9, pair, k). */
int orc_promise_add(orc_engine* o, uint64_t q, const uint64_t* handles, uint32_t n, int64_t expire, uint64_t seed) {
    if (q >= o->E || n == 0 || n > 0x7FFFFFFFu || expire == 0) return GSX_EINVAL; /* (gsx.h: expiry 0 is no time) */
    orc_rng g = {seed, 9, q, 0, 0};
    add_promise(o, q, handles[rng_int31n(&g, (int32_t)n)], expire);
    return 0;
}
int orc_promise_broken(orc_engine* o, int64_t now, uint32_t* counts, uint64_t* total) {
    uint32_t* cnt = (uint32_t*)calloc(o->E ? o->E : 1, sizeof(uint32_t));
    const uint64_t n = broken_promises(o, now, cnt);
    if (counts) memcpy(counts, cnt, sizeof(uint32_t) * o->E);
    if (total) *total = n;
    free(cnt);
    return 0;
}
int orc_promise_fulfill(orc_engine* o, uint32_t node, uint64_t handle) {
    if (node >= o->n_nodes) return GSX_EINVAL;
    fulfill_promises(o, node, handle);
    return 0;
}
int orc_promise_throttle(orc_engine* o, uint64_t q) { /* ThrottlePeer :167-185 */
    if (q >= o->E) return GSX_EINVAL;
    if (o->n_prom) prom_filter(o, prom_keep_other_pair, &q);
    return 0;
}
int orc_promise_count(orc_engine* o, uint64_t* n) {
    *n = o->n_prom;
    return 0;
}

/* mcache.GetForPeer's per-(message, peer) count (mcache.go:66-80), keyed by
 * the responder's pair and the message handle */
static uint32_t peertx_inc(orc_engine* o, uint64_t r, uint64_t handle) {
    if (2 * (o->ptx_n + 1) > o->ptx_cap) {
        size_t oc = o->ptx_cap, nc = oc ? 2 * oc : 1024;
        uint64_t *ok = o->ptx_key, *op = o->ptx_pair;
        uint32_t* ocn = o->ptx_cnt;
        o->ptx_key = (uint64_t*)calloc(nc, 8);
        o->ptx_pair = (uint64_t*)calloc(nc, 8);
        o->ptx_cnt = (uint32_t*)calloc(nc, 4);
        o->ptx_cap = nc;
        o->ptx_n = 0;
        for (size_t i = 0; i < oc; i++)
            if (ocn && ocn[i]) {
                size_t j = mix64(op[i] * 0x9E3779B97F4A7C15ULL ^ ok[i]) & (nc - 1);
                while (o->ptx_cnt[j]) j = (j + 1) & (nc - 1);
                o->ptx_key[j] = ok[i];
                o->ptx_pair[j] = op[i];
                o->ptx_cnt[j] = ocn[i];
                o->ptx_n++;
            }
        free(ok);
        free(op);
        free(ocn);
    }
    size_t j = mix64(r * 0x9E3779B97F4A7C15ULL ^ handle) & (o->ptx_cap - 1);
    while (o->ptx_cnt[j] && !(o->ptx_pair[j] == r && o->ptx_key[j] == handle)) j = (j + 1) & (o->ptx_cap - 1);
    if (!o->ptx_cnt[j]) {
        o->ptx_pair[j] = r;
        o->ptx_key[j] = handle;
        o->ptx_n++;
    }
    return ++o->ptx_cnt[j];
}

typedef struct {
    orc_mc_batch* b;
    bool avail; /* still in the cache after this heartbeat's Shift */
} gx_batch;
typedef struct {
    uint32_t gb, k; /* gossip batch index, message index */
} gx_item;
typedef struct {
    uint64_t q;
    size_t i0, n; /* selected items[i0 .. i0 + n) */
    bool served;
} gx_req;
typedef struct {
    uint32_t x, k, u, v; /* recovered set, message, receiver, the peer that served it */
} gx_recv;
static int u32_cmp(const void* a, const void* b) {
    const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}
static int gx_recv_cmp(const void* a, const void* b) {
    const gx_recv* p = (const gx_recv*)a;
    const gx_recv* q = (const gx_recv*)b;
    if (p->x != q->x) return p->x < q->x ? -1 : 1;
    if (p->k != q->k) return p->k < q->k ? -1 : 1;
    if (p->u != q->u) return p->u < q->u ? -1 : 1;
    return 0;
}

static int gossip_exchange(orc_engine* o, const gsx_gossipsub_params* gp, uint64_t tick, int64_t now,
                           uint64_t seed, gsx_heartbeat_out* out, orc_mc_batch** rec_out, size_t* n_rec) {
    const uint64_t E = o->E;
    const uint32_t T = o->T, N = o->n_nodes;
    uint32_t history = (uint32_t)(gp->history_length > 0 ? gp->history_length : 0);
    if (history > ORC_MC_MAX) history = ORC_MC_MAX;
    const uint32_t nw = (uint32_t)gp->history_gossip < o->mc_n ? (uint32_t)gp->history_gossip : o->mc_n;
    /* the advertised batches per topic (GetGossipIDs order: windows newest first, Put order) */
    size_t nb = 0;
    for (uint32_t w = 0; w < nw; w++) nb += o->mc[w].nb;
    gx_batch* gb = (gx_batch*)malloc(sizeof(gx_batch) * (nb ? nb : 1));
    nb = 0;
    for (uint32_t w = 0; w < nw; w++)
        for (size_t i = 0; i < o->mc[w].nb; i++) {
            gb[nb].b = &o->mc[w].b[i];
            gb[nb].avail = o->mc_n < history || w + 1 < history;
            nb++;
        }
    double* score0 = (double*)malloc(sizeof(double) * (E ? E : 1));
    for (uint64_t r = 0; r < E; r++) score0[r] = score_pair(o, r);
    size_t cap_it = 1024, n_it = 0, cap_rq = 256, n_rq = 0, cap_w = 1024;
    gx_item* items = (gx_item*)malloc(sizeof(gx_item) * cap_it);
    gx_req* reqs = (gx_req*)malloc(sizeof(gx_req) * cap_rq);
    gx_item* W = (gx_item*)malloc(sizeof(gx_item) * cap_w);
    int rc = 0;
    /* handleIHave at every node u, one IHAVE RPC per sending peer v, senders ascending */
    for (uint32_t u = 0; u < N && !rc; u++)
        for (int64_t q = o->row_ptr[u]; q < o->row_ptr[u + 1]; q++) {
            const int64_t r = reverse_pair(o, (uint64_t)q); /* r = (v -> u) carried the IHAVEs */
            if (r < 0) continue;
            uint64_t tb = 0;
            for (uint32_t t = 0; t < T; t++)
                if (o->ihave_len[(size_t)t * E + r]) tb |= 1ull << t;
            if (!tb) continue;
            const uint32_t v = (uint32_t)o->col[q];
            size_t n = 0;
            for (uint32_t t = 0; t < T; t++) {
                if (!(tb >> t & 1) || !joined(o, u, t)) continue; /* gs.mesh[topic] (:638-641) */
                /* a truncated list: the subset v sent u (emitGossip) */
                const uint32_t si = o->sub_idx[t] ? o->sub_idx[t][r] : UINT32_MAX;
                const uint64_t* sub = si != UINT32_MAX ? o->sub_rows[t] + (size_t)o->sub_tw[t] * si : NULL;
                uint32_t base = 0; /* gossip position of the batch's message 0 */
                for (size_t i = 0; i < nb; i++) {
                    const orc_mc_batch* b = gb[i].b;
                    if (b->topic != t) continue;
                    const uint32_t b0 = base;
                    base += b->m;
                    for (uint32_t k = 0; k < b->m; k++) {
                        if (!b->has[(size_t)v * b->m + k]) continue;
                        if (sub && !(sub[(b0 + k) / 64] >> ((b0 + k) % 64) & 1)) continue;
                        if (b->set->seen[(size_t)u * b->m + k]) continue; /* seenMessage (:645) */
                        if (n == cap_w) {
                            cap_w *= 2;
                            W = (gx_item*)realloc(W, sizeof(gx_item) * cap_w);
                        }
                        W[n].gb = (uint32_t)i;
                        W[n].k = k;
                        n++;
                    }
                }
            }
            if (score0[q] < o->th.gossip_threshold) { /* :617-621 */
                out->ihave_ignored++;
                continue;
            }
            if (++o->peerhave[q] > (uint32_t)(gp->max_ihave_messages > 0 ? gp->max_ihave_messages : 0)) { /* :624-628 */
                out->ihave_ignored++;
                continue;
            }
            if ((int64_t)o->iasked[q] >= (int64_t)gp->max_ihave_length) { /* :630-633 */
                out->ihave_ignored++;
                continue;
            }
            if (n == 0) continue; /* :652-654 */
            size_t kk = n;
            const size_t budget = (size_t)((int64_t)gp->max_ihave_length - (int64_t)o->iasked[q]);
            if (kk > budget) kk = budget;
            orc_rng g = {seed, 9, (uint64_t)u << 32 | v, tick << 32, 0}; /* (keyed by node ids: shard-invariant) */
            if (n_it + kk > cap_it) {
                while (n_it + kk > cap_it) cap_it *= 2;
                items = (gx_item*)realloc(items, sizeof(gx_item) * cap_it);
            }
            const size_t i0 = n_it;
            if (kk == n) {
                memcpy(items + n_it, W, sizeof(gx_item) * n);
                n_it += n;
            } else { /* a uniform kk-subset of W in canonical order (selection sampling) */
                size_t sel = 0;
                for (size_t i = 0; i < n && sel < kk; i++)
                    if ((size_t)rng_int31n(&g, (int32_t)(n - i)) < kk - sel) {
                        items[n_it++] = W[i];
                        sel++;
                    }
            }
            o->iasked[q] += (uint32_t)kk;
            const gx_item* pm = &items[i0 + (size_t)rng_int31n(&g, (int32_t)kk)]; /* AddPromise's pick (:53) */
            add_promise(o, (uint64_t)q, ((uint64_t)gb[pm->gb].b->set->serial << 32) | pm->k,
                        now + gp->iwant_followup_ns);
            out->iwant_msgs++;
            out->iwant_ids += kk;
            if (n_rq == cap_rq) {
                cap_rq *= 2;
                reqs = (gx_req*)realloc(reqs, sizeof(gx_req) * cap_rq);
            }
            reqs[n_rq].q = (uint64_t)q;
            reqs[n_rq].i0 = i0;
            reqs[n_rq].n = kk;
            reqs[n_rq].served = false;
            n_rq++;
        }
    orc_prof("(D) ihave");
    /* handleIWant at each asked peer v (:681-716): the asker's score, the cache, GetForPeer's count */
    for (size_t i = 0; i < n_rq && !rc; i++) {
        const int64_t r = reverse_pair(o, reqs[i].q);
        if (score0[r] < o->th.gossip_threshold) continue;
        reqs[i].served = true;
        for (size_t j = reqs[i].i0; j < reqs[i].i0 + reqs[i].n; j++) {
            const gx_batch* x = &gb[items[j].gb];
            const uint64_t handle = ((uint64_t)x->b->set->serial << 32) | items[j].k;
            if (!x->avail || peertx_inc(o, (uint64_t)r, handle) > (uint32_t)gp->gossip_retransmission) {
                items[j].gb = UINT32_MAX; /* not sent */
                continue;
            }
            out->iwant_served++;
        }
    }
    /* the askers receive the answers, senders ascending, ids in canonical order */
    orc_msgset** rs = NULL;
    uint8_t** rh = NULL;
    uint32_t* rt = NULL;
    size_t nr = 0;
    gx_recv* fr = NULL; /* the accepted first receipts: each one's hop-0 frontier entry */
    size_t n_fr = 0, cap_fr = 0;
    for (size_t i = 0; i < n_rq && !rc; i++) {
        if (!reqs[i].served) continue;
        const uint64_t q = reqs[i].q;
        const uint32_t u = o->pair_obs[q];
        if (!(o->eflags[q] & GSX_EDGE_DIRECT) && score0[q] < o->th.graylist_threshold) continue; /* AcceptFrom */
        for (size_t j = reqs[i].i0; j < reqs[i].i0 + reqs[i].n; j++) {
            if (items[j].gb == UINT32_MAX) continue;
            const orc_mc_batch* b = gb[items[j].gb].b;
            orc_msgset* st = b->set;
            const uint32_t k = items[j].k, t = b->topic, val = st->val[k];
            uint8_t* sn = &st->seen[(size_t)u * st->m + k];
            if (*sn) { /* DuplicateMessage */
                out->gossip_duplicates++;
                if (val == GSX_VALIDATION_ACCEPT) mark_duplicate(o, q, t, true, now, now);
                else if (val == GSX_VALIDATION_REJECT) mark_invalid(o, q, t);
                continue;
            }
            *sn = 1;
            fulfill_promises(o, u, ((uint64_t)st->serial << 32) | k); /* Validate / Deliver / Reject */
            if (val == GSX_VALIDATION_ACCEPT) {
                out->gossip_delivered++;
                mark_first(o, q, t);
                size_t x = 0;
                while (x < nr && rs[x] != st) x++;
                if (x == nr) {
                    rs = (orc_msgset**)realloc(rs, sizeof(*rs) * (nr + 1));
                    rh = (uint8_t**)realloc(rh, sizeof(*rh) * (nr + 1));
                    rt = (uint32_t*)realloc(rt, sizeof(*rt) * (nr + 1));
                    rs[nr] = st;
                    rh[nr] = (uint8_t*)calloc((size_t)st->m * N, 1);
                    rt[nr] = t;
                    nr++;
                }
                rh[x][(size_t)u * st->m + k] = 1; /* Put into u's cache */
                if (n_fr == cap_fr) {
                    cap_fr = cap_fr ? 2 * cap_fr : 1024;
                    fr = (gx_recv*)realloc(fr, sizeof(gx_recv) * cap_fr);
                }
                fr[n_fr].x = (uint32_t)x; /* u forwards it on, not back to v (below) */
                fr[n_fr].k = k;
                fr[n_fr].u = u;
                fr[n_fr].v = (uint32_t)o->col[q];
                n_fr++;
            } else {
                out->gossip_rejected++;
                if (val == GSX_VALIDATION_REJECT) mark_invalid(o, q, t);
            }
        }
    }
    /* A delivered message is published on at once (pushMsg -> publishMessage
     * -> GossipSubRouter.Publish: pubsub.go:1046-1090, 1124-1128,
     * gossipsub.go:943-1013): each recovering node forwards it to its gossipsub
     * targets but the peer it came from and the origin, and every node that
     * receives it first does the same, in synchronous hops inside the round
     * (every copy at `now`, senders ascending per receiver as in orc_propagate)
     * with the exchange's score snapshot for the publishThreshold and AcceptFrom
     * tests.  A receiver delivers (P2, P3 in the mesh), fulfils its promises,
     * Puts the copy into its cache (the set's recovered batch) and forwards it;
     * a duplicate is inside the P3 window iff the receiver got the message in
     * this round, or else (an old copy: the engine keeps no per-node time)
     * iff now - the set's call time <= MeshMessageDeliveriesWindow. */
    orc_prof("(D) receive");
    if (n_fr) qsort(fr, n_fr, sizeof(gx_recv), gx_recv_cmp);
    if (n_fr) {
        /* the messages' propagations are independent but for the records they
         * credit, the promise table and the counters: threads take whole
         * messages, count the credits per pair (every step of a counter is the
         * same capped +1, so their order is free), log the fulfilments, and
         * everything shared is applied after, in message order */
        size_t n_grp = 0;
        size_t* grp = (size_t*)malloc(sizeof(size_t) * (n_fr + 1));
        for (size_t a = 0; a < n_fr; a++)
            if (a == 0 || fr[a].x != fr[a - 1].x || fr[a].k != fr[a - 1].k) grp[n_grp++] = a;
        grp[n_grp] = n_fr;
        /* every pair's reverse, once (u's peerStats for the sender of each copy) */
        int64_t* rv = (int64_t*)malloc(sizeof(int64_t) * (E ? E : 1));
#pragma omp parallel for schedule(static)
        for (uint64_t r = 0; r < E; r++) rv[r] = reverse_pair(o, r);
        uint32_t* c_first = (uint32_t*)calloc(E ? E : 1, sizeof(uint32_t)); /* per pair: first receipts (P2, P3) */
        uint32_t* c_win = (uint32_t*)calloc(E ? E : 1, sizeof(uint32_t));   /* duplicates inside the window (P3) */
        uint64_t** ful = (uint64_t**)calloc(n_grp, sizeof(uint64_t*));    /* per message: nodes delivered */
        uint32_t* n_ful = (uint32_t*)calloc(n_grp, sizeof(uint32_t));
        uint64_t s_new = 0, s_dup = 0, s_gray = 0;
        uint64_t max_deg = 1;
        for (uint32_t i = 0; i < N; i++)
            if ((uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]) > max_deg) max_deg = (uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]);
        /* one topic at a time: the per-pair counts are then one topic's */
        for (size_t xt = 0; xt < nr; xt++) {
          bool first_of_topic = true;
          for (size_t y = 0; y < xt; y++) first_of_topic &= rt[y] != rt[xt];
          if (!first_of_topic) continue;
          const uint32_t topic = rt[xt];
#pragma omp parallel reduction(+ : s_new, s_dup, s_gray)
        {
            int32_t* from = (int32_t*)malloc(sizeof(int32_t) * (N ? N : 1));
            for (uint32_t i = 0; i < N; i++) from[i] = -1;
            uint32_t* front = (uint32_t*)malloc(sizeof(uint32_t) * (N ? N : 1));
            uint32_t* next = (uint32_t*)malloc(sizeof(uint32_t) * (N ? N : 1));
            uint32_t* touched = (uint32_t*)malloc(sizeof(uint32_t) * (N ? N : 1));
            uint8_t* infront = (uint8_t*)calloc(N ? N : 1, 1);
            uint64_t* tg = (uint64_t*)malloc(sizeof(uint64_t) * max_deg);
            uint64_t* scratch = (uint64_t*)malloc(sizeof(uint64_t) * max_deg);
#pragma omp for schedule(dynamic, 1)
            for (size_t gi = 0; gi < n_grp; gi++) {
                const uint32_t x = fr[grp[gi]].x, k = fr[grp[gi]].k;
                if (rt[x] != topic) continue;
                orc_msgset* st = rs[x];
                const uint32_t t = rt[x], m = st->m;
                uint8_t* has = rh[x];
                gsx_prop_config cfg;
                memset(&cfg, 0, sizeof(cfg));
                cfg.router = GSX_ROUTER_GOSSIPSUB;
                cfg.topic = t;
                uint32_t nf = 0, n_t = 0;
                for (size_t a = grp[gi]; a < grp[gi + 1]; a++) {
                    front[nf++] = fr[a].u;
                    from[fr[a].u] = (int32_t)fr[a].v;
                    touched[n_t++] = fr[a].u;
                }
                const uint32_t n_t0 = n_t;
                while (nf > 0) {
                    /* senders ascending: a receiver meets its copies lowest sender
                     * first (the arrival order of orc_propagate), so each copy is
                     * handled as it is sent; the next frontier is sorted after */
                    uint32_t nn = 0;
                    for (uint32_t i = 0; i < nf; i++) {
                        const uint32_t v = front[i];
                        const int nt = router_targets(o, &cfg, v, st->src[k], from[v], 0, tg, scratch, score0);
                        for (int j = 0; j < nt; j++) {
                            const uint32_t u = (uint32_t)o->col[tg[j]];
                            const int64_t qr = rv[tg[j]]; /* u's peerStats for v */
                            if (qr >= 0 && !(o->eflags[qr] & GSX_EDGE_DIRECT) &&
                                score0[qr] < o->th.graylist_threshold) {
                                s_gray++; /* AcceptFrom (gossipsub.go:583-594) */
                                continue;
                            }
                            uint8_t* sn = &st->seen[(size_t)u * m + k];
                            if (!*sn) { /* Deliver (P2, P3 in the mesh), Put, Publish on */
                                *sn = 1;
                                from[u] = (int32_t)v;
                                touched[n_t++] = u;
                                has[(size_t)u * m + k] = 1;
                                next[nn++] = u;
                                infront[u] = 1;
                                s_new++;
                                if (qr >= 0) __atomic_fetch_add(&c_first[qr], 1u, __ATOMIC_RELAXED);
                            } else { /* DuplicateMessage: P3 inside the window (gsx.h) */
                                s_dup++;
                                const int64_t validated =
                                    has[(size_t)u * m + k] ? now : st->vtime[st->vcode[(size_t)u * m + k]];
                                if (qr >= 0 && now - validated <= o->tp[t < GSX_MAX_TOPICS ? t : 0].mesh_message_deliveries_window_ns)
                                    __atomic_fetch_add(&c_win[qr], 1u, __ATOMIC_RELAXED);
                            }
                        }
                    }
                    /* the next frontier, ascending (a scan when it is large) */
                    if ((uint64_t)nn * 16 > N) {
                        uint32_t c = 0;
                        for (uint32_t u = 0; u < N; u++)
                            if (infront[u]) {
                                front[c++] = u;
                                infront[u] = 0;
                            }
                        nf = c;
                    } else {
                        qsort(next, nn, sizeof(uint32_t), u32_cmp);
                        for (uint32_t i = 0; i < nn; i++) infront[next[i]] = 0;
                        memcpy(front, next, sizeof(uint32_t) * nn);
                        nf = nn;
                    }
                }
                if (n_t > n_t0) { /* the delivered nodes, for fulfillPromise */
                    ful[gi] = (uint64_t*)malloc(sizeof(uint64_t) * (n_t - n_t0));
                    for (uint32_t i = n_t0; i < n_t; i++) ful[gi][i - n_t0] = touched[i];
                    n_ful[gi] = n_t - n_t0;
                }
                for (uint32_t i = 0; i < n_t; i++) from[touched[i]] = -1;
            }
            free(from);
            free(front);
            free(next);
            free(touched);
            free(infront);
            free(tg);
            free(scratch);
        }
          /* the topic's credits, pair by pair: c_first deliveries (markFirstMessageDelivery),
           * c_win duplicates inside the window (markDuplicateMessageDelivery) */
          for (uint64_t q = 0; q < E; q++) {
              for (uint32_t i = 0; i < c_first[q]; i++) mark_first(o, q, topic);
              for (uint32_t i = 0; i < c_win[q]; i++) mark_duplicate(o, q, topic, true, now, now);
              c_first[q] = c_win[q] = 0;
          }
        }
        out->fwd_delivered += s_new;
        out->fwd_duplicates += s_dup;
        out->fwd_graylisted += s_gray;
        for (size_t gi = 0; gi < n_grp; gi++) {
            const orc_msgset* st = rs[fr[grp[gi]].x];
            const uint64_t handle = ((uint64_t)st->serial << 32) | fr[grp[gi]].k;
            for (uint32_t i = 0; i < n_ful[gi]; i++) fulfill_promises(o, (uint32_t)ful[gi][i], handle);
            free(ful[gi]);
        }
        free(ful);
        free(n_ful);
        free(grp);
        free(rv);
        free(c_first);
        free(c_win);
    }
    free(fr);
    /* the recovered copies: one batch per message set, Put after the Shift in
     * ascending set serial (the sets' creation order, gsx.h) */
    for (size_t a = 1; a < nr; a++)
        for (size_t b = a; b > 0 && rs[b - 1]->serial > rs[b]->serial; b--) {
            orc_msgset* ts = rs[b];
            rs[b] = rs[b - 1];
            rs[b - 1] = ts;
            uint8_t* th = rh[b];
            rh[b] = rh[b - 1];
            rh[b - 1] = th;
            uint32_t tt = rt[b];
            rt[b] = rt[b - 1];
            rt[b - 1] = tt;
        }
    /* the copies recovered in this round were validated at `now` (every copy
     * of the exchange and its forwarding is handled at now): one new code per
     * set */
    for (size_t x = 0; x < nr; x++) {
        orc_msgset* st = rs[x];
        if (st->n_vtime >= 0xFFFF) {
            rc = GSX_ERANGE; /* (a set recovered in 65k rounds) */
            continue;
        }
        const uint16_t c = (uint16_t)st->n_vtime++;
        st->vtime = (int64_t*)realloc(st->vtime, sizeof(int64_t) * st->n_vtime);
        st->vtime[c] = now;
        const size_t cells = (size_t)st->m * N;
        for (size_t i = 0; i < cells; i++)
            if (rh[x][i]) st->vcode[i] = c;
    }
    *rec_out = (orc_mc_batch*)calloc(nr ? nr : 1, sizeof(orc_mc_batch));
    *n_rec = nr;
    for (size_t x = 0; x < nr; x++) {
        orc_mc_batch* rb = &(*rec_out)[x];
        const orc_mc_batch* src = NULL;
        for (size_t i = 0; i < nb && !src; i++)
            if (gb[i].b->set == rs[x]) src = gb[i].b;
        rb->topic = rt[x];
        rb->m = rs[x]->m;
        rb->n = N;
        rb->ids = (uint64_t*)malloc(sizeof(uint64_t) * rb->m);
        memcpy(rb->ids, src->ids, sizeof(uint64_t) * rb->m);
        rb->has = rh[x];
        rb->set = rs[x];
        rs[x]->refs++;
    }
    free(rs);
    free(rh);
    free(rt);
    free(gb);
    free(score0);
    free(items);
    free(reqs);
    free(W);
    return rc;
}

/* (B) every node handles the GRAFTs then PRUNEs sent to it (ctl[t][pair of
 * the sender] 1 / 2), senders ascending; PRUNE answers into resp (:718-843) */
/* ---- peer exchange on PRUNE (gossipsub.go:811-843, 861-910, 1814-1850; gsx.h) ---- */

static void px_record(orc_engine* o, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    if (o->n_px == o->cap_px) {
        o->cap_px = o->cap_px ? 2 * o->cap_px : 256;
        o->pxlog = (uint32_t*)realloc(o->pxlog, 16 * o->cap_px);
    }
    uint32_t* x = o->pxlog + 4 * o->n_px++;
    x[0] = a;
    x[1] = b;
    x[2] = c;
    x[3] = d;
}

/* The PX of the round's PRUNEs: kind 0 those of the heartbeats (A) (ctl == 2,
 * sendGraftPrune :1630-1667), kind 1 the (B) answers (resp, handleGraft
 * :800-806).  makePrune (:1814-1850) lists getPeers(topic, PrunePeers, xp != p
 * && score(xp) >= 0) unless the peer lacks feature PX or doPX is off for it;
 * the receiver, if it accepts the RPC and joined the topic, ignores the list
 * below AcceptPXThreshold (:833-838), else pxConnect (:861-910) queues the
 * listed peers it is not connected to (recorded, never dialled).  `cache` is
 * the score snapshot the receiving step reads, which also feeds the lists. */
static void hb_px(orc_engine* o, const gsx_gossipsub_params* gp, int kind, const uint8_t* w, const double* cache,
                  gsx_heartbeat_out* out) {
    const uint64_t E = o->E;
    uint64_t max_deg = 1;
    for (uint32_t i = 0; i < o->n_nodes; i++)
        if ((uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]) > max_deg) max_deg = (uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]);
    uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * max_deg);
    for (uint32_t u = 0; u < o->n_nodes; u++)
        for (int64_t r = o->row_ptr[u]; r < o->row_ptr[u + 1]; r++)
            for (uint32_t t = 0; t < o->T; t++) {
                const uint8_t x = w[(size_t)t * E + r];
                if (kind == 0 ? x != 2 : x == 0) continue;
                if ((o->eflags[r] & GSX_EDGE_NO_PX) || (o->pxno[r] >> kind & 1)) continue;
                const uint32_t p = (uint32_t)o->col[r];
                int n = 0;
                for (int64_t y = o->row_ptr[u]; y < o->row_ptr[u + 1]; y++) {
                    if (y == r || !in_topic(o, (uint64_t)y, t) || !(o->eflags[y] & GSX_EDGE_GOSSIPSUB)) continue;
                    if (!(cache[y] >= 0)) continue;
                    tmp[n++] = (uint64_t)y;
                }
                orc_rng g = {o->px_seed, 12, ((uint64_t)u << 32) | p,
                             (o->px_tick << 32) | ((uint64_t)t << 24) | ((uint64_t)kind << 23), 0};
                shuffle_pairs(tmp, n, &g);
                if (n > gp->prune_peers) n = gp->prune_peers;
                if (n <= 0) continue;
                out->px_prunes++;
                out->px_peers += (uint64_t)n;
                const int64_t q = reverse_pair(o, (uint64_t)r); /* (p -> u) */
                if (q < 0) continue;
                if (!(o->eflags[q] & GSX_EDGE_DIRECT) && cache[q] < o->th.graylist_threshold) continue; /* AcceptFrom */
                if (!joined(o, p, t)) continue;                                                        /* :816-819 */
                if (cache[q] < o->th.accept_px_threshold) {
                    out->px_ignored++;
                    continue;
                }
                for (int i = 0; i < n; i++) {
                    const uint32_t xp = (uint32_t)o->col[tmp[i]];
                    bool connected = false; /* _, connected := gs.peers[p] (:869-872) */
                    for (int64_t z = o->row_ptr[p]; z < o->row_ptr[p + 1]; z++)
                        if ((uint32_t)o->col[z] == xp) {
                            connected = o->ps[z].connected;
                            break;
                        }
                    if (connected) continue;
                    out->px_connect++;
                    px_record(o, p, xp, u, t | (uint32_t)kind << 8);
                }
            }
    free(tmp);
}

static void hb_receive(orc_engine* o, const gsx_gossipsub_params* gp, const uint8_t* ctl, uint8_t* resp, double* cache,
                       int64_t now, gsx_heartbeat_out* out) {
    const uint64_t E = o->E;
    const uint32_t T = o->T;
    for (uint64_t q = 0; q < E; q++) cache[q] = score_pair(o, q); /* gs.score.Score(p) at handling time */
    for (uint32_t u = 0; u < o->n_nodes; u++) {
        for (int64_t q = o->row_ptr[u]; q < o->row_ptr[u + 1]; q++) { /* q = (u -> v), ascending v */
            const int64_t r = reverse_pair(o, (uint64_t)q);         /* r = (v -> u) */
            if (r < 0) continue;
            const double score = cache[q];
            /* AcceptFrom (gossipsub.go:582-593): a graylisted non-direct sender's RPC is dropped */
            if (!(o->eflags[q] & GSX_EDGE_DIRECT) && score < o->th.graylist_threshold) continue;
            bool nopx = false; /* doPX = false for this RPC's PRUNE answers (:721-781) */
            for (uint32_t t = 0; t < T; t++) { /* handleGraft, :718-809 */
                if (ctl[(size_t)t * E + r] != 1) continue;
                if (!joined(o, u, t)) { /* unknown topic: ignored (:727-733) */
                    nopx = true;
                    continue;
                }
                if (hb_in_mesh(o, (uint64_t)q, t)) continue;
                const uint8_t ef = o->eflags[q];
                if (ef & GSX_EDGE_DIRECT) {
                    resp[(size_t)t * E + q] = 1;
                    out->graft_rejected++;
                    nopx = true;
                    continue;
                }
                const int64_t expire = *hb_backoff(o, (uint64_t)q, t);
                if (expire != 0 && now < expire) {
                    nopx = true;
                    add_penalty(o, (uint64_t)q, 1);
                    out->penalties++;
                    if (now < expire + (gp->graft_flood_threshold_ns - gp->prune_backoff_ns)) {
                        add_penalty(o, (uint64_t)q, 1);
                        out->penalties++;
                    }
                    add_backoff(o, (uint64_t)q, t, now, gp->prune_backoff_ns);
                    resp[(size_t)t * E + q] = 1;
                    out->graft_rejected++;
                    continue;
                }
                if (score < 0) {
                    resp[(size_t)t * E + q] = 1;
                    add_backoff(o, (uint64_t)q, t, now, gp->prune_backoff_ns);
                    out->graft_rejected++;
                    nopx = true;
                    continue;
                }
                int n = 0;
                for (int64_t x = o->row_ptr[u]; x < o->row_ptr[u + 1]; x++) n += hb_in_mesh(o, (uint64_t)x, t);
                if (n >= gp->d_hi && !(ef & GSX_EDGE_OUTBOUND)) {
                    resp[(size_t)t * E + q] = 1;
                    add_backoff(o, (uint64_t)q, t, now, gp->prune_backoff_ns);
                    out->graft_rejected++;
                    continue;
                }
                graft(o, (uint64_t)q, t, now); /* tracer.Graft, :795 */
                o->tr_ag[q] |= 1ull << t;
                out->graft_accepted++;
            }
            if (nopx && o->pxno) o->pxno[q] |= 2;
            for (uint32_t t = 0; t < T; t++) /* handlePrune */
                if (ctl[(size_t)t * E + r] == 2 && joined(o, u, t)) /* (:816-819) */
                    handle_prune(o, gp, (uint64_t)q, t, now, out);
        }
    }
}

/* (C) the GRAFT senders handle the PRUNE answers, AcceptFrom-gated */
static void hb_answers(orc_engine* o, const gsx_gossipsub_params* gp, const uint8_t* resp, double* cache, int64_t now,
                       gsx_heartbeat_out* out) {
    const uint64_t E = o->E;
    const uint32_t T = o->T;
    for (uint64_t q = 0; q < E; q++) cache[q] = score_pair(o, q);
    if (o->pxno) hb_px(o, gp, 1, resp, cache, out); /* the answers' PX, on the snapshot (C) reads */
    for (uint32_t v = 0; v < o->n_nodes; v++)
        for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) {
            const int64_t q = reverse_pair(o, (uint64_t)r);
            if (q < 0) continue;
            if (!(o->eflags[r] & GSX_EDGE_DIRECT) && cache[r] < o->th.graylist_threshold) continue;
            for (uint32_t t = 0; t < T; t++)
                if (resp[(size_t)t * E + q] && joined(o, v, t)) handle_prune(o, gp, (uint64_t)r, t, now, out);
        }
}

int orc_heartbeat(orc_engine* o, const gsx_gossipsub_params* gp, uint64_t tick, int64_t now, uint64_t seed,
                  gsx_heartbeat_out* out) {
    memset(out, 0, sizeof(*out));
    orc_prof(NULL);
    o->gp = *gp;
    const uint64_t E = o->E;
    const uint32_t T = o->T;
    /* clearBackoff (:1585-1604) */
    if (tick % 15 == 0)
        for (size_t i = 0; i < (size_t)T * E; i++)
            if (o->backoff[i] != 0 && o->backoff[i] + 2 * HEARTBEAT_INTERVAL_NS < now) {
                o->backoff[i] = 0;
                out->backoff_cleared++;
            }
    /* clearIHaveCounters (:1566-1576), applyIwantPenalties (:1578-1583): a
     * promise whose expiry is before now is broken (GetBrokenPromises, :79-115) */
    memset(o->peerhave, 0, sizeof(uint32_t) * (E ? E : 1));
    memset(o->iasked, 0, sizeof(uint32_t) * (E ? E : 1));
    if (o->n_prom) {
        uint32_t* cnt = (uint32_t*)calloc(E ? E : 1, sizeof(uint32_t));
        out->broken_promises += broken_promises(o, now, cnt);
        for (uint64_t q = 0; q < E; q++) /* AddPenalty(p, count): one addition of the count */
            if (cnt[q]) add_penalty(o, q, cnt[q]);
        free(cnt);
    }
    double* cache = (double*)malloc(sizeof(double) * (E ? E : 1));
    uint8_t* ctl = (uint8_t*)calloc((size_t)T * (E ? E : 1), 1);
    o->n_px = 0;
    free(o->pxno);
    o->pxno = gp->do_px ? (uint8_t*)calloc(E ? E : 1, 1) : NULL;
    o->px_tick = tick;
    o->px_seed = seed;
    memset(o->tr_sg, 0, 8 * (E ? E : 1));
    memset(o->tr_sp, 0, 8 * (E ? E : 1));
    memset(o->tr_ag, 0, 8 * (E ? E : 1));
    memset(o->tr_hp, 0, 8 * (E ? E : 1));
    uint8_t* resp = (uint8_t*)calloc((size_t)T * (E ? E : 1), 1);
    uint64_t max_deg = 1;
    for (uint32_t i = 0; i < o->n_nodes; i++)
        if ((uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]) > max_deg) max_deg = (uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]);
    uint64_t* plst = (uint64_t*)malloc(sizeof(uint64_t) * max_deg);
    uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * max_deg);
    for (uint64_t r = 0; r < E; r++) cache[r] = score_pair(o, r); /* the heartbeat's score cache */
    hb_ctx c = {o, gp, cache, ctl, tick, now, out, seed, NULL, NULL, NULL, 0};
    /* the truncated IHAVE rows of this round: per topic, one bit per gossip position */
    {
        const uint32_t nwin = (uint32_t)gp->history_gossip < o->mc_n ? (uint32_t)gp->history_gossip : o->mc_n;
        size_t pos[GSX_MAX_TOPICS] = {0};
        for (uint32_t w = 0; w < nwin; w++)
            for (size_t b = 0; b < o->mc[w].nb; b++) pos[o->mc[w].b[b].topic] += o->mc[w].b[b].m;
        for (uint32_t t = 0; t < T; t++) {
            o->sub_tw[t] = (uint32_t)((pos[t] + 63) / 64);
            o->sub_n[t] = 0;
            if (o->sub_idx[t]) memset(o->sub_idx[t], 0xFF, sizeof(uint32_t) * (E ? E : 1));
        }
    }
    memset(o->ihave_len, 0, sizeof(uint32_t) * (size_t)T * (E ? E : 1));
    memset(o->ihave_hash, 0, sizeof(uint64_t) * (size_t)T * (E ? E : 1));
    /* (A) every node's heartbeat, every joined topic in ascending order:
     * mesh maintenance, then IHAVE gossip, one draw stream per (node, topic) */
    for (uint32_t v = 0; v < o->n_nodes; v++) {
        for (uint32_t t = 0; t < T; t++) {
            if (!joined(o, v, t)) continue; /* gs.mesh holds the joined topics */
            orc_rng g = {seed, 8, v, (tick << 32) | ((uint64_t)t << 24), 0};
            hb_unit(&c, v, t, &g, plst, tmp);
            emit_gossip(&c, v, t, &g, tmp, false);
        }
        /* expire fanout for topics not published to in a while (:1517-1524) */
        for (uint32_t t = 0; t < T; t++) {
            int64_t* lp = &o->lastpub[(size_t)v * T + t];
            if (*lp != 0 && *lp + gp->fanout_ttl_ns < now) {
                for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) o->fanout[r] &= ~(1ull << t);
                o->fan_has[v] &= ~(1ull << t);
                *lp = 0;
            }
        }
        /* maintain the fanout of topics published to but not joined (:1526-1554);
         * draws h(seed, 8, node, tick << 32 | topic << 24 | 1 << 23 | k) */
        for (uint32_t t = 0; t < T; t++) {
            if (!(o->fan_has[v] >> t & 1)) continue;
            orc_rng g = {seed, 8, v, (tick << 32) | ((uint64_t)t << 24) | (1ull << 23), 0};
            int have = 0;
            for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) {
                if (!(o->fanout[r] >> t & 1)) continue;
                if (!in_topic(o, (uint64_t)r, t) || cache[r] < o->th.publish_threshold) o->fanout[r] &= ~(1ull << t);
                else have++;
            }
            if (have < gp->d) {
                const int k = get_peers(&c, v, t, gp->d - have, F_NOT_FANOUT | F_NOT_DIRECT, 0, o->th.publish_threshold,
                                        tmp, &g);
                for (int i = 0; i < k; i++) o->fanout[tmp[i]] |= 1ull << t;
            }
            emit_gossip(&c, v, t, &g, tmp, true);
        }
    }
    free(c.mids);
    free(c.mpos);
    free(c.msel);
    orc_prof("(A)");
    /* (B) receivers, (C) the PRUNE answers; the (A) PRUNEs' PX on the snapshot (B) read */
    hb_receive(o, gp, ctl, resp, cache, now, out);
    if (o->pxno) hb_px(o, gp, 0, ctl, cache, out);
    hb_answers(o, gp, resp, cache, now, out);
    free(o->pxno);
    o->pxno = NULL;
    for (uint64_t r = 0; r < E; r++)
        for (uint32_t t = 0; t < T; t++) out->mesh_links += hb_in_mesh(o, r, t);
    /* (D) the IHAVEs just emitted are answered across the Shift */
    orc_mc_batch* rec = NULL;
    size_t n_rec = 0;
    orc_prof("(B)(C)");
    int rc = gp->gossip_exchange ? gossip_exchange(o, gp, tick, now, seed, out, &rec, &n_rec) : 0;
    orc_prof("(D)");
    mcache_shift(o, (uint32_t)gp->history_length); /* :1563 */
    if (n_rec && o->mc_n) {
        orc_mc_window* w0 = &o->mc[0];
        for (size_t i = 0; i < n_rec; i++) {
            if (w0->nb == w0->cap) {
                w0->cap = w0->cap ? 2 * w0->cap : 4;
                w0->b = (orc_mc_batch*)realloc(w0->b, sizeof(orc_mc_batch) * w0->cap);
            }
            w0->b[w0->nb++] = rec[i];
        }
    } else {
        for (size_t i = 0; i < n_rec; i++) batch_free(&rec[i]);
    }
    free(rec);
    free(cache);
    free(ctl);
    free(resp);
    free(plst);
    free(tmp);
    return rc;
}

/* ---- topic membership (A13): subscriptions, Join / Leave, fanout export ---- */

int orc_set_gossipsub_params(orc_engine* o, const gsx_gossipsub_params* gp) {
    o->gp = *gp;
    return 0;
}

int orc_set_subscriptions(orc_engine* o, const uint64_t* joined) {
    if (!o->sub) return GSX_ESTATE;
    const uint64_t all = o->T >= 64 ? ~0ull : ((1ull << o->T) - 1);
    for (uint32_t v = 0; v < o->n_nodes; v++) o->sub[v] = joined[v] & all;
    return 0;
}

int orc_export_membership(orc_engine* o, uint64_t* joined, uint64_t* fanout, int64_t* lastpub) {
    if (!o->sub) return GSX_ESTATE;
    if (joined) memcpy(joined, o->sub, 8 * (size_t)o->n_nodes);
    if (fanout) memcpy(fanout, o->fanout, 8 * (size_t)o->E);
    if (lastpub) memcpy(lastpub, o->lastpub, 8 * (size_t)o->n_nodes * o->T);
    return 0;
}

/* candidates of Join / fanout: v's mesh-capable topic peers, not direct, not
 * in the fanout (skip_fanout), live score >= ref; ascending, shuffled, first count */
static int join_peers(orc_engine* o, uint32_t v, uint32_t t, int count, bool skip_fanout, double ref, uint64_t* out,
                      orc_rng* g) {
    int n = 0;
    for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) {
        const uint8_t ef = o->eflags[r];
        if (!in_topic(o, (uint64_t)r, t) || !(ef & GSX_EDGE_GOSSIPSUB) || (ef & GSX_EDGE_DIRECT)) continue;
        if (skip_fanout && (o->fanout[r] >> t & 1)) continue;
        if (!(score_pair(o, (uint64_t)r) >= ref)) continue;
        out[n++] = (uint64_t)r;
    }
    shuffle_pairs(out, n, g);
    if (count >= 0 && n > count) n = count;
    return n;
}

static uint64_t row_max_deg(const orc_engine* o) {
    uint64_t m = 1;
    for (uint32_t i = 0; i < o->n_nodes; i++)
        if ((uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]) > m) m = (uint64_t)(o->row_ptr[i + 1] - o->row_ptr[i]);
    return m;
}

/* Join (gossipsub.go:1015-1064) of (node, topic) entries in order: the mesh
 * from the fanout (negative scores dropped, topped up to D) or getPeers(D);
 * each mesh peer gets tracer.Graft and a GRAFT, which the peers then handle
 * (handleGraft, :718-809) and whose PRUNE answers the joiner handles.
 * Draws h(seed, 11, node, topic << 24 | k). */
int orc_join(orc_engine* o, const uint32_t* nodes, const uint32_t* topics, size_t n, int64_t now, uint64_t seed,
             gsx_heartbeat_out* out) {
    memset(out, 0, sizeof(*out));
    const uint64_t E = o->E;
    const uint32_t T = o->T;
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= o->n_nodes || topics[i] >= T) return GSX_ERANGE;
    uint8_t* ctl = (uint8_t*)calloc((size_t)T * (E ? E : 1), 1);
    uint8_t* resp = (uint8_t*)calloc((size_t)T * (E ? E : 1), 1);
    double* cache = (double*)malloc(sizeof(double) * (E ? E : 1));
    uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * row_max_deg(o));
    const int D = o->gp.d;
    /* the call's subscriptions are announced first (a synchronous round: every
     * joiner sees the others' new subscriptions) */
    uint8_t* todo = (uint8_t*)calloc(n ? n : 1, 1);
    for (size_t i = 0; i < n; i++)
        if (!joined(o, nodes[i], topics[i])) { /* (a repeated entry finds it joined) */
            o->sub[nodes[i]] |= 1ull << topics[i];
            todo[i] = 1;
        }
    for (size_t i = 0; i < n; i++) {
        const uint32_t v = nodes[i], t = topics[i];
        if (!todo[i]) continue;
        orc_rng g = {seed, 11, v, (uint64_t)t << 24, 0};
        if (o->fan_has[v] >> t & 1) {
            int have = 0;
            for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) {
                if (!(o->fanout[r] >> t & 1)) continue;
                if (score_pair(o, (uint64_t)r) < 0) o->fanout[r] &= ~(1ull << t);
                else have++;
            }
            if (have < D) {
                const int k = join_peers(o, v, t, D - have, true, 0.0, tmp, &g);
                for (int j = 0; j < k; j++) o->fanout[tmp[j]] |= 1ull << t;
            }
        } else {
            const int k = join_peers(o, v, t, D, false, 0.0, tmp, &g);
            for (int j = 0; j < k; j++) o->fanout[tmp[j]] |= 1ull << t; /* (the new mesh, staged) */
        }
        for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) { /* the mesh: tracer.Graft + sendGraft */
            if (!(o->fanout[r] >> t & 1)) continue;
            o->fanout[r] &= ~(1ull << t);
            graft(o, (uint64_t)r, t, now);
            ctl[(size_t)t * E + r] = 1;
            out->grafts++;
        }
        o->fan_has[v] &= ~(1ull << t);
        o->lastpub[(size_t)v * T + t] = 0;
    }
    free(todo);
    gsx_gossipsub_params gp = o->gp;
    o->n_px = 0;  /* PX of the GRAFT answers (makePrune in handleGraft, gsx.h) */
    o->pxno = gp.do_px ? (uint8_t*)calloc(E ? E : 1, 1) : NULL;
    o->px_tick = 0;
    o->px_seed = seed;
    hb_receive(o, &gp, ctl, resp, cache, now, out);
    hb_answers(o, &gp, resp, cache, now, out);
    free(o->pxno);
    o->pxno = NULL;
    for (uint64_t r = 0; r < E; r++)
        for (uint32_t t = 0; t < T; t++) out->mesh_links += hb_in_mesh(o, r, t);
    free(ctl);
    free(resp);
    free(cache);
    free(tmp);
    return 0;
}

/* Leave (gossipsub.go:1066-1082): every mesh peer gets tracer.Prune and a
 * PRUNE (handlePrune at the peer, which backs the leaver off). */
int orc_leave(orc_engine* o, const uint32_t* nodes, const uint32_t* topics, size_t n, int64_t now,
              gsx_heartbeat_out* out) {
    memset(out, 0, sizeof(*out));
    const uint64_t E = o->E;
    const uint32_t T = o->T;
    for (size_t i = 0; i < n; i++)
        if (nodes[i] >= o->n_nodes || topics[i] >= T) return GSX_ERANGE;
    uint8_t* ctl = (uint8_t*)calloc((size_t)T * (E ? E : 1), 1);
    uint8_t* resp = (uint8_t*)calloc((size_t)T * (E ? E : 1), 1);
    double* cache = (double*)malloc(sizeof(double) * (E ? E : 1));
    for (size_t i = 0; i < n; i++) {
        const uint32_t v = nodes[i], t = topics[i];
        if (!joined(o, v, t)) continue;
        o->sub[v] &= ~(1ull << t);
        for (int64_t r = o->row_ptr[v]; r < o->row_ptr[v + 1]; r++) {
            if (!hb_in_mesh(o, (uint64_t)r, t)) continue;
            prune(o, (uint64_t)r, t);
            ctl[(size_t)t * E + r] = 2;
            out->prunes++;
        }
    }
    gsx_gossipsub_params gp = o->gp;
    o->n_px = 0;  /* sendPrune -> makePrune(p, topic, doPX) (:1089-1093): PX on every Leave PRUNE */
    o->pxno = gp.do_px ? (uint8_t*)calloc(E ? E : 1, 1) : NULL;
    o->px_tick = 0;
    o->px_seed = 0;
    hb_receive(o, &gp, ctl, resp, cache, now, out);
    if (o->pxno) hb_px(o, &gp, 0, ctl, cache, out);
    free(o->pxno);
    o->pxno = NULL;
    for (uint64_t r = 0; r < E; r++)
        for (uint32_t t = 0; t < T; t++) out->mesh_links += hb_in_mesh(o, r, t);
    free(ctl);
    free(resp);
    free(cache);
    return 0;
}

static int px_cmp(const void* a, const void* b) {
    const uint32_t *x = (const uint32_t*)a, *y = (const uint32_t*)b;
    for (int i = 0; i < 4; i++)
        if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
    return 0;
}
int orc_hb_px_records(orc_engine* o, uint32_t* out, size_t cap, size_t* n) {
    *n = o->n_px;
    qsort(o->pxlog, o->n_px, 16, px_cmp);
    if (cap && out) memcpy(out, o->pxlog, 16 * (cap < o->n_px ? cap : o->n_px));
    return 0;
}

int orc_hb_trace_words(orc_engine* o, uint64_t* sent_graft, uint64_t* sent_prune, uint64_t* acc_graft,
                       uint64_t* handled_prune) {
    if (!o->tr_sg) return GSX_ESTATE;
    if (sent_graft) memcpy(sent_graft, o->tr_sg, 8 * o->E);
    if (sent_prune) memcpy(sent_prune, o->tr_sp, 8 * o->E);
    if (acc_graft) memcpy(acc_graft, o->tr_ag, 8 * o->E);
    if (handled_prune) memcpy(handled_prune, o->tr_hp, 8 * o->E);
    return 0;
}

int orc_export_backoff(orc_engine* o, int64_t* out) {
    memcpy(out, o->backoff, sizeof(int64_t) * (size_t)o->T * o->E);
    return 0;
}

int orc_mcache_ids(orc_engine* o, uint32_t node, uint32_t topic, uint32_t n_windows, uint64_t* out, size_t cap,
                   size_t* n_out) {
    size_t n = 0;
    const uint32_t nw = n_windows < o->mc_n ? n_windows : o->mc_n;
    for (uint32_t w = 0; w < nw; w++)
        for (size_t b = 0; b < o->mc[w].nb; b++) {
            const orc_mc_batch* mb = &o->mc[w].b[b];
            if (topic != GSX_ANY_TOPIC && mb->topic != topic) continue;
            for (uint32_t k = 0; k < mb->m; k++)
                if (mb->has[(size_t)node * mb->m + k]) {
                    if (n < cap) out[n] = mb->ids[k];
                    n++;
                }
        }
    *n_out = n;
    return 0;
}

/* Message-parallel replicas (gsx.h gsx_mcache_*): the newest cached batch's
 * cache membership and message-set rows, [node][n_msgs] bytes each; pop;
 * and Put of a whole batch from its message blocks (block k: the batch's
 * messages [sum part_msgs[<k], + part_msgs[k]), rows [node][part_msgs[k]]),
 * with the publish step's fanout pick for every source (idempotent). */
static orc_mc_batch* mcache_newest(orc_engine* o) {
    if (!o->mc || o->mc_n == 0 || o->mc[0].nb == 0) return NULL;
    return &o->mc[0].b[o->mc[0].nb - 1];
}

int orc_mcache_last(orc_engine* o, uint32_t* n_msgs) {
    const orc_mc_batch* b = mcache_newest(o);
    if (!b) return GSX_ESTATE;
    *n_msgs = b->m;
    return 0;
}

int orc_mcache_copy_last(orc_engine* o, uint8_t* cache_rows, uint8_t* set_rows, uint8_t* hop_rows) {
    const orc_mc_batch* b = mcache_newest(o);
    if (!b || !b->set) return GSX_ESTATE;
    memcpy(cache_rows, b->has, (size_t)b->m * b->n);
    memcpy(set_rows, b->set->seen, (size_t)b->m * b->n);
    if (hop_rows) /* a propagated set's codes are its arrival hops (<= GSX_MAX_HOPS) */
        for (size_t i = 0; i < (size_t)b->m * b->n; i++) hop_rows[i] = (uint8_t)b->set->vcode[i];
    return 0;
}

int orc_mcache_pop(orc_engine* o) {
    orc_mc_batch* b = mcache_newest(o);
    if (!b) return GSX_ESTATE;
    if (b->set && b->set->serial == o->msg_serial && b->set->refs == 1) o->msg_serial--;
    batch_free(b);
    o->mc[0].nb--;
    return 0;
}

int orc_mcache_put(orc_engine* o, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg, uint32_t n_parts,
                   const uint32_t* part_msgs, const uint8_t* const* cache_parts, const uint8_t* const* set_parts,
                   const uint8_t* const* hop_parts) {
    if (!o->mc || !m || cfg->router != GSX_ROUTER_GOSSIPSUB) return GSX_EINVAL;
    size_t tot = 0;
    for (uint32_t k = 0; k < n_parts; k++) tot += part_msgs[k];
    if (tot != m) return GSX_EINVAL;
    fanout_publish(o, msgs, m, cfg, NULL);
    const uint32_t N = o->n_nodes;
    orc_mc_window* w0 = &o->mc[0];
    if (w0->nb == w0->cap) {
        w0->cap = w0->cap ? 2 * w0->cap : 4;
        w0->b = (orc_mc_batch*)realloc(w0->b, sizeof(orc_mc_batch) * w0->cap);
    }
    orc_mc_batch* b = &w0->b[w0->nb++];
    b->topic = cfg->topic;
    b->m = (uint32_t)m;
    b->n = N;
    b->ids = (uint64_t*)malloc(sizeof(uint64_t) * m);
    b->has = (uint8_t*)calloc(m * (size_t)(N ? N : 1), 1);
    b->set = (orc_msgset*)calloc(1, sizeof(orc_msgset));
    b->set->serial = ++o->msg_serial;
    b->set->m = (uint32_t)m;
    b->set->n = N;
    b->set->refs = 1;
    b->set->val = (uint32_t*)malloc(sizeof(uint32_t) * m);
    b->set->src = (uint32_t*)malloc(sizeof(uint32_t) * m);
    b->set->t0 = cfg->now_ns;
    b->set->seen = (uint8_t*)calloc(m * (size_t)(N ? N : 1), 1);
    b->set->vcode = (uint16_t*)calloc(m * (size_t)(N ? N : 1), sizeof(uint16_t));
    b->set->n_vtime = cfg->max_hops + 1;
    b->set->vtime = (int64_t*)malloc(sizeof(int64_t) * b->set->n_vtime);
    for (uint32_t h = 0; h <= cfg->max_hops; h++)
        b->set->vtime[h] = cfg->now_ns + (int64_t)h * (cfg->hop_latency_ns + cfg->validation_delay_ns);
    for (size_t k = 0; k < m; k++) {
        b->ids[k] = msgs[k].msg_id;
        b->set->val[k] = msgs[k].validation;
        b->set->src[k] = msgs[k].source;
    }
    size_t off = 0;
    for (uint32_t k = 0; k < n_parts; k++) {
        const size_t nk = part_msgs[k];
        for (uint32_t i = 0; i < N && nk; i++) {
            memcpy(b->has + (size_t)i * m + off, cache_parts[k] + (size_t)i * nk, nk);
            memcpy(b->set->seen + (size_t)i * m + off, set_parts[k] + (size_t)i * nk, nk);
            if (hop_parts && hop_parts[k])
                for (size_t j = 0; j < nk; j++)
                    b->set->vcode[(size_t)i * m + off + j] = hop_parts[k][(size_t)i * nk + j];
        }
        off += nk;
    }
    return 0;
}

int orc_gossip_results(orc_engine* o, uint32_t* len, uint64_t* hash) {
    if (len) memcpy(len, o->ihave_len, sizeof(uint32_t) * (size_t)o->T * o->E);
    if (hash) memcpy(hash, o->ihave_hash, sizeof(uint64_t) * (size_t)o->T * o->E);
    return 0;
}

int orc_import_backoff(orc_engine* o, const int64_t* in) {
    memcpy(o->backoff, in, sizeof(int64_t) * (size_t)o->T * o->E);
    return 0;
}

/* ------------------------------------------------------------------------ */

int orc_import_state(orc_engine* o, const gsx_state_view* s) {
    uint64_t E = o->E;
    for (uint64_t p = 0; p < E; p++) {
        orc_peer_stats* ps = &o->ps[p];
        ps->present = (s->pair_flags[p] & GSX_PAIR_PRESENT) != 0;
        ps->connected = (s->pair_flags[p] & GSX_PAIR_CONNECTED) != 0;
        ps->expire = s->expire_ns[p];
        ps->behaviour_penalty = s->behaviour_penalty[p];
        for (uint32_t t = 0; t < o->T; t++) {
            size_t r = (size_t)t * E + p;
            orc_topic_stats* ts = &o->ts[p * o->T + t];
            ts->first_message_deliveries = s->first_message_deliveries[r];
            ts->mesh_message_deliveries = s->mesh_message_deliveries[r];
            ts->mesh_failure_penalty = s->mesh_failure_penalty[r];
            ts->invalid_message_deliveries = s->invalid_message_deliveries[r];
            ts->graft_time = s->graft_time_ns[r];
            ts->mesh_time = s->mesh_time_ns[r];
            ts->in_mesh = (s->rec_flags[r] & GSX_REC_IN_MESH) != 0;
            ts->mesh_message_deliveries_active = (s->rec_flags[r] & GSX_REC_ACTIVE) != 0;
        }
    }
    ipcount_rebuild(o);
    o->last_refresh = s->last_refresh_ns;
    return 0;
}

int orc_export_state(orc_engine* o, gsx_state_view* s) {
    s->last_refresh_ns = o->last_refresh;
    uint64_t E = o->E;
    for (uint64_t p = 0; p < E; p++) {
        const orc_peer_stats* ps = &o->ps[p];
        if (s->pair_flags) s->pair_flags[p] = (uint8_t)((ps->present ? GSX_PAIR_PRESENT : 0) |
                                                        (ps->connected ? GSX_PAIR_CONNECTED : 0));
        if (s->expire_ns) s->expire_ns[p] = ps->expire;
        if (s->behaviour_penalty) s->behaviour_penalty[p] = ps->behaviour_penalty;
        static const orc_topic_stats none; /* a deleted peerStats has no topicStats: export zeros */
        for (uint32_t t = 0; t < o->T; t++) {
            size_t r = (size_t)t * E + p;
            const orc_topic_stats* ts = ps->present ? &o->ts[p * o->T + t] : &none;
            if (s->first_message_deliveries) s->first_message_deliveries[r] = ts->first_message_deliveries;
            if (s->mesh_message_deliveries) s->mesh_message_deliveries[r] = ts->mesh_message_deliveries;
            if (s->mesh_failure_penalty) s->mesh_failure_penalty[r] = ts->mesh_failure_penalty;
            if (s->invalid_message_deliveries) s->invalid_message_deliveries[r] = ts->invalid_message_deliveries;
            if (s->graft_time_ns) s->graft_time_ns[r] = ts->graft_time;
            /* meshTime is only read while in the mesh (score.go:279, 479-481); the view reports 0 otherwise */
            if (s->mesh_time_ns) s->mesh_time_ns[r] = ts->in_mesh ? ts->mesh_time : 0;
            if (s->rec_flags)
                s->rec_flags[r] = (uint8_t)((ts->in_mesh ? GSX_REC_IN_MESH : 0) |
                                            (ts->mesh_message_deliveries_active ? GSX_REC_ACTIVE : 0));
        }
    }
    return 0;
}
