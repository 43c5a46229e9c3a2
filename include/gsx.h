/*
 * gsx.h — C ABI of the MI355X-native GossipSub scoring engine.
 *
 * This is the drop-in boundary for the reference's peer-scoring path
 * (`/root/reference/score.go`, `score_params.go`).  In the reference the scorer
 * is the concrete type `*peerScore` held by the router (`gossipsub.go:425`) and
 * reached through `WithPeerScore` (`gossipsub.go:263-304`), `Score()`
 * (`score.go:247`), `AddPenalty()` (`score.go:384`), `SetTopicScoreParams()`
 * (`score.go:194`), the RawTracer methods it implements (`score.go:588-830`)
 * and its background ticker (`score.go:401-438`).  Every entry point below
 * names the reference function it replaces.
 *
 * Model.  One engine holds the state of MANY observers (routers) at once: an
 * overlay in CSR form, observer i owning the directed "pairs"
 * row_ptr[i] .. row_ptr[i+1]-1, pair p standing for the reference's
 * `peerStats` entry that observer keeps for neighbour col[p].  A Go cgo shim
 * that replaces `score.go` inside one router uses one observer whose pairs
 * are its peer slots.  Topics are dense indices 0..n_topics-1 (the host maps
 * topic strings to indices, like `ps.params.Topics[topic]`).
 *
 * Conventions.
 *  - Every function returns 0 on success or a negative errno-style code
 *    (GSX_E*).  Nothing throws or aborts across the ABI.
 *  - The caller owns every host buffer; the engine copies to HBM.
 *  - One engine is externally synchronised (the reference serialises with
 *    `peerScore`'s own mutex, `score.go:65`).  Work is ordered on the
 *    engine's HIP stream; gsx_sync() waits for it.
 *  - Times are int64 nanoseconds on a caller-supplied clock: the reference
 *    reads `time.Now()` inside the scorer (`score.go:501,636,657,711,839`);
 *    the engine takes `now_ns` as an argument instead.
 *  - There is no CPU fallback: without a usable gfx950 device gsx_create
 *    fails with GSX_ENODEV.
 */
#ifndef GSX_H
#define GSX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSX_ABI_VERSION 5

/* ---- status codes ------------------------------------------------------ */
#define GSX_OK 0
#define GSX_EINVAL (-22)  /* bad argument / params failed validate()        */
#define GSX_ENOMEM (-12)  /* host or device allocation failed                */
#define GSX_ENODEV (-19)  /* no HIP device / kernel image for this device    */
#define GSX_ERANGE (-34)  /* index out of range                              */
#define GSX_ESTATE (-71)  /* call out of order (e.g. no overlay loaded)      */
#define GSX_EDEVICE (-5)  /* HIP runtime error                               */

/* ---- parameters (score_params.go) ---------------------------------------- */

/* TopicScoreParams, score_params.go:98-148.  Durations are nanoseconds. */
typedef struct gsx_topic_score_params {
    double topic_weight;
    /* P1 */
    double time_in_mesh_weight;
    int64_t time_in_mesh_quantum_ns;
    double time_in_mesh_cap;
    /* P2 */
    double first_message_deliveries_weight;
    double first_message_deliveries_decay;
    double first_message_deliveries_cap;
    /* P3 */
    double mesh_message_deliveries_weight;
    double mesh_message_deliveries_decay;
    double mesh_message_deliveries_cap;
    double mesh_message_deliveries_threshold;
    int64_t mesh_message_deliveries_window_ns;
    int64_t mesh_message_deliveries_activation_ns;
    /* P3b */
    double mesh_failure_penalty_weight;
    double mesh_failure_penalty_decay;
    /* P4 */
    double invalid_message_deliveries_weight;
    double invalid_message_deliveries_decay;
} gsx_topic_score_params;

/* PeerScoreParams, score_params.go:53-96, minus the three fields that are not
 * plain data in Go:
 *   Topics                      -> gsx_set_topic_params() per topic index
 *   AppSpecificScore (closure)  -> gsx_set_app_scores() snapshot per pair
 *   IPColocationFactorWhitelist -> gsx_set_ip_whitelist() per IP id
 * `app_specific_score_set` mirrors the `AppSpecificScore == nil` check of
 * validate() (score_params.go:165). */
typedef struct gsx_peer_score_params {
    double topic_score_cap;
    double app_specific_weight;
    int32_t app_specific_score_set;
    int32_t ip_colocation_factor_threshold;
    double ip_colocation_factor_weight;
    double behaviour_penalty_weight;
    double behaviour_penalty_threshold;
    double behaviour_penalty_decay;
    int64_t decay_interval_ns;
    double decay_to_zero;
    int64_t retain_score_ns;
} gsx_peer_score_params;

/* PeerScoreThresholds, score_params.go:12-32. */
typedef struct gsx_thresholds {
    double gossip_threshold;
    double publish_threshold;
    double graylist_threshold;
    double accept_px_threshold;
    double opportunistic_graft_threshold;
} gsx_thresholds;

/* validate() twins: PeerScoreParams.validate (score_params.go:151-198, topic
 * validation is separate), TopicScoreParams.validate (:200-268),
 * PeerScoreThresholds.validate (:34-51).  Return 0 or GSX_EINVAL. */
int gsx_validate_peer_params(const gsx_peer_score_params* p);
int gsx_validate_topic_params(const gsx_topic_score_params* p);
int gsx_validate_thresholds(const gsx_thresholds* p);

/* ScoreParameterDecayWithBase, score_params.go:282-287 (integer Duration
 * division, then pow).  ScoreParameterDecay(d) == ..._with_base(d, 1s, 0.01). */
double gsx_score_parameter_decay_with_base(int64_t decay_ns, int64_t base_ns, double decay_to_zero);
double gsx_score_parameter_decay(int64_t decay_ns);

/* ---- engine lifecycle ----------------------------------------------------- */

typedef struct gsx_engine gsx_engine;

typedef struct gsx_config {
    uint32_t n_topics;   /* dense topic indices 0..n_topics-1, <= GSX_MAX_TOPICS */
    int32_t device;      /* HIP device ordinal                                   */
    uint32_t reserved[6];
} gsx_config;

#define GSX_MAX_TOPICS 64

int gsx_create(const gsx_config* cfg, gsx_engine** out);
int gsx_destroy(gsx_engine* e);
/* Last HIP / engine error as text (valid until the next call). */
const char* gsx_last_error(gsx_engine* e);
int gsx_abi_version(void);

/* newPeerScore(params) / the threshold copy of WithPeerScore
 * (score.go:180-188, gossipsub.go:282-287).  Like newPeerScore these do NOT
 * validate: WithPeerScore = gsx_validate_* (gossipsub.go:270-280) followed by
 * these setters, and the reference's unit tests build scorers from
 * unvalidated params (e.g. DecayToZero 0). */
int gsx_set_peer_params(gsx_engine* e, const gsx_peer_score_params* p);
int gsx_set_thresholds(gsx_engine* e, const gsx_thresholds* t);
/* SetTopicScoreParams (score.go:194-234): installs params for `topic`; if the
 * topic was already scored and a delivery cap is lowered, recaps fmd/mmd of
 * every record of that topic on the device.  Does NOT validate (the reference
 * notes "assumes that the topic score parameters have already been
 * validated"); call gsx_validate_topic_params first, as Topic.SetScoreParams
 * does (topic.go:36-74). */
int gsx_set_topic_params(gsx_engine* e, uint32_t topic, const gsx_topic_score_params* p);

/* Edge flags, one byte per pair. */
#define GSX_EDGE_OUTBOUND 0x01u  /* gs.outbound[p] (gossipsub.go:510-537)     */
#define GSX_EDGE_DIRECT 0x02u    /* gs.direct[p]                               */
#define GSX_EDGE_GOSSIPSUB 0x04u /* peer speaks a mesh protocol (feature Mesh) */
#define GSX_EDGE_FLOODSUB 0x08u  /* peer speaks floodsub                       */
#define GSX_EDGE_NO_PX 0x10u     /* mesh peer without feature PX (gossipsub v1.0,
                                    gossipsub_feat.go:28-34): its PRUNEs carry no
                                    peer exchange (makePrune, gossipsub.go:1815-1818) */

#define GSX_NO_IP 0xFFFFFFFFu

/* Overlay in CSR: n_nodes observers; row_ptr[n_nodes+1]; col[row_ptr[n]] are
 * neighbour node ids (the peer each pair stands for).  edge_flags may be NULL
 * (all zero).  node_ips[2*n] gives up to two IP ids per node (IPv4, or IPv6
 * address + /64: score.go:1002-1013), GSX_NO_IP for none; may be NULL.
 * Every pair starts NOT present (no peerStats), as before AddPeer. */
int gsx_load_overlay(gsx_engine* e, uint32_t n_nodes, const int64_t* row_ptr, const int32_t* col,
                     const uint8_t* edge_flags, const uint32_t* node_ips);
int gsx_num_pairs(gsx_engine* e, uint64_t* out_pairs);

/* IPColocationFactorWhitelist (score.go:346-367), resolved on the host to the
 * list of whitelisted IP ids.  Replaces any previous list. */
int gsx_set_ip_whitelist(gsx_engine* e, const uint32_t* ip_ids, size_t n);

/* AppSpecificScore snapshot (score.go:320): app[p] for every pair. */
int gsx_set_app_scores(gsx_engine* e, const double* app, size_t n_pairs);
/* setIPs (score.go:1021-1059) for pairs whose peer the observer now sees on
 * other addresses: refreshIPs (score.go:560-586) calls it for its connected
 * peers, a shim's AddPeer before the GSX_EV_ADD_PEER of a peer whose
 * addresses changed.  ips: 2 per pair (GSX_NO_IP for none; an IPv6 peer's
 * address + /64).  A present pair (connected or retained) leaves the
 * (observer, IP) sets of its old list and joins those of the new one; an
 * absent pair only records the list, counted by its next AddPeer.  Applied
 * after the queued events, in the order given. */
int gsx_set_pair_ips(gsx_engine* e, const uint64_t* pairs, const uint32_t* ips, size_t n);

/* ---- events: the RawTracer calls that mutate counters --------------------- */

enum gsx_event_kind {
    GSX_EV_ADD_PEER = 1,         /* AddPeer           score.go:588-602                 */
    GSX_EV_REMOVE_PEER = 2,      /* RemovePeer        score.go:604-637                 */
    GSX_EV_GRAFT = 3,            /* Graft             score.go:642-660                 */
    GSX_EV_PRUNE = 4,            /* Prune             score.go:662-684                 */
    GSX_EV_FIRST_DELIVERY = 5,   /* markFirstMessageDelivery     score.go:912-939      */
    GSX_EV_MESH_DELIVERY = 6,    /* markDuplicateMessageDelivery score.go:944-974,
                                    window already checked by the caller               */
    GSX_EV_INVALID_DELIVERY = 7, /* markInvalidMessageDelivery   score.go:894-907      */
    GSX_EV_PENALTY = 8,          /* AddPenalty(p, arg) score.go:384-398                */
    GSX_EV_APP_SCORE = 9         /* AppSpecificScore(p) as score() reads it (score.go:320):
                                    arg = the IEEE-754 bits of the pair's new value    */
};

/* 32-byte event record.  `pair` selects (observer, peer); `topic` is used by
 * GRAFT, PRUNE and the DELIVERY kinds; `arg` is the penalty count for PENALTY
 * and the application score's bits for APP_SCORE (a one-pair
 * gsx_set_app_scores: a router re-reads AppSpecificScore(p) only for the peer
 * it scores, and the engine re-scores only that observer's row). */
typedef struct gsx_event {
    uint32_t kind;
    uint32_t topic;
    uint64_t pair;
    int64_t now_ns;
    int64_t arg;
} gsx_event;

/* Appends events; they are applied on the device, in the given order per
 * observer, before the next refresh/score/export call (or at gsx_flush). */
int gsx_apply_events(gsx_engine* e, const gsx_event* ev, size_t n);
int gsx_flush(gsx_engine* e);

/* ---- message-level tracer calls (delivery records, score.go:686-870) ----- */
/* These keep the reference's per-message delivery records (status, validated
 * time, peers that delivered a duplicate) keyed by (observer, msg_id) on the
 * host and turn them into the counter events above.  `pair` is the
 * ReceivedFrom peer as seen by its observer.  Self-published messages must not
 * be traced (trace.go:98,110,141,171). */
enum gsx_reject_reason {
    GSX_REJECT_BLACKLISTED_PEER = 0,   /* "blacklisted peer"        tracer.go:28 */
    GSX_REJECT_BLACKLISTED_SOURCE = 1, /* "blacklisted source"      tracer.go:29 */
    GSX_REJECT_MISSING_SIGNATURE = 2,  /* "missing signature"       tracer.go:30 */
    GSX_REJECT_UNEXPECTED_SIGNATURE = 3,
    GSX_REJECT_UNEXPECTED_AUTH_INFO = 4,
    GSX_REJECT_INVALID_SIGNATURE = 5,
    GSX_REJECT_VALIDATION_QUEUE_FULL = 6,
    GSX_REJECT_VALIDATION_THROTTLED = 7,
    GSX_REJECT_VALIDATION_FAILED = 8,
    GSX_REJECT_VALIDATION_IGNORED = 9,
    GSX_REJECT_SELF_ORIGIN = 10        /* "self originated message" tracer.go:38 */
};

int gsx_trace_validate(gsx_engine* e, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now_ns);
int gsx_trace_deliver(gsx_engine* e, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now_ns);
int gsx_trace_reject(gsx_engine* e, uint64_t pair, uint64_t msg_id, uint32_t topic, int32_t reason,
                     int64_t now_ns);
int gsx_trace_duplicate(gsx_engine* e, uint64_t pair, uint64_t msg_id, uint32_t topic, int64_t now_ns);
/* messageDeliveries.gc (score.go:856-870): drop records with expire < now. */
int gsx_gc_deliveries(gsx_engine* e, int64_t now_ns);
int gsx_num_delivery_records(gsx_engine* e, uint64_t* out);

/* ---- refresh and evaluation ----------------------------------------------- */

/* refreshScores (score.go:497-558): purge expired retained pairs, decay every
 * connected pair's counters, update meshTime / activation, decay P7 — fused on
 * the device with the evaluation of score() (score.go:258-335) for every
 * pair, whose result stays in HBM. */
int gsx_refresh(gsx_engine* e, int64_t now_ns);

/* score() for every pair (score.go:258-335; 0 for pairs with no peerStats).
 * Re-evaluates on the device if anything changed since the last refresh. */
int gsx_scores(gsx_engine* e, double* out, size_t n_pairs);
/* Score(p) for one pair (score.go:247-256). */
int gsx_score(gsx_engine* e, uint64_t pair, double* out);
/* Score(p) for n pairs at once (out[i] for pairs[i]): what one RPC of a
 * router asks (AcceptFrom, gossipsub.go:589; the Publish targets and their
 * thresholds, :960-989) with one flush of the queued tracer calls, one
 * re-score and one copy.  On an engine of at most 65,536 pairs whose host
 * score copy was current, the flush, the re-score of the touched observers'
 * rows and the copy are one kernel launch that writes the host-mapped copy and
 * signals a host-mapped flag (no stream synchronisation). */
int gsx_score_many(gsx_engine* e, const uint64_t* pairs, size_t n, double* out);
/* Device pointer of the score vector (valid until the next call). */
int gsx_device_scores(gsx_engine* e, const double** dptr);

int gsx_sync(gsx_engine* e);
/* Queues every deferred score update: the queued events, and the re-scores a
 * gossipsub propagation's credit fold leaves to the next score reader (pairs
 * whose score was at or above every forwarding threshold and only rose: the
 * fwd bytes stay exact meanwhile).  Every score reader settles them itself;
 * this puts the work at a point of the caller's choosing (e.g. right after a
 * batch, as the fold would have done). */
int gsx_settle_scores(gsx_engine* e);

/* ---- state import / export (inspection, synthetic workloads, checkpoints) -- */
/* Record arrays are topic-major: element [t * n_pairs + p].  Mirrors the
 * fields of topicStats (score.go:37-62) and peerStats (score.go:17-35). */
#define GSX_REC_IN_MESH 0x01u
#define GSX_REC_ACTIVE 0x02u
#define GSX_PAIR_PRESENT 0x01u   /* a peerStats entry exists              */
#define GSX_PAIR_CONNECTED 0x02u /* peerStats.connected                   */

typedef struct gsx_state_view {
    /* per record, n_topics * n_pairs */
    double* first_message_deliveries;
    double* mesh_message_deliveries;
    double* mesh_failure_penalty;
    double* invalid_message_deliveries;
    int64_t* graft_time_ns;
    int64_t* mesh_time_ns;
    uint8_t* rec_flags; /* GSX_REC_* */
    /* per pair, n_pairs */
    uint8_t* pair_flags; /* GSX_PAIR_* */
    int64_t* expire_ns;
    double* behaviour_penalty;
    /* time of the last refreshScores() pass (0 if none) */
    int64_t last_refresh_ns;
} gsx_state_view;

/* Import overwrites all state (and rebuilds the per-observer IP counters from
 * the present pairs); export copies it back.  NULL members are skipped on
 * export; on import every member must be non-NULL.
 *
 * mesh_time_ns is topicStats.meshTime, which the reference only reads while
 * the peer is in the mesh (score.go:279, 479-481): export writes 0 for
 * records not in the mesh, and import requires every in-mesh record's
 * meshTime to be either 0 (grafted since the last refresh) or
 * last_refresh_ns - graft_time_ns (what that refresh wrote, score.go:545);
 * any other value is GSX_EINVAL (the engine derives meshTime instead of
 * streaming it). */
int gsx_import_state(gsx_engine* e, const gsx_state_view* s);
int gsx_export_state(gsx_engine* e, gsx_state_view* s);

/* WithPeerScoreInspect's extended view (ExtendedPeerScoreInspectFn,
 * inspectScoresExtended score.go:463-493): a PeerScoreSnapshot per pair
 * whose observer keeps peerStats for the peer (present = 1), its
 * TopicScoreSnapshot per topic.  NULL members are skipped.
 * Differences: Topics covers every topic index (a topicStats the reference
 * never created reads as zeros, which is what it contributes); the app score
 * is the last gsx_set_app_scores snapshot, not a fresh closure call. */
typedef struct gsx_score_snapshot {
    /* per pair, n_pairs (PeerScoreSnapshot, score.go:125-131) */
    uint8_t* present;
    double* score;
    double* app_specific_score;
    double* ip_colocation_factor; /* unweighted P6 */
    double* behaviour_penalty;
    /* per record, [topic][pair] (TopicScoreSnapshot, score.go:133-138) */
    int64_t* time_in_mesh_ns; /* meshTime while in the mesh, else 0 */
    double* first_message_deliveries;
    double* mesh_message_deliveries;
    double* invalid_message_deliveries;
} gsx_score_snapshot;
int gsx_peer_score_snapshot(gsx_engine* e, gsx_score_snapshot* s);

/* Seeded synthetic counter state, generated on the device (BASELINE.md cfg3
 * initialisation).  Every draw is u = (h(seed, 4, a, k) >> 11) * 2^-53 with
 * h the SplitMix64-based counter hash of gsx/synth.py, a = t*n_pairs + p for
 * records and a = p for pairs:
 *   fmd = u1*fmd_max, mmd = u2*mmd_max, mfp = u3*mfp_max,
 *   imd = col[p] >= sybil_first_node ? u4*imd_max_sybil : 0,
 *   inMesh = u5 < p_in_mesh, graftTime = now - (int64)(u6*graft_window_ns),
 *   meshTime = inMesh ? now - graftTime : 0,
 *   pair = present|connected; present only if u7 < p_disconnected; absent if
 *   u8 < p_absent; expire = now + (int64)((u9 - 0.5)*expire_jitter_ns),
 *   bp = u10*bp_max.
 * Rebuilds the IP counters like gsx_import_state. */
typedef struct gsx_synth_spec {
    uint64_t seed;
    int64_t now_ns;
    double fmd_max, mmd_max, mfp_max, imd_max_sybil;
    double p_in_mesh;
    int64_t graft_window_ns;
    double bp_max;
    double p_disconnected, p_absent;
    int64_t expire_jitter_ns;
    uint32_t sybil_first_node;
    uint32_t reserved;
} gsx_synth_spec;

int gsx_synthesize_state(gsx_engine* e, const gsx_synth_spec* spec);

/* Timing of the most recent fused refresh+score launch, measured with HIP
 * events on the engine stream (ms).  Requires gsx_sync. */
int gsx_last_refresh_ms(gsx_engine* e, float* ms);

/* ---- message propagation (floodsub / gossipsub / randomsub forwarding) ---- */
/* Synchronous-hop restatement of the forwarding path (SURVEY.md §7, §8a
 * A13-A14): pushMsg's seen-dedup (pubsub.go:1046-1090, 919-936) and the
 * routers' Publish (floodsub.go:76-100, gossipsub.go:943-1013,
 * randomsub.go:99-160) over the loaded overlay.
 *   - hop 0: message m is published at its source (origin = source);
 *   - hop h: every vertex that first saw m at hop h-1 sends it to its
 *     router's targets for the topic, except the peer it first got m from and
 *     the origin (floodsub.go:82, gossipsub.go:1007, randomsub.go:113);
 *   - a vertex first seeing m at hop h records the LOWEST-indexed sender of
 *     that hop as its first deliverer; later or other copies are duplicates;
 *   - "in topic" (ps.topics[topic]) = the pair is present and connected;
 *     mesh membership = the scorer's inMesh flag of (pair, topic), which the
 *     router keeps in step through Graft/Prune traces;
 *   - a receiver validates for validation_delay_ns before it delivers and
 *     forwards; a duplicate is inside the P3 window iff it arrives at most
 *     MeshMessageDeliveriesWindow after the first copy finished validating
 *     (score.go:965); a message validation does not accept (gsx_msg.validation)
 *     is seen but neither delivered nor forwarded;
 *   - gossipsub only: a receiver u drops every copy from a sender v that is
 *     not one of its direct peers and whose score (u's record of v) is below
 *     GraylistThreshold — AcceptFrom (gossipsub.go:583-594) returns
 *     AcceptNone and handleIncomingRPC drops the whole RPC before pushMsg
 *     (pubsub.go:1014-1017): not seen, no Deliver / Duplicate / Reject trace,
 *     no P2 / P3 / P4; counted in gsx_prop_out.graylisted.  Floodsub and
 *     RandomSub accept everything (AcceptAll);
 *   - score gates (graylist, publishThreshold, flood publish) read the scores
 *     as they stand when the call starts; the call's credits land at its end
 *     (a sequence of calls is a sequence of RPCs: the next call sees them).
 * With credit_scores set, first receipts and duplicates are folded into the
 * receiver's counters exactly as DeliverMessage / DuplicateMessage would
 * (score.go:695-719, 788-820: +1 then cap, one step per message). */
enum gsx_router { GSX_ROUTER_FLOODSUB = 0, GSX_ROUTER_GOSSIPSUB = 1, GSX_ROUTER_RANDOMSUB = 2 };

typedef struct gsx_prop_config {
    uint32_t router;          /* gsx_router                                        */
    uint32_t topic;           /* the messages' topic                               */
    uint32_t flood_publish;   /* WithFloodPublish (gossipsub.go:306-317, 953-960)  */
    uint32_t max_hops;        /* hop bound, <= GSX_MAX_HOPS                        */
    int64_t hop_latency_ns;   /* simulated time per hop                           */
    int64_t now_ns;           /* publish time                                      */
    uint32_t credit_scores;   /* GSX_CREDIT_*: fold deliveries into P2/P3 counters */
    uint32_t randomsub_size;  /* RandomSub's `size` (randomsub.go:21-27)           */
    uint64_t seed;            /* RandomSub draws: h(seed, 7, vertex, msg_id<<16|k) */
    int64_t validation_delay_ns; /* time a receiver validates before forwarding / delivering
                                  * (validation.go:230-351); >= 0.  A hop takes
                                  * hop_latency_ns + validation_delay_ns, and a duplicate is inside
                                  * the P3 window iff it arrives <= window after the first copy
                                  * finished validating (score.go:806-809, 965). */
} gsx_prop_config;

#define GSX_MAX_HOPS 64

/* Validation outcome of a message at every receiver (validation.go:230-351,
 * score.go:721-786).  A message that is not accepted is marked seen but not
 * delivered, not forwarded and not cached (it travels one hop, from its
 * source); REJECT (ValidationFailed) adds one invalid delivery (P4) to the
 * sender's record, IGNORE and THROTTLE penalise nobody. */
#define GSX_VALIDATION_ACCEPT 0u
#define GSX_VALIDATION_REJECT 1u
#define GSX_VALIDATION_IGNORE 2u
#define GSX_VALIDATION_THROTTLE 3u

typedef struct gsx_msg {
    uint32_t source;      /* publishing node (the origin)  */
    uint32_t validation;  /* GSX_VALIDATION_*              */
    uint64_t msg_id;      /* used by RandomSub's draws     */
} gsx_msg;

typedef struct gsx_prop_out {
    uint64_t deliveries;     /* first receipts by vertices other than the source */
    uint64_t duplicates;     /* receipts of an already seen message             */
    uint64_t transmissions;  /* sends: deliveries + duplicates + rejected + ignored + graylisted */
    uint32_t hops;           /* last hop with a first receipt                   */
    uint32_t hop_launches;   /* hop (and pack) launches timed in hop_kernel_ms  */
    uint64_t hop_deliveries[GSX_MAX_HOPS + 1]; /* first receipts per hop       */
    /* Push-minimal traffic terms of SURVEY.md §8d, summed over hops and
     * 64-message words: (pair, word) with a non-empty eligible send, and
     * (vertex, word) gaining new bits. */
    uint64_t edge_sends;
    uint64_t new_words;
    double hop_kernel_ms;    /* device time of the hop / pack kernels (HIP events) */
    uint64_t rejected;       /* receipts of REJECT messages (RejectMessage, P4 to the sender) */
    uint64_t ignored;        /* receipts of IGNORE / THROTTLE messages                      */
    uint64_t graylisted;     /* copies dropped by the receiver's AcceptFrom (gossipsub only):
                              * sender not direct and scored below GraylistThreshold       */
} gsx_prop_out;

/* credit_scores values */
#define GSX_CREDIT_OFF 0u
#define GSX_CREDIT_NOW 1u   /* fold this call's credits at its end              */
#define GSX_CREDIT_DEFER 2u /* add them to the pending counts (gsx_prop_fold_credits) */

/* Propagates m messages (any m; processed in 64-message words). */
int gsx_propagate(gsx_engine* e, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg, gsx_prop_out* out);
/* Per (node, message) results of the last propagation: arrival hop
 * (0xFF = never; 0 at the source) and first deliverer node (global id, -1 =
 * none), laid out [message][node] over this engine's nodes.  Either pointer
 * may be NULL. */
int gsx_prop_results(gsx_engine* e, uint8_t* hop, int32_t* first_from);
/* Duplicate receipts of the last propagation (the copies pushMsg traces as
 * DuplicateMessage, pubsub.go:1046-1060 -> trace.go:136-164): rows[pair *
 * n_words + w] bit b is set when the pair's neighbour sent its observer a
 * copy of message 64 * w + b that the observer had already seen.  The copy
 * arrived at hop hop(message, neighbour) + 1.  Copies the observer's
 * AcceptFrom drops (graylisted senders) are not duplicates: they are never
 * pushed.  The popcount over all rows equals gsx_prop_out.duplicates.  Needs
 * first-deliverer tracking (gsx_prop_set_tracking) in that call, an
 * unsharded engine, and n_words = ceil(m / 64) of the call; replaces the
 * reference's per-copy tracer call with one export (f4).  Host buffer of
 * n_pairs * n_words u64. */
int gsx_prop_duplicates(gsx_engine* e, uint64_t* rows, size_t n_words);
/* Whether propagation keeps, per pair, the messages its observer first got
 * from the neighbour (the deliveryRecord's first deliverer, score.go:833-854)
 * for gsx_prop_results' first_from.  On by default.  Off, a call keeps only
 * per-pair counts (P2/P3 credits and duplicate accounting are unchanged)
 * and gsx_prop_results(first_from != NULL) fails with GSX_ESTATE; the hop
 * kernel then does no per-pair row read-modify-writes.  RandomSub keeps the
 * rows either way (its draws exclude the peer a message came from). */
int gsx_prop_set_tracking(gsx_engine* e, uint32_t first_deliverers);

/* Pending P2/P3 credit counts per pair (first receipts, in-window duplicates)
 * accumulated by GSX_CREDIT_DEFER calls.  Pointers may be host or device
 * memory (n_pairs u32 each; NULL skips).  Message-parallel replicas sum
 * them across ranks (RCCL all-reduce) and fold the sums: folding the sum of
 * counts is exactly folding every message's steps (they are all "+1 then
 * cap"). */
int gsx_prop_pending_credits(gsx_engine* e, uint32_t* first, uint32_t* dup);
/* Pending invalid-delivery counts per pair (REJECT messages, P4), n_pairs
 * u32, host or device memory: read, or replace (message-parallel replicas sum
 * them like the credits).  gsx_prop_fold_credits folds them into imd. */
int gsx_prop_pending_invalid(gsx_engine* e, uint32_t* inv);
int gsx_prop_replace_pending_invalid(gsx_engine* e, const uint32_t* inv);
/* Folds credit counts into fmd / mmd of the pending topic (score.go:912-974)
 * and clears them.  first/dup (both or neither, host or device memory)
 * replace the pending counts before folding. */
int gsx_prop_fold_credits(gsx_engine* e, const uint32_t* first, const uint32_t* dup);

/* Orders the engine's work on a caller's HIP stream (hipStream_t; NULL = the
 * engine's own), e.g. torch's current stream, so that its kernels and the
 * caller's RCCL collectives on the same device are stream-ordered. */
int gsx_set_stream(gsx_engine* e, void* stream);

/* ---- range sharding ------------------------------------------ */
/* One engine per rank owns nodes node_lo .. node_lo + n_local - 1 of an
 * n_total-node overlay: row_ptr has n_local + 1 entries, col holds GLOBAL
 * node ids, node_ips covers all n_total nodes.  Scoring needs nothing else
 * (every pair belongs to its observer's rank).  Propagation exchanges, per
 * hop, what each cross-shard pair (v -> u) sends:
 *   gsx_shard_recv_plan  -> this rank's receive list (u local, v remote),
 *                           grouped by v's rank, pairs ascending; the host
 *                           sends list k to rank k;
 *   gsx_shard_send_plan  <- the lists the other ranks sent here, concatenated
 *                           in rank order;
 *   gsx_prop_begin, then per hop gsx_prop_pack (send rows, [n_send][words])
 *   -> all-to-all (send counts per rank x words u64) -> gsx_prop_step (the
 *   received rows) until a hop delivers nothing on any rank, gsx_prop_end.
 * Words per call: 1 for m <= 64, 2 for m <= 128, else ceil(m/64) rounded up
 * to a multiple of 4.  Per-rank results equal the single-engine run's rows
 * of those nodes bit for bit. */
int gsx_load_overlay_shard(gsx_engine* e, uint32_t n_total, uint32_t node_lo, uint32_t n_local,
                           const int64_t* row_ptr, const int32_t* col, const uint8_t* edge_flags,
                           const uint32_t* node_ips);
/* rank_lo[n_ranks + 1]: rank k owns rank_lo[k] .. rank_lo[k+1]-1.  Writes
 * recv_counts[n_ranks] and, if non-NULL, the (u, v) global ids per slot. */
int gsx_shard_recv_plan(gsx_engine* e, uint32_t n_ranks, const uint32_t* rank_lo, uint64_t* recv_counts,
                        uint32_t* recv_u, uint32_t* recv_v);
int gsx_shard_send_plan(gsx_engine* e, const uint64_t* send_counts, const uint32_t* req_u, const uint32_t* req_v);
int gsx_shard_counts(gsx_engine* e, uint64_t* n_send, uint64_t* n_recv);
/* Compacted exchange (only non-empty rows travel): dest_halo_base[k] = the
 * receive slot, on rank k, of the first row this rank sends to k (rank k's
 * receive slots run source rank by source rank, so it is the sum of what
 * k receives from ranks below this one). */
int gsx_shard_set_halo_bases(gsx_engine* e, const uint64_t* dest_halo_base);

/* Stepped propagation (any engine; required on a shard).  gsx_propagate is
 * begin + max_hops steps + end.  send / recv are device pointers (rows of
 * the call's word count); gsx_prop_step returns the hop's first receipts on
 * this rank in *n_new (NULL: no host sync). */
int gsx_prop_begin(gsx_engine* e, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg);
int gsx_prop_pack(gsx_engine* e, uint64_t* send);
int gsx_prop_step(gsx_engine* e, const uint64_t* recv, uint64_t* n_new);
int gsx_prop_end(gsx_engine* e, gsx_prop_out* out);
/* Compacted per-hop exchange: out (device, n_send x (words + 1) u64) gets,
 * for destination k, counts[k] (host) entries [receive slot on k][words]
 * starting at entry send_base[k] (the dense segment's first slot); only
 * non-empty rows are written.  The receiver passes the entries it got (in
 * any order, concatenated) to gsx_prop_step_compact, which scatters them
 * into the engine's own halo and runs the hop. */
int gsx_prop_pack_compact(gsx_engine* e, uint64_t* out, uint64_t* counts);
int gsx_prop_step_compact(gsx_engine* e, const uint64_t* entries, uint64_t n_entries, uint64_t* n_new);
/* As gsx_prop_pack_compact with the counts left on the device, ordered on the
 * engine's stream (no host sync): d_counts (device, n_ranks x 2 i64) gets
 * (entries for rank k, this rank's first receipts of hop P.h — the hop just
 * run).  One all-to-all of these pairs gives every receiver its entry counts
 * and, summed, whether the previous hop delivered anything on any rank, so a
 * sharded hop needs one host round trip (RangeSharded). */
int gsx_prop_pack_compact_dev(gsx_engine* e, uint64_t* out, int64_t* d_counts);
/* The first receipts of hops 0 .. GSX_MAX_HOPS of the call in flight on this
 * rank, copied to d_out (device, GSX_MAX_HOPS + 1 i64) in stream order with no
 * host sync: with the dense exchange (gsx_prop_pack / gsx_prop_step with
 * n_new NULL) a driver runs several hops back to back and sums these over the
 * ranks once per chunk to find the hop that delivered nothing anywhere (the
 * hops after it deliver nothing and change nothing). */
int gsx_prop_hop_counts_dev(gsx_engine* e, int64_t* d_out);
/* Range shards, before gsx_prop_end: the last hop of the call in flight that
 * delivered on ANY rank (the ranks' hop counts summed; 0: none).  The call's
 * message set keeps the validation times of hops 0 .. last_hop (gsx.h (D)),
 * the same table on every rank and on one engine holding the whole overlay
 * (which takes its own last delivering hop); without it a shard keeps every
 * hop it launched.  Unsharded engines ignore it. */
int gsx_prop_set_last_hop(gsx_engine* e, uint32_t last_hop);

/* Range shards, the replicated frontier.  A lean call (every duplicate inside
 * the P3 window or no credits, no RandomSub draws, no first-deliverer rows;
 * GSX_SHARD_PAIRS=1 in the environment turns it off) keeps every node's
 * frontier row of the last two hops on every rank, so a remote sender's row is
 * gathered as a local one and the hops exchange whole frontier rows instead
 * of per-pair rows (gsx_prop_pack* / gsx_prop_step* are then refused).  The
 * reference's semantics are unchanged (floodsub.go:76-100, gossipsub.go:943-
 * 1013): the `from` exclusion never changes a first receipt, so each cross
 * pair's copies are accounted once, at the call's end.  A driver runs, after
 * gsx_prop_begin:
 *   gsx_prop_rep              whether this call does (1) or takes the per-pair
 *                             exchange (0);
 *   gsx_prop_rep_fwd_pack     the fwd byte of every send slot's pair (device,
 *                             n_send bytes), moved like a hop's dense rows
 *                             (send splits -> receive splits) and handed to
 *   gsx_prop_rep_fwd_recv     (device, n_recv bytes): the remote pins;
 *   gsx_prop_rep_step         hop 1 with no parts (hop 0 is known everywhere:
 *                             the message list), then per hop h >= 2 ...
 *   gsx_prop_rep_pack_dev     this rank's rows of the hop just run: entries
 *                             [global node id][W words] into out (device,
 *                             room for n_local entries), and d_counts[0] =
 *                             entries, d_counts[1] = this rank's first
 *                             receipts of that hop (device i64, no sync);
 *   gsx_prop_rep_step         the other ranks' entries (parts[k]: device,
 *                             counts[k] entries each, host arrays) and the
 *                             next hop, until a hop delivered nothing on any
 *                             rank;
 *   gsx_prop_rep_sends_pack   per send slot, what its pair sent over the call
 *                             (device u64: sends | own unaccepted copies << 32;
 *                             one-word calls: sends | copies << 16 | the hops
 *                             its row was non-empty << 32, the edge sends),
 *                             moved like the fwd bytes to
 *   gsx_prop_rep_sends_recv   (device u64 per receive slot): duplicates (P3
 *                             credits) or graylisted copies at the receivers;
 * then gsx_prop_set_last_hop and gsx_prop_end as for the per-pair exchange.
 *
 * Dense rows instead of entries (no host read per hop): after the fwd bytes,
 *   gsx_prop_rep_rows(e, 1)   for this call (before hop 1: no very sparse
 *                             marking, remote rows mark no receivers);
 *   gsx_prop_rep_step         hop 1 with no parts, then per hop h >= 2:
 *   gsx_prop_rep_rows_export  this rank's slice of the hop's rows (device,
 *                             n_local x W words) and its occupancy-bit row
 *                             (device, (n_total + 63) / 64 + 1 words) ...
 *   gsx_prop_rep_rows_step    ... every rank's slice (parts[k]: rank k's
 *                             rows, the shard plan's ranges; one all-gather)
 *                             and the bit rows summed over the ranks (one
 *                             all-reduce: the ranks own disjoint bits), then
 *                             the next hop; the driver reads the summed
 *                             per-hop receipts (gsx_prop_hop_counts_dev) once
 *                             per chunk of hops to find the end: the hops
 *                             after an empty one run empty and change nothing. */
int gsx_prop_rep(gsx_engine* e, uint32_t* on);
int gsx_prop_rep_rows(gsx_engine* e, uint32_t on);
int gsx_prop_rep_rows_export(gsx_engine* e, uint64_t* rows, uint64_t* occ);
int gsx_prop_rep_rows_step(gsx_engine* e, uint32_t n_parts, const uint64_t* const* parts, const uint64_t* occ_sum);
int gsx_prop_rep_fwd_pack(gsx_engine* e, uint8_t* out);
int gsx_prop_rep_fwd_recv(gsx_engine* e, const uint8_t* in);
int gsx_prop_rep_pack_dev(gsx_engine* e, uint64_t* out, int64_t* d_counts);
int gsx_prop_rep_step(gsx_engine* e, uint32_t n_parts, const uint64_t* const* parts, const uint64_t* counts);
int gsx_prop_rep_sends_pack(gsx_engine* e, uint64_t* out);
int gsx_prop_rep_sends_recv(gsx_engine* e, const uint64_t* in);

/* ---- heartbeat mesh maintenance (gossipsub.go:1303-1564) ------------------- */

/* The GossipSubParams fields the heartbeat and its control handling read
 * (gossipsub.go:62-199); gsx_default_gossipsub_params gives
 * DefaultGossipSubParams (gossipsub.go:230-260). */
typedef struct gsx_gossipsub_params {
    int32_t d, d_lo, d_hi, d_score, d_out;  /* GossipSubD/Dlo/Dhi/Dscore/Dout   :33-37 */
    int32_t opportunistic_graft_peers;      /* :54                               */
    uint64_t opportunistic_graft_ticks;     /* :53                               */
    int64_t prune_backoff_ns;               /* :47                               */
    int64_t graft_flood_threshold_ns;       /* :55                               */
    int32_t d_lazy;                         /* :40                               */
    int32_t history_length, history_gossip; /* :38, :238 (HistoryGossip = 5!)   */
    int32_t max_ihave_length;               /* :56                               */
    double gossip_factor;                   /* :41                               */
    int32_t max_ihave_messages;             /* :57                               */
    int32_t gossip_retransmission;          /* :42                               */
    int64_t iwant_followup_ns;              /* :58                               */
    int32_t gossip_exchange;                /* 1 (default): run step (D) below (handleIHave /
                                               handleIWant, :615-720); 0: IHAVEs are only emitted */
    int32_t reserved0;
    int64_t fanout_ttl_ns;                  /* :45 (GossipSubFanoutTTL)          */
    int32_t do_px;                          /* WithPeerExchange (:325-333); default 0 */
    int32_t prune_peers;                    /* :46 (GossipSubPrunePeers = 16)    */
} gsx_gossipsub_params;

/* With gossip_exchange on, one gossipsub batch (a gsx_propagate / gsx_prop_begin
 * call, or a gsx_mcache_put) holds at most this many messages (GSX_ERANGE
 * otherwise: split the batch over several calls); the forwarding of recovered
 * messages counts back-sends per message set group in 16 bits. */
#define GSX_GX_MAX_SET_MSGS 65535u

int gsx_default_gossipsub_params(gsx_gossipsub_params* out);
int gsx_set_gossipsub_params(gsx_engine* e, const gsx_gossipsub_params* p);

/* One heartbeat of every node at once, a synchronous round:
 *  (A) every (node, topic) runs the mesh maintenance of gossipsub.go:1344-1510
 *      with the scores of the heartbeat start (the router's per-heartbeat
 *      cache, :1333-1341): prune negative-score peers, graft up to D when below
 *      Dlo, prune down to D keeping Dscore by score and Dout outbound when
 *      above Dhi, top up outbound peers, opportunistic graft every
 *      OpportunisticGraftTicks; Graft/Prune traces update the scorer, pruned
 *      peers are backed off (:845-859);
 *  (B) every node handles the GRAFTs then PRUNEs sent to it (handleGraft /
 *      handlePrune, :718-843), senders in ascending order, with the scores of
 *      that moment: backoff / score / Dhi checks, P7 penalties for GRAFTs
 *      inside the backoff (:752-770), PRUNE answers;
 *  (C) the GRAFT senders handle those PRUNE answers;
 *  (D) (gossip_exchange) the IHAVEs of (A) are handled: every node, senders
 *      ascending, runs handleIHave (:615-679) on the one IHAVE RPC it got from
 *      each peer (all topics): score >= GossipThreshold, peerhave <=
 *      MaxIHaveMessages, iasked < MaxIHaveLength, ids it has not seen; it
 *      asks for min(|iwant|, MaxIHaveLength - iasked) of them (a uniform
 *      subset, selection sampling with draws h(seed, 9, u << 32 | v, tick << 32 | k)
 *      over the canonical order topic / cache order / message index) and
 *      tracks one promise (AddPromise, gossip_tracer.go:48-75: the element at
 *      Int31n(asked) in canonical order, expiring IWantFollowupTime later);
 *      the peer answers (handleIWant, :681-716) if the asker's score >=
 *      GossipThreshold, with every asked message still in its cache after
 *      this heartbeat's Shift (mcache.GetForPeer: the oldest advertised window
 *      is gone when HistoryGossip == HistoryLength, the reference default);
 *      the asker then receives them, senders ascending, ids in canonical
 *      order: a first receipt is delivered (P2/P3 credit, or P4 when its
 *      validation rejects it), fulfils the node's promises for it
 *      (gossip_tracer.go:119-153) and is Put into its cache window 0 (after
 *      the Shift: one batch per message set, in the sets' creation order);
 *      a further copy is a duplicate.  A delivered message is published on
 *      at once (pushMsg -> Publish, pubsub.go:1046-1128, gossipsub.go:943-1013):
 *      the recovering node forwards it to its gossipsub targets (direct
 *      peers, floodsub peers >= PublishThreshold, its mesh) but the peer that
 *      served it and the origin, and every node receiving it first does the
 *      same, in synchronous hops within the round (every copy at `now`;
 *      per receiver senders ascending; the publishThreshold and AcceptFrom
 *      tests read the scores as (D) started); a forwarded first receipt is
 *      delivered (P2, P3 in the mesh), fulfils promises and is Put into the
 *      same recovered batch; a forwarded duplicate counts for P3 (in the
 *      mesh) iff now - the time the receiver's copy finished validating <=
 *      MeshMessageDeliveriesWindow (score.go:944-974: drec.validated per
 *      (observer, message)): `now` for a copy of this round; for an older
 *      one, the call's now_ns + arrival hop * (hop_latency_ns +
 *      validation_delay_ns) (its source: now_ns) when it came with the
 *      propagation, or the `now` of the heartbeat whose exchange recovered
 *      it.  The engine keeps these times as a code per (node, message) over a
 *      short per-set time list (bit planes beside the set's seen rows, built
 *      from the call's arrival hops when hop_latency_ns + validation_delay_ns
 *      > 0 and the gossip exchange is on), so a window boundary that falls
 *      between two arrival hops splits the copies exactly as the reference
 *      does.  A set cached while the exchange was off keeps no hops: a later
 *      round whose window would split its copies fails with GSX_ESTATE.
 *      At the start of every heartbeat
 *      the IHAVE counters are cleared (:1566-1576) and promises that expired
 *      before now are broken: AddPenalty(peer, count) (:1578-1583, P7).
 *      A truncated IHAVE list (below) is handled as the subset its target
 *      got.  The promises of a pair are unbounded (gossip_tracer.go:59-74:
 *      the engine doubles its per-pair slots whenever a pair could fill them).
 * Randomness (shufflePeers, :1890-1895) is Go's Int31n rejection rule over
 * draws h(seed, 8, node, tick << 32 | topic << 24 | k); candidate lists are in
 * ascending peer order; the unstable sort.Slice of :1393 is a stable sort
 * after the shuffle.  clearBackoff runs when tick % 15 == 0 (:1585-1604).
 * All nodes are subscribed to (joined) every topic; "in topic" = present and
 * connected; mesh membership is the scorer's inMesh flag.
 * After the maintenance of (node, topic) the node emits IHAVE gossip for that
 * topic (emitGossip, :1669-1723) from its message cache (mcache.go): the ids
 * of the gossipsub batches it saw (gsx_propagate with the gossipsub router
 * Puts every message a node receives or publishes into its cache window 0;
 * within a batch the insertion order is ascending message index), read
 * newest window first over HistoryGossip windows; the list's order is never
 * observable (a receiver collects it into a set, :643-650), so it is not
 * shuffled and draws nothing; targets are the non-mesh, non-direct
 * mesh-capable topic peers whose live score (after the node's maintenance of
 * topics <= t) is >= GossipThreshold, max(Dlazy, GossipFactor * |eligible|)
 * of them, shuffled.  A list of L > MaxIHaveLength ids reaches each target
 * as its own uniform MaxIHaveLength-subset (the reference reshuffles the list
 * per target and keeps a prefix, :1708-1720, which gives i.i.d. uniform
 * subsets): Floyd's sampling of k = min(MaxIHaveLength, L - MaxIHaveLength)
 * positions of the list (for j = L - k .. L - 1: x = Int31n(j + 1), take x
 * unless taken, else j) with draws h(seed, 13, node << 32 | peer, tick << 32
 * | topic << 24 | fan << 23 | k) (fan: the fanout pass), the taken positions
 * when k == MaxIHaveLength, else the others.
 * Every heartbeat ends with mcache.Shift() (:1563).  */
typedef struct gsx_heartbeat_out {
    uint64_t grafts;          /* peers grafted by the heartbeats (A)              */
    uint64_t prunes;          /* peers pruned by the heartbeats (A)               */
    uint64_t graft_accepted;  /* GRAFTs accepted by their receivers (B)            */
    uint64_t graft_rejected;  /* GRAFTs answered with PRUNE (B)                    */
    uint64_t prunes_handled;  /* handlePrune calls (B + C)                         */
    uint64_t penalties;       /* AddPenalty(p, 1) calls (B)                        */
    uint64_t backoff_cleared; /* entries dropped by clearBackoff                   */
    uint64_t mesh_links;      /* in-mesh (pair, topic) after the round             */
    uint64_t ihave_msgs;      /* IHAVE control messages emitted (emitGossip)       */
    uint64_t ihave_ids;       /* message ids advertised over all of them           */
    uint64_t broken_promises; /* IWANT promises expired unfulfilled (AddPenalty)   */
    uint64_t ihave_ignored;   /* IHAVE RPCs ignored: score / MaxIHaveMessages / iasked (D) */
    uint64_t iwant_msgs;      /* IWANT requests sent (D)                           */
    uint64_t iwant_ids;       /* message ids requested in them                     */
    uint64_t iwant_served;    /* messages sent back by handleIWant (D)             */
    uint64_t gossip_delivered;  /* first receipts of served messages, accepted (D) */
    uint64_t gossip_rejected;   /* first receipts validation did not accept (D)    */
    uint64_t gossip_duplicates; /* further copies of served messages (D)           */
    uint64_t px_prunes;       /* PRUNEs sent with a non-empty PX list (do_px)      */
    uint64_t px_peers;        /* peer ids listed in them                           */
    uint64_t px_ignored;      /* PX lists ignored: receiver's score of the sender
                                 below AcceptPXThreshold (:833-838)               */
    uint64_t px_connect;      /* listed peers the receiver is not connected to:
                                 pxConnect's connection candidates (:861-910)     */
    uint64_t fwd_delivered;   /* first receipts of recovered messages forwarded on (D) */
    uint64_t fwd_duplicates;  /* further copies of them                             */
    uint64_t fwd_graylisted;  /* copies of them the receiver's AcceptFrom dropped   */
} gsx_heartbeat_out;

int gsx_heartbeat(gsx_engine* e, uint64_t tick, int64_t now_ns, uint64_t seed, gsx_heartbeat_out* out);

/* Allocates (and clears) the heartbeat's device buffers for the loaded
 * overlay and the current gossipsub params now instead of at the first
 * gsx_heartbeat: the round state (GRAFT/PRUNE words, marks, IHAVE slots, mesh
 * counts), with the gossip exchange on its promise / IHAVE / request arrays and
 * the forwarding's frontier and per-pair buffers, and the truncated-list bound
 * of the topics (a host pass over the rows).  The setup the reference's router
 * does when it attaches (gossipsub.go:467-510, NewGossipSub's maps), so the
 * first round costs what every round costs.  Optional; idempotent. */
int gsx_hb_reserve(gsx_engine* e);

/* The gossipTracer's promises of every router (gossip_tracer.go:48-185; one
 * router per observer, keyed by its pair to the promising peer and the
 * message handle: the message set's serial << 32 | index inside the engine,
 * any 64-bit id through these calls), the state step (D) keeps:
 *  gsx_promise_add      AddPromise(p, msgIDs) (:48-75): tracks handles[Int31n(n)]
 *                       (draws h(seed, 9, pair, k)) expiring at expire_ns,
 *                       unless that (pair, message) promise exists;
 *                       GSX_EINVAL for expire_ns == 0 (the engine's free-slot
 *                       mark; AddPromise's expiry is now + IWantFollowupTime);
 *  gsx_promise_broken   GetBrokenPromises (:79-115): the promises expired
 *                       before now are dropped and counted per pair (counts
 *                       [n_pairs], may be NULL; no penalty: the heartbeat
 *                       applies AddPenalty itself);
 *  gsx_promise_fulfill  fulfillPromise (:119-126, Deliver / Validate / Reject):
 *                       drops every promise of the node for the message;
 *  gsx_promise_throttle ThrottlePeer (:167-185): drops the pair's promises;
 *  gsx_promise_count    promises outstanding. */
int gsx_promise_add(gsx_engine* e, uint64_t pair, const uint64_t* handles, uint32_t n, int64_t expire_ns,
                    uint64_t seed);
int gsx_promise_broken(gsx_engine* e, int64_t now_ns, uint32_t* counts, uint64_t* total);
int gsx_promise_fulfill(gsx_engine* e, uint32_t node, uint64_t handle);
int gsx_promise_throttle(gsx_engine* e, uint64_t pair);
int gsx_promise_count(gsx_engine* e, uint64_t* n);
/* The same round in steps, for a range shard (required there; any engine
 * may use them): gsx_hb_begin runs (A); gsx_hb_pack_ctl writes, per send
 * slot of the shard plan, the GRAFT and PRUNE bits of the pair it carries
 * ([n_send][2] u64, device); after the all-to-all, gsx_hb_recv runs (B) with
 * the received [n_recv][2] words; gsx_hb_pack_resp writes the PRUNE answers
 * per send slot ([n_send] u64); after the second all-to-all gsx_hb_end runs
 * (C), fills *out with this rank's counters and shifts the message cache. */
int gsx_hb_begin(gsx_engine* e, uint64_t tick, int64_t now_ns, uint64_t seed);
int gsx_hb_pack_ctl(gsx_engine* e, uint64_t* send);
int gsx_hb_recv(gsx_engine* e, const uint64_t* halo_ctl);
int gsx_hb_pack_resp(gsx_engine* e, uint64_t* send);
int gsx_hb_end(gsx_engine* e, const uint64_t* halo_resp, gsx_heartbeat_out* out);
/* The gossip exchange (D) on a range shard (gossip_exchange on): gsx_hb_end
 * runs (C) and prepares (D); these steps carry it across the ranks and
 * gsx_gx_end ends the round (its counters then; gsx_hb_end's *out is zero).
 * Everything (D) computes belongs to the receiver of an IHAVE (its counters,
 * promises, records, receipts and cache), so a cross-shard pair needs from
 * the sender's rank only the IHAVE's topics, whether the sender answers
 * IWANTs (its score of the receiver), and its cache rows of the advertised
 * batches when they hold a message some node lacks; the forwarding of
 * recovered messages needs the senders' topic slots and, per hop, their
 * frontier rows and back-send counts.  All travel as entries routed by the
 * shard plan's receive slots.  An IHAVE list truncated to MaxIHaveLength on
 * a cross-shard pair reaches the receiver as the subset its target got: the
 * sender's rank draws it as one engine does (the draws are keyed by global
 * node ids) and sends that topic's cache rows of the pair masked with it, so
 * the entry layout is the same for whole and truncated lists.
 * While a sharded exchange is in flight (gsx_gx_pending), every call that
 * starts a round, a propagation, a Join / Leave or a state import / export
 * fails with GSX_ESTATE until gsx_gx_end.
 *   gsx_gx_pending      1 when one is in flight (*n_sets: its message sets), else 0
 *   gsx_gx_common       this rank's common words, [n_sets][64] u64 (host): the
 *                       messages every node of the rank had seen
 *   gsx_gx_set_common   their AND over every rank (the caller's all-gather)
 *   gsx_gx_pack_ihave   per send slot: IHAVE topic bits, answer bit ([n_send][2], device)
 *   gsx_gx_recv_ihave   the received [n_recv][2] words
 *   gsx_gx_rows_words   the sender-row entry width (1 + the advertised batches' words)
 *   gsx_gx_rows_pack    this rank's sender-row entries: with out null the
 *                       count pass (counts[n_ranks]), then the pack into out
 *                       (device, destination by destination; the same for gsx_gxf_pack)
 *   gsx_gx_rows_recv    the received entries (read until gsx_gx_exchange returns)
 *   gsx_gx_exchange     handleIHave / handleIWant and the receipts; *n_runs:
 *                       forwarding runs (each: begin, pack_fout / recv_fout,
 *                       then per hop h = 1, 2, ...: pack, the all-to-all, step,
 *                       until a hop leaves no frontier on any rank; end)
 *   gsx_gxf_step        hop h with the received entries; *n_front: this rank's new frontier
 *                       (NULL: no host sync; see gsx_gxf_pack_dev)
 *   gsx_gx_got          per message set: a node of this rank delivered one of its messages
 *   gsx_gx_end          with their OR over every rank: the merge, the Shift, the
 *                       recovered copies Put (the same batches on every rank) */
int gsx_gx_pending(gsx_engine* e, uint32_t* n_sets);
int gsx_gx_common(gsx_engine* e, uint64_t* common);
int gsx_gx_set_common(gsx_engine* e, const uint64_t* common);
int gsx_gx_pack_ihave(gsx_engine* e, uint64_t* send);
int gsx_gx_recv_ihave(gsx_engine* e, const uint64_t* recv);
int gsx_gx_rows_words(gsx_engine* e, uint32_t* words);
int gsx_gx_rows_pack(gsx_engine* e, uint64_t* counts, uint64_t* out);
int gsx_gx_rows_recv(gsx_engine* e, const uint64_t* entries, uint64_t n);
int gsx_gx_exchange(gsx_engine* e, uint32_t* n_runs);
int gsx_gxf_begin(gsx_engine* e, uint32_t run);
int gsx_gxf_entry_words(gsx_engine* e, uint32_t* words);
int gsx_gxf_pack_fout(gsx_engine* e, uint64_t* send);
int gsx_gxf_recv_fout(gsx_engine* e, const uint64_t* recv);
int gsx_gxf_pack(gsx_engine* e, uint32_t hop, uint64_t* counts, uint64_t* out);
int gsx_gxf_step(gsx_engine* e, uint32_t hop, const uint64_t* entries, uint64_t n, uint64_t* n_front);
/* gsx_gxf_pack with no host sync: out (device, n_send entries of
 * gsx_gxf_entry_words) gets destination d's entries from entry send_base[d]
 * (the shard plan's send segment of d) on, and d_counts (device, n_ranks x 2
 * i64) the pairs (entries for rank d, this rank's frontier size of hop - 1).
 * One all-to-all of the pairs gives every rank its entry splits and, summed,
 * whether hop - 1 left a frontier on any rank (the run is over when it did
 * not), so a forwarding hop needs one host round trip; gsx_gxf_step with
 * n_front NULL then runs the hop without a sync (keep the entries alive until
 * the stream has run it). */
int gsx_gxf_pack_dev(gsx_engine* e, uint32_t hop, uint64_t* out, int64_t* d_counts);
int gsx_gxf_end(gsx_engine* e);
int gsx_gx_got(gsx_engine* e, uint8_t* got);
int gsx_gx_end(gsx_engine* e, const uint8_t* got_all, gsx_heartbeat_out* out);
/* backoff expiry per [topic][pair] (0 = no entry), n_topics * n_pairs
 * (gs.backoff, gossipsub.go:436; zeroed by gsx_load_overlay) */
int gsx_export_backoff(gsx_engine* e, int64_t* out);
int gsx_import_backoff(gsx_engine* e, const int64_t* in);
/* The IHAVEs of the last gsx_heartbeat, per [topic][pair (sender -> target)]:
 * number of ids (0 = none sent) and a digest of the advertised ids, the sum
 * over the list of mix64(id + 0x9E3779B97F4A7C15) (mod 2^64, mix64 =
 * SplitMix64's finaliser).  The order inside an IHAVE is not reported: the
 * receiver collects the ids into a set (handleIHave, gossipsub.go:641-650).
 * Either pointer may be NULL. */
int gsx_gossip_results(gsx_engine* e, uint32_t* ihave_len, uint64_t* ihave_digest);
/* ---- topic membership (gossipsub.go:943-1083, 1517-1554) ------------------
 * By default every node has joined every topic.  gsx_set_subscriptions sets
 * the joined topics of every node (bit t of joined[node], n_nodes words) as
 * the state of the overlay, without protocol effects: gs.mesh[t] exists at a
 * node iff it joined t (only joined (node, topic) units run the mesh
 * maintenance and its gossip, and GRAFT / PRUNE / IHAVE of other topics are
 * ignored, :727-733, :816-819, :638-641), and every node knows its peers'
 * subscriptions (gs.p.topics: the "in topic" filter of getPeers, of
 * forwarding and of gossip targets).  A gossipsub publisher that has not
 * joined the topic sends to its fanout (:981-998): when empty it is filled
 * with getPeers(D) of non-direct peers with score >= PublishThreshold (draws
 * h(seed of the call, 10, source, topic << 24 | k)), and lastpub = now.  The
 * heartbeat then expires fanouts after FanoutTTL and keeps them at D
 * (:1517-1554; draws h(seed, 8, node, tick << 32 | topic << 24 | 1 << 23 | k),
 * which the node's fanout gossip continues).  gsx_join / gsx_leave change
 * membership with the protocol's effects, as one synchronous round: the
 * call's subscriptions are announced first; Join builds the mesh from the
 * fanout (negative scores dropped, topped up to D) or getPeers(D) (draws
 * h(seed, 11, node, topic << 24 | k)) and sends GRAFTs; Leave prunes the mesh
 * (tracer.Prune, PRUNE sent, no backoff at the leaver); the peers then
 * handle them as in step (B) and the joiners the PRUNE answers as in (C).
 * *out gets the round's counters (grafts / prunes of the joiners / leavers,
 * the receivers' accepted / rejected / handled, mesh_links after).  Copies
 * forwarded to a mesh peer that has left the topic (the receiver ignores
 * them, pubsub.go handleIncomingRPC) are not counted as transmissions.
 * Unsharded engines only (GSX_ESTATE on a range shard). */
int gsx_set_subscriptions(gsx_engine* e, const uint64_t* joined);
int gsx_join(gsx_engine* e, const uint32_t* nodes, const uint32_t* topics, size_t n, int64_t now_ns, uint64_t seed,
             gsx_heartbeat_out* out);
int gsx_leave(gsx_engine* e, const uint32_t* nodes, const uint32_t* topics, size_t n, int64_t now_ns,
              gsx_heartbeat_out* out);
/* joined topics per node [n_nodes], fanout topic bits per pair [E] (the
 * peer is in the owner's fanout), lastpub per [node][topic] (0 = none); any
 * pointer may be NULL */
int gsx_export_membership(gsx_engine* e, uint64_t* joined, uint64_t* fanout, int64_t* lastpub);

/* ---- peer exchange on PRUNE (gossipsub.go:811-843, 861-910, 1814-1850) -----
 * With do_px set (gsx_set_gossipsub_params; off by default, as in the
 * reference) every PRUNE of a heartbeat round (step (A), sendGraftPrune
 * :1630-1667, and the (B) answers to rejected GRAFTs, handleGraft :718-809)
 * carries a PX list unless
 *   - the pruned peer has GSX_EDGE_NO_PX (makePrune :1815-1818),
 *   - (A) pruned it for a negative score (noPX, :1361-1368; then all of the
 *     node's PRUNEs to it that round go without PX),
 *   - it is a (B) answer and the same GRAFT RPC held a GRAFT of a topic the
 *     node has not joined, from a direct peer, inside the backoff or from a
 *     negative-score peer (doPX = false, :721-781).
 * The list is getPeers(topic, PrunePeers, xp != pruned peer && score(xp) >= 0)
 * (:1822-1826; mesh-capable connected topic peers, direct ones included),
 * candidates in ascending peer order shuffled with draws h(seed, 12, node << 32
 * | pruned peer, tick << 32 | topic << 24 | kind << 23 | k) (kind 0 = (A), 1 =
 * answer) and truncated.  The receiver, if it accepts the RPC (AcceptFrom)
 * and has joined the topic, ignores the list when its score of the pruner is
 * below AcceptPXThreshold, else every listed peer it has no connection to is
 * a connection candidate (pxConnect): recorded, never dialled (the overlay
 * is fixed).  Scores: the list of an (A) PRUNE and the (B) receiver's check
 * read the scores as (A) left them (the snapshot (B) reads); an answer's
 * list and the (C) receiver's check read the scores as (B) left them (the
 * snapshot (C) reads) — the reference builds an answer's list right after
 * handling that one RPC's GRAFTs.  PX runs in gsx_heartbeat and the gsx_hb_*
 * steps of an unsharded engine (GSX_ESTATE on a range shard with do_px) and
 * in gsx_join / gsx_leave rounds: every Leave PRUNE carries PX (sendPrune,
 * :1089-1093), Join's GRAFT answers as above; their draws use tick 0 and the
 * call's seed (0 for gsx_leave), the snapshot the round's (B) reads.
 * gsx_hb_set_px_log(e, cap) keeps up to cap connection candidates of each
 * round (0, the default: counters only); gsx_hb_px_records copies those of the
 * last round as [n][4] u32 (receiver, candidate, pruner, topic | kind << 8),
 * sorted ascending, *n = the records kept (min(px_connect, log cap); which
 * ones are kept when the round had more is unspecified); up to cap rows are
 * written. */
int gsx_hb_set_px_log(gsx_engine* e, size_t cap);
/* Peer exchange on range shards: a PRUNE of a cross-shard pair carries its PX
 * list (makePrune, gossipsub.go:1814-1850) to the receiver's rank, whose
 * handlePrune reads it (:811-843, pxConnect :861-910).  kind 0 = the (A)
 * PRUNEs, between gsx_hb_begin and gsx_hb_recv; kind 1 = the (B) answers,
 * between gsx_hb_recv and gsx_hb_end.  Per kind:
 *   gsx_hb_px_count  entries this rank sends to each rank (host, n_ranks u64);
 *   gsx_hb_px_pack   writes them to `out` (device), grouped by destination in
 *                    rank order; an entry is gsx_hb_px_entry_words u32:
 *                    (receive slot at the destination, topic | kind << 8, n,
 *                    n peer ids, global) — and handles the PRUNEs whose
 *                    receiver is local;
 *   gsx_hb_px_recv   the receivers' side of the entries the other ranks sent.
 * The counters and PX records summed over ranks equal one engine's round. */
int gsx_hb_px_entry_words(gsx_engine* e, uint32_t* words);
int gsx_hb_px_count(gsx_engine* e, uint32_t kind, uint64_t* counts);
int gsx_hb_px_pack(gsx_engine* e, uint32_t kind, uint32_t* out);
int gsx_hb_px_recv(gsx_engine* e, uint32_t kind, const uint32_t* entries, uint64_t n);
int gsx_hb_px_records(gsx_engine* e, uint32_t* out, size_t cap, size_t* n);

/* The tracer's GRAFT / PRUNE calls of the last heartbeat, as topic bit words
 * per pair p = (observer -> peer), E words each (any pointer may be NULL):
 *   sent_graft    graftPeer (:1353-1359)             Graft(peer, topic) by observer
 *   sent_prune    prunePeer (:1345-1351)             Prune(peer, topic) by observer
 *   acc_graft     handleGraft accepting it (:794-796) Graft(peer, topic) by observer
 *   handled_prune handlePrune of the peer's PRUNE, (B) and the (C) answers
 *                 (:821-822)                         Prune(peer, topic) by observer
 * so popcounts give grafts + graft_accepted GRAFT and prunes + prunes_handled
 * PRUNE events.  Recorded only while gsx_hb_set_tracing(e, 1) (off by
 * default: the control words are then kept until the next round's start). */
int gsx_hb_set_tracing(gsx_engine* e, uint32_t on);
int gsx_hb_trace_words(gsx_engine* e, uint64_t* sent_graft, uint64_t* sent_prune, uint64_t* acc_graft,
                       uint64_t* handled_prune);
/* Drop every cached message window (mcache.go, a fresh cache). */
int gsx_mcache_clear(gsx_engine* e);
/* mcache.GetGossipIDs of one node (mcache.go:82-92) over its first n_windows
 * windows (HistoryGossip for the gossip view, HistoryLength for every id the
 * cache still holds, i.e. mcache.Get); topic GSX_ANY_TOPIC matches all.
 * Writes up to cap ids, *n_out = the full count. */
#define GSX_ANY_TOPIC 0xFFFFFFFFu
int gsx_mcache_ids(gsx_engine* e, uint32_t node, uint32_t topic, uint32_t n_windows, uint64_t* out, size_t cap,
                   size_t* n_out);

/* Message-parallel replicas (gsx/shard.py MessageParallel): every replica
 * holds the whole overlay and propagates one block of a gossipsub batch, so
 * its cache (mcache.go Put, gossipsub.go:943-944) holds that block only.  To
 * leave every replica's cache — and the heartbeats that read it (emitGossip,
 * the gossip exchange) — equal to one engine's that propagated the whole
 * batch, each replica takes its block's rows out of the cache and the blocks
 * go back in as one batch:
 *   gsx_mcache_last       the newest cached batch's rows: n_words per node, n_msgs;
 *   gsx_mcache_copy_last  its cache rows (after the uncache of dropped
 *                         messages) and its message set's rows (every node
 *                         that saw each message), [node][n_words] u64 each,
 *                         and n_planes planes of the set's validation codes
 *                         (each node's arrival hop of each message, bit b in
 *                         plane b, [plane][node][n_words]; zero-extended, at
 *                         least the set's; 0 planes: none copied) into caller
 *                         device buffers (engine stream order); a set
 *                         propagated with the gossip exchange off kept no
 *                         codes: n_planes must then be 0 (GSX_ESTATE);
 *   gsx_mcache_pop        drops it (the next message set reuses its serial);
 *   gsx_mcache_put        Puts msgs[0..m) of cfg's topic as one batch: block k
 *                         is messages [sum part_msgs[<k], + part_msgs[k]) with
 *                         its rows (device, [node][words(part_msgs[k])],
 *                         words() = the propagation's row width, gsx.h
 *                         gsx_propagate) at cache_parts[k] / set_parts[k], and
 *                         its code planes ([n_planes][node][words], n_planes
 *                         <= 8) at code_parts[k] (n_planes 0: every copy
 *                         validated at cfg's now_ns).
 *                         Publishing at unjoined sources (the fanout pick of
 *                         gossipsub.go:981-998, idempotent) runs for every
 *                         source of msgs, as the whole call would have.
 * Unsharded engines, gossipsub batches. */
int gsx_mcache_last(gsx_engine* e, uint32_t* n_words, uint32_t* n_msgs);
int gsx_mcache_copy_last(gsx_engine* e, uint64_t* cache_rows, uint64_t* set_rows, uint64_t* code_rows,
                         uint32_t n_planes);
int gsx_mcache_pop(gsx_engine* e);
int gsx_mcache_put(gsx_engine* e, const gsx_msg* msgs, size_t m, const gsx_prop_config* cfg, uint32_t n_parts,
                   const uint32_t* part_msgs, const uint64_t* const* cache_parts, const uint64_t* const* set_parts,
                   const uint64_t* const* code_parts, uint32_t n_planes);

/* Per-launch timing of the fused refresh+score kernel over a region: after
 * gsx_timing_begin, each of the next (up to max_launches) gsx_refresh calls
 * brackets its kernel with a pair of HIP events on the engine stream;
 * gsx_timing_end waits for them and returns the sum / min / max of the
 * per-launch durations (ms) and their count. */
int gsx_timing_begin(gsx_engine* e, uint32_t max_launches);
int gsx_timing_end(gsx_engine* e, double* total_ms, double* min_ms, double* max_ms, uint32_t* n_launches);

#ifdef __cplusplus
}
#endif
#endif /* GSX_H */
