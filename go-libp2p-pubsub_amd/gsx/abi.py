"""ctypes mirror of include/gsx.h (types and the shared-library handle).

The structures here are byte-for-byte the C structs of the boundary; the
engine itself is libgsx.so (HIP, gfx950).  Loading fails loudly when the
library is missing: there is no Python or CPU fallback for the engine.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSX_LIB") or os.path.join(HERE, "libgsx.so")  # GSX_LIB: a tuning build

GSX_OK = 0
GSX_EINVAL = -22
GSX_ENOMEM = -12
GSX_ENODEV = -19
GSX_ERANGE = -34
GSX_ESTATE = -71
GSX_EDEVICE = -5

GSX_MAX_TOPICS = 64
GSX_NO_IP = 0xFFFFFFFF

GSX_EDGE_OUTBOUND = 0x01
GSX_EDGE_DIRECT = 0x02
GSX_EDGE_GOSSIPSUB = 0x04
GSX_EDGE_FLOODSUB = 0x08
GSX_EDGE_NO_PX = 0x10

GSX_REC_IN_MESH = 0x01
GSX_REC_ACTIVE = 0x02
GSX_PAIR_PRESENT = 0x01
GSX_PAIR_CONNECTED = 0x02

# gsx_event_kind
EV_ADD_PEER = 1
EV_REMOVE_PEER = 2
EV_GRAFT = 3
EV_PRUNE = 4
EV_FIRST_DELIVERY = 5
EV_MESH_DELIVERY = 6
EV_INVALID_DELIVERY = 7
EV_PENALTY = 8
EV_APP_SCORE = 9  # arg = the float64 bits of the pair's new AppSpecificScore (score.go:320)

# gsx_reject_reason, with the reference's strings (tracer.go:28-38)
REJECT_REASONS = {
    "blacklisted peer": 0,
    "blacklisted source": 1,
    "missing signature": 2,
    "unexpected signature": 3,
    "unexpected auth info": 4,
    "invalid signature": 5,
    "validation queue full": 6,
    "validation throttled": 7,
    "validation failed": 8,
    "validation ignored": 9,
    "self originated message": 10,
}

SECOND = 1_000_000_000
MILLISECOND = 1_000_000
MINUTE = 60 * SECOND
HOUR = 60 * MINUTE


class TopicScoreParams(C.Structure):
    """TopicScoreParams, score_params.go:98-148 (durations in ns)."""

    _fields_ = [
        ("topic_weight", C.c_double),
        ("time_in_mesh_weight", C.c_double),
        ("time_in_mesh_quantum_ns", C.c_int64),
        ("time_in_mesh_cap", C.c_double),
        ("first_message_deliveries_weight", C.c_double),
        ("first_message_deliveries_decay", C.c_double),
        ("first_message_deliveries_cap", C.c_double),
        ("mesh_message_deliveries_weight", C.c_double),
        ("mesh_message_deliveries_decay", C.c_double),
        ("mesh_message_deliveries_cap", C.c_double),
        ("mesh_message_deliveries_threshold", C.c_double),
        ("mesh_message_deliveries_window_ns", C.c_int64),
        ("mesh_message_deliveries_activation_ns", C.c_int64),
        ("mesh_failure_penalty_weight", C.c_double),
        ("mesh_failure_penalty_decay", C.c_double),
        ("invalid_message_deliveries_weight", C.c_double),
        ("invalid_message_deliveries_decay", C.c_double),
    ]


class PeerScoreParams(C.Structure):
    """PeerScoreParams, score_params.go:53-96 minus Topics/closure/whitelist."""

    _fields_ = [
        ("topic_score_cap", C.c_double),
        ("app_specific_weight", C.c_double),
        ("app_specific_score_set", C.c_int32),
        ("ip_colocation_factor_threshold", C.c_int32),
        ("ip_colocation_factor_weight", C.c_double),
        ("behaviour_penalty_weight", C.c_double),
        ("behaviour_penalty_threshold", C.c_double),
        ("behaviour_penalty_decay", C.c_double),
        ("decay_interval_ns", C.c_int64),
        ("decay_to_zero", C.c_double),
        ("retain_score_ns", C.c_int64),
    ]


class Thresholds(C.Structure):
    """PeerScoreThresholds, score_params.go:12-32."""

    _fields_ = [
        ("gossip_threshold", C.c_double),
        ("publish_threshold", C.c_double),
        ("graylist_threshold", C.c_double),
        ("accept_px_threshold", C.c_double),
        ("opportunistic_graft_threshold", C.c_double),
    ]


class Config(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("device", C.c_int32), ("reserved", C.c_uint32 * 6)]


class Event(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32),
        ("topic", C.c_uint32),
        ("pair", C.c_uint64),
        ("now_ns", C.c_int64),
        ("arg", C.c_int64),
    ]


EVENT_DTYPE = None  # numpy dtype matching Event, built lazily


def event_dtype():
    global EVENT_DTYPE
    if EVENT_DTYPE is None:
        import numpy as np

        EVENT_DTYPE = np.dtype(
            [("kind", "<u4"), ("topic", "<u4"), ("pair", "<u8"), ("now_ns", "<i8"), ("arg", "<i8")], align=True
        )
        assert EVENT_DTYPE.itemsize == C.sizeof(Event)
    return EVENT_DTYPE


class StateView(C.Structure):
    _fields_ = [
        ("first_message_deliveries", C.POINTER(C.c_double)),
        ("mesh_message_deliveries", C.POINTER(C.c_double)),
        ("mesh_failure_penalty", C.POINTER(C.c_double)),
        ("invalid_message_deliveries", C.POINTER(C.c_double)),
        ("graft_time_ns", C.POINTER(C.c_int64)),
        ("mesh_time_ns", C.POINTER(C.c_int64)),
        ("rec_flags", C.POINTER(C.c_uint8)),
        ("pair_flags", C.POINTER(C.c_uint8)),
        ("expire_ns", C.POINTER(C.c_int64)),
        ("behaviour_penalty", C.POINTER(C.c_double)),
        ("last_refresh_ns", C.c_int64),
    ]


STATE_FIELDS = [f for f, _ in StateView._fields_][:-1]  # the array members
RECORD_FIELDS = STATE_FIELDS[:7]
PAIR_FIELDS = STATE_FIELDS[7:]
STATE_DTYPES = {
    "first_message_deliveries": "<f8",
    "mesh_message_deliveries": "<f8",
    "mesh_failure_penalty": "<f8",
    "invalid_message_deliveries": "<f8",
    "graft_time_ns": "<i8",
    "mesh_time_ns": "<i8",
    "rec_flags": "u1",
    "pair_flags": "u1",
    "expire_ns": "<i8",
    "behaviour_penalty": "<f8",
}

class ScoreSnapshot(C.Structure):
    """gsx_score_snapshot: PeerScoreSnapshot / TopicScoreSnapshot (score.go:125-138)."""
    _fields_ = [
        ("present", C.POINTER(C.c_uint8)),
        ("score", C.POINTER(C.c_double)),
        ("app_specific_score", C.POINTER(C.c_double)),
        ("ip_colocation_factor", C.POINTER(C.c_double)),
        ("behaviour_penalty", C.POINTER(C.c_double)),
        ("time_in_mesh_ns", C.POINTER(C.c_int64)),
        ("first_message_deliveries", C.POINTER(C.c_double)),
        ("mesh_message_deliveries", C.POINTER(C.c_double)),
        ("invalid_message_deliveries", C.POINTER(C.c_double)),
    ]


SNAPSHOT_PAIR = {"present": "u1", "score": "<f8", "app_specific_score": "<f8", "ip_colocation_factor": "<f8",
                 "behaviour_penalty": "<f8"}
SNAPSHOT_RECORD = {"time_in_mesh_ns": "<i8", "first_message_deliveries": "<f8", "mesh_message_deliveries": "<f8",
                   "invalid_message_deliveries": "<f8"}


class SynthSpec(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("now_ns", C.c_int64),
        ("fmd_max", C.c_double),
        ("mmd_max", C.c_double),
        ("mfp_max", C.c_double),
        ("imd_max_sybil", C.c_double),
        ("p_in_mesh", C.c_double),
        ("graft_window_ns", C.c_int64),
        ("bp_max", C.c_double),
        ("p_disconnected", C.c_double),
        ("p_absent", C.c_double),
        ("expire_jitter_ns", C.c_int64),
        ("sybil_first_node", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


GSX_ROUTER_FLOODSUB = 0
GSX_ROUTER_GOSSIPSUB = 1
GSX_ROUTER_RANDOMSUB = 2
GSX_MAX_HOPS = 64
GXF_MAX_HOPS = 4096  # hops of one forwarding run of the gossip exchange (gsx_device.h)
GSX_CREDIT_OFF = 0
GSX_CREDIT_NOW = 1
GSX_CREDIT_DEFER = 2
GSX_ANY_TOPIC = 0xFFFFFFFF


GSX_VALIDATION_ACCEPT, GSX_VALIDATION_REJECT, GSX_VALIDATION_IGNORE, GSX_VALIDATION_THROTTLE = 0, 1, 2, 3


def prop_words(m: int) -> int:
    """Words per call (gsx.h): 1, 2, or ceil(m/64) rounded up to a multiple of 4."""
    w = (m + 63) // 64
    if w <= 2:
        return max(w, 1)
    return (w + 3) & ~3


class PropConfig(C.Structure):
    _fields_ = [
        ("router", C.c_uint32),
        ("topic", C.c_uint32),
        ("flood_publish", C.c_uint32),
        ("max_hops", C.c_uint32),
        ("hop_latency_ns", C.c_int64),
        ("now_ns", C.c_int64),
        ("credit_scores", C.c_uint32),
        ("randomsub_size", C.c_uint32),
        ("seed", C.c_uint64),
        ("validation_delay_ns", C.c_int64),
    ]


class PropOut(C.Structure):
    _fields_ = [
        ("deliveries", C.c_uint64),
        ("duplicates", C.c_uint64),
        ("transmissions", C.c_uint64),
        ("hops", C.c_uint32),
        ("hop_launches", C.c_uint32),
        ("hop_deliveries", C.c_uint64 * (GSX_MAX_HOPS + 1)),
        ("edge_sends", C.c_uint64),
        ("new_words", C.c_uint64),
        ("hop_kernel_ms", C.c_double),
        ("rejected", C.c_uint64),
        ("ignored", C.c_uint64),
        ("graylisted", C.c_uint64),
    ]

    def as_dict(self):
        return dict(deliveries=self.deliveries, duplicates=self.duplicates, transmissions=self.transmissions,
                    hops=self.hops, hop_deliveries=list(self.hop_deliveries)[: self.hops + 1],
                    rejected=self.rejected, ignored=self.ignored, graylisted=self.graylisted)


class Msg(C.Structure):
    _fields_ = [("source", C.c_uint32), ("validation", C.c_uint32), ("msg_id", C.c_uint64)]


_MSG_DTYPE = None


def msg_dtype():
    global _MSG_DTYPE
    if _MSG_DTYPE is None:
        import numpy as np

        _MSG_DTYPE = np.dtype([("source", "<u4"), ("validation", "<u4"), ("msg_id", "<u8")], align=True)
        assert _MSG_DTYPE.itemsize == C.sizeof(Msg)
    return _MSG_DTYPE


class GossipSubParams(C.Structure):
    _fields_ = [
        ("d", C.c_int32),
        ("d_lo", C.c_int32),
        ("d_hi", C.c_int32),
        ("d_score", C.c_int32),
        ("d_out", C.c_int32),
        ("opportunistic_graft_peers", C.c_int32),
        ("opportunistic_graft_ticks", C.c_uint64),
        ("prune_backoff_ns", C.c_int64),
        ("graft_flood_threshold_ns", C.c_int64),
        ("d_lazy", C.c_int32),
        ("history_length", C.c_int32),
        ("history_gossip", C.c_int32),
        ("max_ihave_length", C.c_int32),
        ("gossip_factor", C.c_double),
        ("max_ihave_messages", C.c_int32),
        ("gossip_retransmission", C.c_int32),
        ("iwant_followup_ns", C.c_int64),
        ("gossip_exchange", C.c_int32),
        ("reserved0", C.c_int32),
        ("fanout_ttl_ns", C.c_int64),
        ("do_px", C.c_int32),
        ("prune_peers", C.c_int32),
    ]


class HeartbeatOut(C.Structure):
    _fields_ = [
        ("grafts", C.c_uint64),
        ("prunes", C.c_uint64),
        ("graft_accepted", C.c_uint64),
        ("graft_rejected", C.c_uint64),
        ("prunes_handled", C.c_uint64),
        ("penalties", C.c_uint64),
        ("backoff_cleared", C.c_uint64),
        ("mesh_links", C.c_uint64),
        ("ihave_msgs", C.c_uint64),
        ("ihave_ids", C.c_uint64),
        ("broken_promises", C.c_uint64),
        ("ihave_ignored", C.c_uint64),
        ("iwant_msgs", C.c_uint64),
        ("iwant_ids", C.c_uint64),
        ("iwant_served", C.c_uint64),
        ("gossip_delivered", C.c_uint64),
        ("gossip_rejected", C.c_uint64),
        ("gossip_duplicates", C.c_uint64),
        ("px_prunes", C.c_uint64),
        ("px_peers", C.c_uint64),
        ("px_ignored", C.c_uint64),
        ("px_connect", C.c_uint64),
        ("fwd_delivered", C.c_uint64),
        ("fwd_duplicates", C.c_uint64),
        ("fwd_graylisted", C.c_uint64),
    ]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


P = C.POINTER
_u64p = P(C.c_uint64)

# Every entry point of include/gsx.h: name -> (restype, argtypes)
SIGNATURES = {
    "gsx_abi_version": (C.c_int, []),
    "gsx_validate_peer_params": (C.c_int, [P(PeerScoreParams)]),
    "gsx_validate_topic_params": (C.c_int, [P(TopicScoreParams)]),
    "gsx_validate_thresholds": (C.c_int, [P(Thresholds)]),
    "gsx_score_parameter_decay_with_base": (C.c_double, [C.c_int64, C.c_int64, C.c_double]),
    "gsx_score_parameter_decay": (C.c_double, [C.c_int64]),
    "gsx_create": (C.c_int, [P(Config), P(C.c_void_p)]),
    "gsx_destroy": (C.c_int, [C.c_void_p]),
    "gsx_last_error": (C.c_char_p, [C.c_void_p]),
    "gsx_set_peer_params": (C.c_int, [C.c_void_p, P(PeerScoreParams)]),
    "gsx_set_thresholds": (C.c_int, [C.c_void_p, P(Thresholds)]),
    "gsx_set_topic_params": (C.c_int, [C.c_void_p, C.c_uint32, P(TopicScoreParams)]),
    "gsx_load_overlay": (
        C.c_int,
        [C.c_void_p, C.c_uint32, P(C.c_int64), P(C.c_int32), P(C.c_uint8), P(C.c_uint32)],
    ),
    "gsx_num_pairs": (C.c_int, [C.c_void_p, _u64p]),
    "gsx_set_ip_whitelist": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_size_t]),
    "gsx_set_app_scores": (C.c_int, [C.c_void_p, P(C.c_double), C.c_size_t]),
    "gsx_apply_events": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "gsx_flush": (C.c_int, [C.c_void_p]),
    "gsx_trace_validate": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_int64]),
    "gsx_trace_deliver": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_int64]),
    "gsx_trace_reject": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_int32, C.c_int64]),
    "gsx_trace_duplicate": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_int64]),
    "gsx_gc_deliveries": (C.c_int, [C.c_void_p, C.c_int64]),
    "gsx_num_delivery_records": (C.c_int, [C.c_void_p, _u64p]),
    "gsx_refresh": (C.c_int, [C.c_void_p, C.c_int64]),
    "gsx_scores": (C.c_int, [C.c_void_p, P(C.c_double), C.c_size_t]),
    "gsx_score": (C.c_int, [C.c_void_p, C.c_uint64, P(C.c_double)]),
    "gsx_score_many": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_size_t, P(C.c_double)]),
    "gsx_gx_pending": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "gsx_gx_common": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "gsx_gx_set_common": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "gsx_gx_pack_ihave": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_gx_recv_ihave": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_gx_rows_words": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "gsx_gx_rows_pack": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_void_p]),
    "gsx_gx_rows_recv": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "gsx_gx_exchange": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "gsx_gxf_begin": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gsx_gxf_entry_words": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "gsx_gxf_pack_fout": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_gxf_recv_fout": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_gxf_pack": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_uint64), C.c_void_p]),
    "gsx_gxf_step": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, P(C.c_uint64)]),
    "gsx_gxf_pack_dev": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    "gsx_gxf_end": (C.c_int, [C.c_void_p]),
    "gsx_gx_got": (C.c_int, [C.c_void_p, P(C.c_uint8)]),
    "gsx_gx_end": (C.c_int, [C.c_void_p, P(C.c_uint8), P(HeartbeatOut)]),
    "gsx_device_scores": (C.c_int, [C.c_void_p, P(C.c_void_p)]),
    "gsx_sync": (C.c_int, [C.c_void_p]),
    "gsx_settle_scores": (C.c_int, [C.c_void_p]),
    "gsx_import_state": (C.c_int, [C.c_void_p, P(StateView)]),
    "gsx_export_state": (C.c_int, [C.c_void_p, P(StateView)]),
    "gsx_last_refresh_ms": (C.c_int, [C.c_void_p, P(C.c_float)]),
    "gsx_synthesize_state": (C.c_int, [C.c_void_p, P(SynthSpec)]),
    "gsx_propagate": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, P(PropConfig), P(PropOut)]),
    "gsx_prop_results": (C.c_int, [C.c_void_p, P(C.c_uint8), P(C.c_int32)]),
    "gsx_prop_set_tracking": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gsx_prop_duplicates": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_size_t]),
    "gsx_set_pair_ips": (C.c_int, [C.c_void_p, P(C.c_uint64), P(C.c_uint32), C.c_size_t]),
    "gsx_peer_score_snapshot": (C.c_int, [C.c_void_p, P(ScoreSnapshot)]),
    "gsx_prop_pending_invalid": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_prop_replace_pending_invalid": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_prop_pending_credits": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "gsx_prop_fold_credits": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "gsx_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_load_overlay_shard": (
        C.c_int,
        [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_int64), P(C.c_int32), P(C.c_uint8), P(C.c_uint32)],
    ),
    "gsx_shard_recv_plan": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_uint32), _u64p, P(C.c_uint32), P(C.c_uint32)]),
    "gsx_shard_send_plan": (C.c_int, [C.c_void_p, _u64p, P(C.c_uint32), P(C.c_uint32)]),
    "gsx_shard_counts": (C.c_int, [C.c_void_p, _u64p, _u64p]),
    "gsx_shard_set_halo_bases": (C.c_int, [C.c_void_p, _u64p]),
    "gsx_prop_pack_compact": (C.c_int, [C.c_void_p, C.c_void_p, _u64p]),
    "gsx_prop_step_compact": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, _u64p]),
    "gsx_prop_pack_compact_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "gsx_prop_hop_counts_dev": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_prop_set_last_hop": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gsx_prop_rep": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "gsx_prop_rep_fwd_pack": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_prop_rep_fwd_recv": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_prop_rep_pack_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "gsx_prop_rep_step": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_void_p), P(C.c_uint64)]),
    "gsx_prop_rep_sends_pack": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_prop_rep_rows": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gsx_prop_rep_rows_export": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "gsx_prop_rep_rows_step": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_void_p), C.c_void_p]),
    "gsx_prop_rep_sends_recv": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_hb_set_px_log": (C.c_int, [C.c_void_p, C.c_size_t]),
    "gsx_hb_px_records": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_size_t, P(C.c_size_t)]),
    "gsx_prop_begin": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, P(PropConfig)]),
    "gsx_prop_pack": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_prop_step": (C.c_int, [C.c_void_p, C.c_void_p, _u64p]),
    "gsx_prop_end": (C.c_int, [C.c_void_p, P(PropOut)]),
    "gsx_default_gossipsub_params": (C.c_int, [P(GossipSubParams)]),
    "gsx_set_gossipsub_params": (C.c_int, [C.c_void_p, P(GossipSubParams)]),
    "gsx_heartbeat": (C.c_int, [C.c_void_p, C.c_uint64, C.c_int64, C.c_uint64, P(HeartbeatOut)]),
    "gsx_hb_reserve": (C.c_int, [C.c_void_p]),
    "gsx_hb_begin": (C.c_int, [C.c_void_p, C.c_uint64, C.c_int64, C.c_uint64]),
    "gsx_hb_pack_ctl": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_hb_recv": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_hb_pack_resp": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gsx_hb_end": (C.c_int, [C.c_void_p, C.c_void_p, P(HeartbeatOut)]),
    "gsx_export_backoff": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "gsx_import_backoff": (C.c_int, [C.c_void_p, P(C.c_int64)]),
    "gsx_gossip_results": (C.c_int, [C.c_void_p, P(C.c_uint32), P(C.c_uint64)]),
    "gsx_mcache_clear": (C.c_int, [C.c_void_p]),
    "gsx_hb_px_entry_words": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "gsx_hb_px_count": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_uint64)]),
    "gsx_hb_px_pack": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "gsx_hb_px_recv": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]),
    "gsx_mcache_last": (C.c_int, [C.c_void_p, P(C.c_uint32), P(C.c_uint32)]),
    "gsx_mcache_copy_last": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    "gsx_mcache_pop": (C.c_int, [C.c_void_p]),
    "gsx_mcache_put": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, P(PropConfig), C.c_uint32, P(C.c_uint32),
                                 P(C.c_void_p), P(C.c_void_p), P(C.c_void_p), C.c_uint32]),
    "gsx_hb_set_tracing": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gsx_set_subscriptions": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "gsx_join": (C.c_int, [C.c_void_p, P(C.c_uint32), P(C.c_uint32), C.c_size_t, C.c_int64, C.c_uint64,
                           P(HeartbeatOut)]),
    "gsx_leave": (C.c_int, [C.c_void_p, P(C.c_uint32), P(C.c_uint32), C.c_size_t, C.c_int64, P(HeartbeatOut)]),
    "gsx_export_membership": (C.c_int, [C.c_void_p, P(C.c_uint64), P(C.c_uint64), P(C.c_int64)]),
    "gsx_hb_trace_words": (C.c_int, [C.c_void_p, P(C.c_uint64), P(C.c_uint64), P(C.c_uint64), P(C.c_uint64)]),
    "gsx_promise_add": (C.c_int, [C.c_void_p, C.c_uint64, P(C.c_uint64), C.c_uint32, C.c_int64, C.c_uint64]),
    "gsx_promise_broken": (C.c_int, [C.c_void_p, C.c_int64, P(C.c_uint32), P(C.c_uint64)]),
    "gsx_promise_fulfill": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64]),
    "gsx_promise_throttle": (C.c_int, [C.c_void_p, C.c_uint64]),
    "gsx_promise_count": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "gsx_mcache_ids": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_uint64), C.c_size_t,
                                 P(C.c_size_t)]),
    "gsx_timing_begin": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gsx_timing_end": (
        C.c_int,
        [C.c_void_p, P(C.c_double), P(C.c_double), P(C.c_double), P(C.c_uint32)],
    ),
}

_lib = None


def load_library(path: str = LIB_PATH):
    """Load libgsx.so (built by `make -C go-libp2p-pubsub_amd`).  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: build it with `make -C go-libp2p-pubsub_amd` "
            "(the engine has no CPU fallback)"
        )
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class GsxError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with {code}")
        self.code = code
