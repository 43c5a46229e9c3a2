"""Python handle on the HIP engine (libgsx.so) through the C ABI of include/gsx.h.

This is plumbing for tests and bench.py: every call goes straight to the
C ABI; nothing here computes scores.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Iterable, Optional

import numpy as np

from . import abi
from .abi import GsxError, prop_words


def _ptr(a: Optional[np.ndarray], ctype):
    if a is None:
        return C.cast(None, C.POINTER(ctype))
    return a.ctypes.data_as(C.POINTER(ctype))


_CTYPES = {"<f8": C.c_double, "<i8": C.c_int64, "u1": C.c_uint8}


def default_gossipsub_params(**kw) -> abi.GossipSubParams:
    """DefaultGossipSubParams (gossipsub.go:230-260, gsx_default_gossipsub_params) with overrides."""
    gp = abi.GossipSubParams()
    rc = abi.load_library().gsx_default_gossipsub_params(C.byref(gp))
    if rc != 0:
        raise RuntimeError(f"gsx_default_gossipsub_params -> {rc}")
    for k, v in kw.items():
        setattr(gp, k, v)
    return gp


def make_struct(cls, **kw):
    s = cls()
    for k, v in kw.items():
        if not hasattr(s, k):
            raise AttributeError(f"{cls.__name__} has no field {k}")
        setattr(s, k, v)
    return s


class Engine:
    def __init__(self, n_topics: int, device: int = 0):
        self.lib = abi.load_library()
        cfg = abi.Config(n_topics=n_topics, device=device)
        h = C.c_void_p()
        rc = self.lib.gsx_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise GsxError(rc, "gsx_create (needs a gfx950 GPU)")
        self.h = h
        self.n_topics = n_topics
        self.n_pairs = 0

    # -- helpers ---------------------------------------------------------------
    def _chk(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.gsx_last_error(self.h)
            raise GsxError(rc, f"{what}: {msg.decode() if msg else ''}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.gsx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- params ------------------------------------------------------------------
    def set_peer_params(self, p: abi.PeerScoreParams):
        self._chk(self.lib.gsx_set_peer_params(self.h, C.byref(p)), "gsx_set_peer_params")

    def set_thresholds(self, t: abi.Thresholds):
        self._chk(self.lib.gsx_set_thresholds(self.h, C.byref(t)), "gsx_set_thresholds")

    def set_topic_params(self, topic: int, p: abi.TopicScoreParams):
        self._chk(self.lib.gsx_set_topic_params(self.h, topic, C.byref(p)), "gsx_set_topic_params")

    # -- overlay -------------------------------------------------------------------
    def load_overlay(self, row_ptr, col, edge_flags=None, node_ips=None):
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        n = len(row_ptr) - 1
        ef = None if edge_flags is None else np.ascontiguousarray(edge_flags, dtype=np.uint8)
        ips = None if node_ips is None else np.ascontiguousarray(node_ips, dtype=np.uint32).reshape(-1)
        self._chk(
            self.lib.gsx_load_overlay(
                self.h, n, _ptr(row_ptr, C.c_int64), _ptr(col, C.c_int32), _ptr(ef, C.c_uint8), _ptr(ips, C.c_uint32)
            ),
            "gsx_load_overlay",
        )
        v = C.c_uint64()
        self._chk(self.lib.gsx_num_pairs(self.h, C.byref(v)), "gsx_num_pairs")
        self.n_pairs = int(v.value)
        self.n_nodes = n

    def set_ip_whitelist(self, ips: Iterable[int]):
        a = np.ascontiguousarray(list(ips), dtype=np.uint32)
        self._chk(self.lib.gsx_set_ip_whitelist(self.h, _ptr(a, C.c_uint32), len(a)), "gsx_set_ip_whitelist")

    def set_app_scores(self, app):
        a = np.ascontiguousarray(app, dtype=np.float64)
        self._chk(self.lib.gsx_set_app_scores(self.h, _ptr(a, C.c_double), len(a)), "gsx_set_app_scores")

    # -- events ------------------------------------------------------------------
    def apply_events(self, events):
        ev = np.ascontiguousarray(events, dtype=abi.event_dtype())
        self._chk(self.lib.gsx_apply_events(self.h, ev.ctypes.data_as(C.c_void_p), len(ev)), "gsx_apply_events")

    def flush(self):
        self._chk(self.lib.gsx_flush(self.h), "gsx_flush")

    def trace_validate(self, pair, msg, topic, now):
        self._chk(self.lib.gsx_trace_validate(self.h, pair, msg, topic, now), "gsx_trace_validate")

    def trace_deliver(self, pair, msg, topic, now):
        self._chk(self.lib.gsx_trace_deliver(self.h, pair, msg, topic, now), "gsx_trace_deliver")

    def trace_reject(self, pair, msg, topic, reason, now):
        if isinstance(reason, str):
            reason = abi.REJECT_REASONS[reason]
        self._chk(self.lib.gsx_trace_reject(self.h, pair, msg, topic, reason, now), "gsx_trace_reject")

    def trace_duplicate(self, pair, msg, topic, now):
        self._chk(self.lib.gsx_trace_duplicate(self.h, pair, msg, topic, now), "gsx_trace_duplicate")

    def gc_deliveries(self, now):
        self._chk(self.lib.gsx_gc_deliveries(self.h, now), "gsx_gc_deliveries")

    def num_delivery_records(self) -> int:
        v = C.c_uint64()
        self._chk(self.lib.gsx_num_delivery_records(self.h, C.byref(v)), "gsx_num_delivery_records")
        return int(v.value)

    # -- refresh / score ---------------------------------------------------------------
    def refresh(self, now: int):
        self._chk(self.lib.gsx_refresh(self.h, now), "gsx_refresh")

    def scores(self) -> np.ndarray:
        out = np.empty(self.n_pairs, dtype=np.float64)
        self._chk(self.lib.gsx_scores(self.h, _ptr(out, C.c_double), self.n_pairs), "gsx_scores")
        return out

    def set_pair_ips(self, pairs, ips):
        """gsx_set_pair_ips: setIPs for these pairs (ips: [n, 2] u32, GSX_NO_IP for none)."""
        pairs = np.ascontiguousarray(pairs, dtype=np.uint64).reshape(-1)
        ips = np.ascontiguousarray(ips, dtype=np.uint32).reshape(-1, 2)
        if len(ips) != len(pairs):
            raise ValueError("one IP pair per pair")
        self._chk(self.lib.gsx_set_pair_ips(self.h, _ptr(pairs, C.c_uint64), _ptr(ips, C.c_uint32), len(pairs)),
                  "gsx_set_pair_ips")

    def score(self, pair: int) -> float:
        v = C.c_double()
        self._chk(self.lib.gsx_score(self.h, pair, C.byref(v)), "gsx_score")
        return float(v.value)

    def score_many(self, pairs) -> np.ndarray:
        """Score(p) of many pairs with one flush / re-score / copy (gsx_score_many)."""
        pairs = np.ascontiguousarray(pairs, dtype=np.uint64)
        out = np.empty(len(pairs), dtype=np.float64)
        self._chk(self.lib.gsx_score_many(self.h, _ptr(pairs, C.c_uint64), len(pairs), _ptr(out, C.c_double)),
                  "gsx_score_many")
        return out

    def device_scores_ptr(self) -> int:
        v = C.c_void_p()
        self._chk(self.lib.gsx_device_scores(self.h, C.byref(v)), "gsx_device_scores")
        return int(v.value or 0)

    def sync(self):
        self._chk(self.lib.gsx_sync(self.h), "gsx_sync")

    def settle_scores(self):
        """gsx_settle_scores: the deferred re-scores of lazy credit folds, queued now."""
        self._chk(self.lib.gsx_settle_scores(self.h), "gsx_settle_scores")

    def last_refresh_ms(self) -> float:
        v = C.c_float()
        self._chk(self.lib.gsx_last_refresh_ms(self.h, C.byref(v)), "gsx_last_refresh_ms")
        return float(v.value)

    def propagate(self, msgs, cfg: abi.PropConfig, want_results: bool = False):
        """-> (PropOut, hop [m, n] or None, first_from [m, n] or None)"""
        ms = np.ascontiguousarray(msgs, dtype=abi.msg_dtype())
        out = abi.PropOut()
        self._chk(
            self.lib.gsx_propagate(self.h, ms.ctypes.data_as(C.c_void_p), len(ms), C.byref(cfg), C.byref(out)),
            "gsx_propagate",
        )
        hop = frm = None
        if want_results:
            n = self.n_nodes
            hop = np.empty((len(ms), n), dtype=np.uint8)
            frm = np.empty((len(ms), n), dtype=np.int32) if self._track else None
            self._chk(self.lib.gsx_prop_results(self.h, _ptr(hop, C.c_uint8), _ptr(frm, C.c_int32)), "gsx_prop_results")
        return out, hop, frm

    _track = True

    def prop_duplicates(self, n_msgs: int) -> np.ndarray:
        """gsx_prop_duplicates: [n_pairs, ceil(m / 64)] u64, bit m of row q = the
        pair's neighbour sent its observer a copy of message m it had already seen."""
        W = (n_msgs + 63) // 64
        rows = np.zeros((self.n_pairs, W), dtype=np.uint64)
        self._chk(self.lib.gsx_prop_duplicates(self.h, _ptr(rows, C.c_uint64), W), "gsx_prop_duplicates")
        return rows

    def set_prop_tracking(self, first_deliverers: bool):
        """gsx_prop_set_tracking: keep first-deliverer rows (results' first_from) or only counts."""
        self._chk(self.lib.gsx_prop_set_tracking(self.h, 1 if first_deliverers else 0), "gsx_prop_set_tracking")
        self._track = bool(first_deliverers)

    # -- stepped / sharded propagation (gsx.h "range sharding") --------------------------
    def load_overlay_shard(self, n_total, node_lo, row_ptr, col, edge_flags=None, node_ips=None):
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        n = len(row_ptr) - 1
        ef = None if edge_flags is None else np.ascontiguousarray(edge_flags, dtype=np.uint8)
        ips = None if node_ips is None else np.ascontiguousarray(node_ips, dtype=np.uint32).reshape(-1)
        self._chk(
            self.lib.gsx_load_overlay_shard(self.h, n_total, node_lo, n, _ptr(row_ptr, C.c_int64),
                                            _ptr(col, C.c_int32), _ptr(ef, C.c_uint8), _ptr(ips, C.c_uint32)),
            "gsx_load_overlay_shard",
        )
        v = C.c_uint64()
        self._chk(self.lib.gsx_num_pairs(self.h, C.byref(v)), "gsx_num_pairs")
        self.n_pairs = int(v.value)
        self.n_nodes = n
        self.node_lo = node_lo
        self.n_total = n_total

    def shard_recv_plan(self, rank_lo):
        """-> (recv_counts [world] u64, recv_u, recv_v): this rank's receive list."""
        rl = np.ascontiguousarray(rank_lo, dtype=np.uint32)
        self._rank_lo = rl
        w = len(rl) - 1
        cnt = np.zeros(w, dtype=np.uint64)
        self._chk(self.lib.gsx_shard_recv_plan(self.h, w, _ptr(rl, C.c_uint32), _ptr(cnt, C.c_uint64), None, None),
                  "gsx_shard_recv_plan")
        n = int(cnt.sum())
        ru = np.empty(n, dtype=np.uint32)
        rv = np.empty(n, dtype=np.uint32)
        self._chk(self.lib.gsx_shard_recv_plan(self.h, w, _ptr(rl, C.c_uint32), _ptr(cnt, C.c_uint64),
                                               _ptr(ru, C.c_uint32), _ptr(rv, C.c_uint32)), "gsx_shard_recv_plan")
        return cnt, ru, rv

    def shard_send_plan(self, send_counts, req_u, req_v):
        sc = np.ascontiguousarray(send_counts, dtype=np.uint64)
        u = np.ascontiguousarray(req_u, dtype=np.uint32)
        v = np.ascontiguousarray(req_v, dtype=np.uint32)
        self._chk(self.lib.gsx_shard_send_plan(self.h, _ptr(sc, C.c_uint64), _ptr(u, C.c_uint32),
                                               _ptr(v, C.c_uint32)), "gsx_shard_send_plan")

    def shard_set_halo_bases(self, dest_halo_base):
        b = np.ascontiguousarray(dest_halo_base, dtype=np.uint64)
        self._chk(self.lib.gsx_shard_set_halo_bases(self.h, _ptr(b, C.c_uint64)), "gsx_shard_set_halo_bases")

    def prop_pack_compact(self, out) -> np.ndarray:
        """out: device buffer [n_send][words + 1] u64; -> entries per destination rank."""
        p = out.data_ptr() if hasattr(out, "data_ptr") else out
        w = len(self._rank_lo) - 1
        cnt = np.zeros(w, dtype=np.uint64)
        self._chk(self.lib.gsx_prop_pack_compact(self.h, C.c_void_p(p or None), _ptr(cnt, C.c_uint64)),
                  "gsx_prop_pack_compact")
        return cnt

    def prop_pack_compact_dev(self, out, counts):
        """As prop_pack_compact, the counts left on the device: counts (device
        tensor [n_ranks, 2] i64) = (entries for rank k, this rank's first
        receipts of the hop just run); no host sync."""
        p = out.data_ptr() if hasattr(out, "data_ptr") else out
        self._chk(self.lib.gsx_prop_pack_compact_dev(self.h, C.c_void_p(p or None), C.c_void_p(counts.data_ptr())),
                  "gsx_prop_pack_compact_dev")

    def prop_step_compact(self, entries, n: int, sync: bool = True):
        """-> this hop's first receipts on this rank; sync=False: no host sync, -> None."""
        p = entries.data_ptr() if hasattr(entries, "data_ptr") else entries
        v = C.c_uint64()
        self._chk(self.lib.gsx_prop_step_compact(self.h, C.c_void_p(p or None), n, C.byref(v) if sync else None),
                  "gsx_prop_step_compact")
        return int(v.value) if sync else None

    def shard_counts(self):
        a, b = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.gsx_shard_counts(self.h, C.byref(a), C.byref(b)), "gsx_shard_counts")
        return int(a.value), int(b.value)

    def set_stream(self, stream_handle: int):
        """Order the engine's work on a HIP stream (e.g. torch.cuda.current_stream().cuda_stream); 0 = own."""
        self._chk(self.lib.gsx_set_stream(self.h, C.c_void_p(stream_handle or None)), "gsx_set_stream")

    def prop_begin(self, msgs, cfg: abi.PropConfig):
        ms = np.ascontiguousarray(msgs, dtype=abi.msg_dtype())
        self._chk(self.lib.gsx_prop_begin(self.h, ms.ctypes.data_as(C.c_void_p), len(ms), C.byref(cfg)),
                  "gsx_prop_begin")
        self._prop_msgs = len(ms)

    def prop_pack(self, send):
        """send: device buffer (torch tensor or pointer) of [n_send][words] u64 rows."""
        p = send.data_ptr() if hasattr(send, "data_ptr") else send
        self._chk(self.lib.gsx_prop_pack(self.h, C.c_void_p(p or None)), "gsx_prop_pack")

    def prop_step(self, recv, sync: bool = True):
        """recv: device buffer (torch tensor or pointer) of the received rows; -> this hop's first
        receipts (sync=False: no host sync, -> None)."""
        p = recv.data_ptr() if hasattr(recv, "data_ptr") else recv
        n = C.c_uint64()
        self._chk(self.lib.gsx_prop_step(self.h, C.c_void_p(p or None), C.byref(n) if sync else None),
                  "gsx_prop_step")
        return int(n.value) if sync else None

    def prop_hop_counts_dev(self, out):
        """out: device int64 buffer of GSX_MAX_HOPS + 1: the call's first receipts per hop (no host sync)."""
        p = out.data_ptr() if hasattr(out, "data_ptr") else out
        self._chk(self.lib.gsx_prop_hop_counts_dev(self.h, C.c_void_p(p)), "gsx_prop_hop_counts_dev")

    # -- range shards, replicated frontier (gsx.h gsx_prop_rep_*) --
    def prop_rep(self) -> bool:
        v = C.c_uint32()
        self._chk(self.lib.gsx_prop_rep(self.h, C.byref(v)), "gsx_prop_rep")
        return bool(v.value)

    def prop_rep_fwd_pack(self, out):
        self._chk(self.lib.gsx_prop_rep_fwd_pack(self.h, self._p(out)), "gsx_prop_rep_fwd_pack")

    def prop_rep_fwd_recv(self, inp):
        self._chk(self.lib.gsx_prop_rep_fwd_recv(self.h, self._p(inp)), "gsx_prop_rep_fwd_recv")

    def prop_rep_pack_dev(self, out, d_counts):
        """This rank's frontier rows of the hop just run as entries into out; (entries, receipts) into d_counts."""
        self._chk(self.lib.gsx_prop_rep_pack_dev(self.h, self._p(out), self._p(d_counts)), "gsx_prop_rep_pack_dev")

    def prop_rep_step(self, parts=(), counts=()):
        """The other ranks' entries (device tensors, counts[k] rows each), then the next hop."""
        n = len(parts)
        pp = (C.c_void_p * max(n, 1))(*[self._p(t).value for t in parts])
        cc = (C.c_uint64 * max(n, 1))(*[int(c) for c in counts])
        self._chk(self.lib.gsx_prop_rep_step(self.h, n, pp, cc), "gsx_prop_rep_step")

    def prop_rep_rows(self, on: bool = True):
        """This call's replicated frontier moves as dense row slices (gsx_prop_rep_rows)."""
        self._chk(self.lib.gsx_prop_rep_rows(self.h, 1 if on else 0), "gsx_prop_rep_rows")

    def prop_rep_rows_export(self, rows, occ):
        """This rank's rows of the hop just run (n_local x W) and its occupancy-bit row (device)."""
        self._chk(self.lib.gsx_prop_rep_rows_export(self.h, self._p(rows), self._p(occ)), "gsx_prop_rep_rows_export")

    def prop_rep_rows_step(self, parts, occ_sum):
        """Every rank's rows of the hop (parts[k], the shard plan's ranges) and the summed bit row, then the next hop."""
        n = len(parts)
        pp = (C.c_void_p * max(n, 1))(*[self._p(t).value for t in parts])
        self._chk(self.lib.gsx_prop_rep_rows_step(self.h, n, pp, self._p(occ_sum)), "gsx_prop_rep_rows_step")

    def prop_rep_sends_pack(self, out):
        self._chk(self.lib.gsx_prop_rep_sends_pack(self.h, self._p(out)), "gsx_prop_rep_sends_pack")

    def prop_rep_sends_recv(self, inp):
        self._chk(self.lib.gsx_prop_rep_sends_recv(self.h, self._p(inp)), "gsx_prop_rep_sends_recv")

    def prop_set_last_hop(self, last_hop: int):
        """gsx_prop_set_last_hop: the last hop that delivered on any rank (range shards)."""
        self._chk(self.lib.gsx_prop_set_last_hop(self.h, int(last_hop)), "gsx_prop_set_last_hop")

    def prop_end(self) -> abi.PropOut:
        out = abi.PropOut()
        self._chk(self.lib.gsx_prop_end(self.h, C.byref(out)), "gsx_prop_end")
        return out

    def prop_results(self, n_msgs: int):
        """-> (hop [m, n_local] u8, first_from [m, n_local] i32) of the last propagation."""
        hop = np.empty((n_msgs, self.n_nodes), dtype=np.uint8)
        frm = np.empty((n_msgs, self.n_nodes), dtype=np.int32) if self._track else None
        self._chk(self.lib.gsx_prop_results(self.h, _ptr(hop, C.c_uint8), _ptr(frm, C.c_int32)), "gsx_prop_results")
        return hop, frm

    def pending_credits(self, first_ptr: int, dup_ptr: int):
        """Copy the pending (GSX_CREDIT_DEFER) counts to caller memory (host or device pointers)."""
        self._chk(self.lib.gsx_prop_pending_credits(self.h, C.c_void_p(first_ptr or None), C.c_void_p(dup_ptr or None)),
                  "gsx_prop_pending_credits")

    def pending_invalid(self, inv_ptr: int):
        """Copy the pending invalid-delivery counts (P4 of REJECT messages) to caller memory."""
        self._chk(self.lib.gsx_prop_pending_invalid(self.h, C.c_void_p(inv_ptr or None)), "gsx_prop_pending_invalid")

    def replace_pending_invalid(self, inv_ptr: int):
        self._chk(self.lib.gsx_prop_replace_pending_invalid(self.h, C.c_void_p(inv_ptr or None)),
                  "gsx_prop_replace_pending_invalid")

    def fold_credits(self, first_ptr: int = 0, dup_ptr: int = 0):
        self._chk(self.lib.gsx_prop_fold_credits(self.h, C.c_void_p(first_ptr or None), C.c_void_p(dup_ptr or None)),
                  "gsx_prop_fold_credits")

    # -- heartbeat (gossipsub.go:1303-1604) ----------------------------------------------
    def set_gossipsub_params(self, gp: abi.GossipSubParams):
        self._chk(self.lib.gsx_set_gossipsub_params(self.h, C.byref(gp)), "gsx_set_gossipsub_params")
        self._do_px = bool(gp.do_px)
        self._gx_on = bool(gp.gossip_exchange)

    _do_px = False

    def hb_px_enabled(self) -> bool:
        return self._do_px

    # peer exchange on range shards (gsx.h gsx_hb_px_*)
    def hb_px_entry_words(self) -> int:
        w = C.c_uint32()
        self._chk(self.lib.gsx_hb_px_entry_words(self.h, C.byref(w)), "gsx_hb_px_entry_words")
        return int(w.value)

    def hb_px_count(self, kind: int, n_ranks: int) -> np.ndarray:
        c = np.zeros(n_ranks, dtype=np.uint64)
        self._chk(self.lib.gsx_hb_px_count(self.h, kind, _ptr(c, C.c_uint64)), "gsx_hb_px_count")
        return c

    def hb_px_pack(self, kind: int, out):
        self._chk(self.lib.gsx_hb_px_pack(self.h, kind, self._p(out)), "gsx_hb_px_pack")

    def hb_px_recv(self, kind: int, entries, n: int):
        self._chk(self.lib.gsx_hb_px_recv(self.h, kind, self._p(entries), n), "gsx_hb_px_recv")

    def hb_reserve(self):
        """The heartbeat's device buffers allocated now (gsx_hb_reserve), not in the first round."""
        self._chk(self.lib.gsx_hb_reserve(self.h), "gsx_hb_reserve")

    def heartbeat(self, tick: int, now: int, seed: int) -> abi.HeartbeatOut:
        out = abi.HeartbeatOut()
        self._chk(self.lib.gsx_heartbeat(self.h, tick, now, seed, C.byref(out)), "gsx_heartbeat")
        return out

    @staticmethod
    def _p(t):
        return C.c_void_p((t.data_ptr() if hasattr(t, "data_ptr") else t) or None)

    def hb_begin(self, tick: int, now: int, seed: int):
        self._chk(self.lib.gsx_hb_begin(self.h, tick, now, seed), "gsx_hb_begin")

    def hb_pack_ctl(self, send):
        self._chk(self.lib.gsx_hb_pack_ctl(self.h, self._p(send)), "gsx_hb_pack_ctl")

    def hb_recv(self, halo_ctl):
        self._chk(self.lib.gsx_hb_recv(self.h, self._p(halo_ctl)), "gsx_hb_recv")

    def hb_pack_resp(self, send):
        self._chk(self.lib.gsx_hb_pack_resp(self.h, self._p(send)), "gsx_hb_pack_resp")

    def hb_end(self, halo_resp) -> abi.HeartbeatOut:
        out = abi.HeartbeatOut()
        self._chk(self.lib.gsx_hb_end(self.h, self._p(halo_resp), C.byref(out)), "gsx_hb_end")
        return out

    # ---- the gossip exchange across range shards (gsx_gx_*, gsx_gxf_*) ----
    def gx_pending(self):
        """-> the message sets of the sharded exchange in flight, or None."""
        n = C.c_uint32()
        rc = self.lib.gsx_gx_pending(self.h, C.byref(n))
        return int(n.value) if rc == 1 else None

    def gx_common(self, n_sets: int) -> np.ndarray:
        c = np.empty(64 * n_sets, dtype=np.uint64)
        self._chk(self.lib.gsx_gx_common(self.h, _ptr(c, C.c_uint64)), "gsx_gx_common")
        return c

    def gx_set_common(self, c: np.ndarray):
        c = np.ascontiguousarray(c, dtype=np.uint64)
        self._chk(self.lib.gsx_gx_set_common(self.h, _ptr(c, C.c_uint64)), "gsx_gx_set_common")

    def gx_pack_ihave(self, send):
        self._chk(self.lib.gsx_gx_pack_ihave(self.h, self._p(send)), "gsx_gx_pack_ihave")

    def gx_recv_ihave(self, recv):
        self._chk(self.lib.gsx_gx_recv_ihave(self.h, self._p(recv)), "gsx_gx_recv_ihave")

    def gx_rows_words(self) -> int:
        w = C.c_uint32()
        self._chk(self.lib.gsx_gx_rows_words(self.h, C.byref(w)), "gsx_gx_rows_words")
        return int(w.value)

    def gx_rows_pack(self, n_ranks: int, out=None) -> np.ndarray:
        """out None: the count pass -> entries per destination; else the pack."""
        cnt = np.zeros(n_ranks, dtype=np.uint64)
        self._chk(self.lib.gsx_gx_rows_pack(self.h, _ptr(cnt, C.c_uint64), self._p(out) if out is not None else None),
                  "gsx_gx_rows_pack")
        return cnt

    def gx_rows_recv(self, entries, n: int):
        self._chk(self.lib.gsx_gx_rows_recv(self.h, self._p(entries), n), "gsx_gx_rows_recv")

    def gx_exchange(self) -> int:
        n = C.c_uint32()
        self._chk(self.lib.gsx_gx_exchange(self.h, C.byref(n)), "gsx_gx_exchange")
        return int(n.value)

    def gxf_begin(self, run: int):
        self._chk(self.lib.gsx_gxf_begin(self.h, run), "gsx_gxf_begin")

    def gxf_entry_words(self) -> int:
        w = C.c_uint32()
        self._chk(self.lib.gsx_gxf_entry_words(self.h, C.byref(w)), "gsx_gxf_entry_words")
        return int(w.value)

    def gxf_pack_fout(self, send):
        self._chk(self.lib.gsx_gxf_pack_fout(self.h, self._p(send)), "gsx_gxf_pack_fout")

    def gxf_recv_fout(self, recv):
        self._chk(self.lib.gsx_gxf_recv_fout(self.h, self._p(recv)), "gsx_gxf_recv_fout")

    def gxf_pack(self, hop: int, n_ranks: int, out=None) -> np.ndarray:
        cnt = np.zeros(n_ranks, dtype=np.uint64)
        self._chk(self.lib.gsx_gxf_pack(self.h, hop, _ptr(cnt, C.c_uint64), self._p(out) if out is not None else None),
                  "gsx_gxf_pack")
        return cnt

    def gxf_step(self, hop: int, entries, n: int, sync: bool = True):
        """-> this rank's new frontier (sync=False: no host sync, -> None)."""
        f = C.c_uint64()
        self._chk(self.lib.gsx_gxf_step(self.h, hop, self._p(entries), n, C.byref(f) if sync else None),
                  "gsx_gxf_step")
        return int(f.value) if sync else None

    def gxf_pack_dev(self, hop: int, out, d_counts):
        """Entries into out (dense segments), (entries per rank, frontier of hop - 1) into d_counts; no sync."""
        self._chk(self.lib.gsx_gxf_pack_dev(self.h, hop, self._p(out), self._p(d_counts)), "gsx_gxf_pack_dev")

    def gxf_end(self):
        self._chk(self.lib.gsx_gxf_end(self.h), "gsx_gxf_end")

    def gx_got(self, n_sets: int) -> np.ndarray:
        g = np.zeros(max(n_sets, 1), dtype=np.uint8)
        self._chk(self.lib.gsx_gx_got(self.h, _ptr(g, C.c_uint8)), "gsx_gx_got")
        return g[:n_sets]

    def gx_end(self, got_all) -> abi.HeartbeatOut:
        out = abi.HeartbeatOut()
        g = np.ascontiguousarray(got_all, dtype=np.uint8)
        if len(g) == 0:
            g = np.zeros(1, dtype=np.uint8)
        self._chk(self.lib.gsx_gx_end(self.h, _ptr(g, C.c_uint8), C.byref(out)), "gsx_gx_end")
        return out

    def export_backoff(self) -> np.ndarray:
        b = np.empty((self.n_topics, self.n_pairs), dtype=np.int64)
        self._chk(self.lib.gsx_export_backoff(self.h, _ptr(b, C.c_int64)), "gsx_export_backoff")
        return b

    def import_backoff(self, b):
        b = np.ascontiguousarray(b, dtype=np.int64).reshape(self.n_topics, self.n_pairs)
        self._chk(self.lib.gsx_import_backoff(self.h, _ptr(b, C.c_int64)), "gsx_import_backoff")

    def gossip_results(self):
        """-> (ihave_len [T, E] u32, ihave_digest [T, E] u64) of the last heartbeat."""
        ln = np.empty((self.n_topics, self.n_pairs), dtype=np.uint32)
        dg = np.empty((self.n_topics, self.n_pairs), dtype=np.uint64)
        self._chk(self.lib.gsx_gossip_results(self.h, _ptr(ln, C.c_uint32), _ptr(dg, C.c_uint64)),
                  "gsx_gossip_results")
        return ln, dg

    def mcache_clear(self):
        self._chk(self.lib.gsx_mcache_clear(self.h), "gsx_mcache_clear")

    # -- message-parallel replicas: a batch from its message blocks (gsx.h gsx_mcache_*) --------
    # A block travels as one 1-D int64 device tensor: the cache rows, the
    # message set's rows, then its validation-code planes (the arrival hops,
    # vc_planes(cfg) of them), [n_nodes][words(n_msgs)] u64 each.
    def vc_planes(self, cfg) -> int:
        """Code planes a propagated block carries: the bits of its arrival hops
        and the code after the last (the room gsx_propagate leaves for a
        recovery round); none when every hop takes no time (every copy
        validated at now_ns), and none with the gossip exchange off (the
        calls then keep no hop codes, so the merged set keeps none either,
        as one engine's: gsx_mcache_copy_last refuses planes of such a set)."""
        if cfg is None or cfg.hop_latency_ns + cfg.validation_delay_ns <= 0 or not getattr(self, "_gx_on", True):
            return 0
        return int(cfg.max_hops + 1).bit_length()

    def mcache_part_size(self, n_msgs: int, cfg=None) -> int:
        return (2 + self.vc_planes(cfg)) * self.n_nodes * prop_words(n_msgs)

    def mcache_take_block(self, pad: int, device, cfg=None):
        """The newest cached batch (this replica's block) out of the cache ->
        (tensor of max(pad, its size) int64 on `device`, n_msgs); stream-ordered."""
        import torch

        W, m = C.c_uint32(), C.c_uint32()
        self._chk(self.lib.gsx_mcache_last(self.h, C.byref(W), C.byref(m)), "gsx_mcache_last")
        n = self.n_nodes * W.value
        p = self.vc_planes(cfg)
        t = torch.zeros(max(pad, (2 + p) * n), dtype=torch.int64, device=device)
        self._chk(self.lib.gsx_mcache_copy_last(self.h, C.c_void_p(t.data_ptr()), C.c_void_p(t.data_ptr() + 8 * n),
                                                C.c_void_p(t.data_ptr() + 16 * n), p), "gsx_mcache_copy_last")
        self._chk(self.lib.gsx_mcache_pop(self.h), "gsx_mcache_pop")
        return t, m.value

    def mcache_empty_block(self, pad: int, device):
        import torch

        return torch.zeros(pad, dtype=torch.int64, device=device)

    def mcache_put(self, msgs, cfg: abi.PropConfig, blocks, part_msgs):
        """gsx_mcache_put: msgs as one cached batch from the blocks (tensors as
        mcache_take_block returns them, block k = part_msgs[k] messages)."""
        ms = np.ascontiguousarray(msgs, dtype=abi.msg_dtype())
        k = len(blocks)
        sz = [self.n_nodes * prop_words(int(n)) for n in part_msgs]
        cp = (C.c_void_p * k)(*[b.data_ptr() for b in blocks])
        sp = (C.c_void_p * k)(*[b.data_ptr() + 8 * z for b, z in zip(blocks, sz)])
        vp = (C.c_void_p * k)(*[b.data_ptr() + 16 * z for b, z in zip(blocks, sz)])
        pm = np.ascontiguousarray(part_msgs, dtype=np.uint32)
        self._chk(self.lib.gsx_mcache_put(self.h, ms.ctypes.data_as(C.c_void_p), len(ms), C.byref(cfg), k,
                                          _ptr(pm, C.c_uint32), cp, sp, vp, self.vc_planes(cfg)), "gsx_mcache_put")

    def set_subscriptions(self, joined):
        """Joined topics per node (bit t of joined[v]); gsx_set_subscriptions."""
        j = np.ascontiguousarray(joined, dtype=np.uint64)
        self._chk(self.lib.gsx_set_subscriptions(self.h, _ptr(j, C.c_uint64)), "gsx_set_subscriptions")

    def export_membership(self):
        """-> (joined [N] u64, fanout [E] u64 topic bits, lastpub [N, T] i64)"""
        j = np.empty(self.n_nodes, dtype=np.uint64)
        f = np.empty(self.n_pairs, dtype=np.uint64)
        lp = np.empty((self.n_nodes, self.n_topics), dtype=np.int64)
        self._chk(self.lib.gsx_export_membership(self.h, _ptr(j, C.c_uint64), _ptr(f, C.c_uint64),
                                                 _ptr(lp, C.c_int64)), "gsx_export_membership")
        return j, f, lp

    def join(self, nodes, topics, now: int, seed: int) -> abi.HeartbeatOut:
        nd = np.ascontiguousarray(nodes, dtype=np.uint32)
        tp = np.ascontiguousarray(topics, dtype=np.uint32)
        out = abi.HeartbeatOut()
        self._chk(self.lib.gsx_join(self.h, _ptr(nd, C.c_uint32), _ptr(tp, C.c_uint32), len(nd), now, seed,
                                    C.byref(out)), "gsx_join")
        return out

    def leave(self, nodes, topics, now: int) -> abi.HeartbeatOut:
        nd = np.ascontiguousarray(nodes, dtype=np.uint32)
        tp = np.ascontiguousarray(topics, dtype=np.uint32)
        out = abi.HeartbeatOut()
        self._chk(self.lib.gsx_leave(self.h, _ptr(nd, C.c_uint32), _ptr(tp, C.c_uint32), len(nd), now,
                                     C.byref(out)), "gsx_leave")
        return out

    def hb_set_tracing(self, on: bool = True):
        self._chk(self.lib.gsx_hb_set_tracing(self.h, 1 if on else 0), "gsx_hb_set_tracing")

    def hb_set_px_log(self, cap: int):
        """Keep up to cap PX connection candidates per heartbeat (gsx_hb_set_px_log)."""
        self._chk(self.lib.gsx_hb_set_px_log(self.h, cap), "gsx_hb_set_px_log")

    def hb_px_records(self):
        """-> [n, 4] u32 (receiver, candidate, pruner, topic | kind << 8) of the last
        heartbeat, sorted (gsx_hb_px_records: min(px_connect, log cap) of them are kept)."""
        n = C.c_size_t()
        self._chk(self.lib.gsx_hb_px_records(self.h, None, 0, C.byref(n)), "gsx_hb_px_records")
        out = np.zeros((n.value, 4), dtype=np.uint32)
        self._chk(self.lib.gsx_hb_px_records(self.h, _ptr(out, C.c_uint32), n.value, C.byref(n)), "gsx_hb_px_records")
        return out

    def hb_trace_words(self):
        """-> (sent_graft, sent_prune, acc_graft, handled_prune) [E] u64 topic words
        of the last heartbeat (gsx_hb_trace_words; hb_set_tracing first)."""
        w = [np.empty(self.n_pairs, dtype=np.uint64) for _ in range(4)]
        self._chk(self.lib.gsx_hb_trace_words(self.h, *[_ptr(x, C.c_uint64) for x in w]), "gsx_hb_trace_words")
        return tuple(w)

    def mcache_ids(self, node: int, topic: int, n_windows: int) -> np.ndarray:
        """mcache.GetGossipIDs of `node` over its first n_windows windows."""
        n = C.c_size_t()
        self._chk(self.lib.gsx_mcache_ids(self.h, node, topic, n_windows, None, 0, C.byref(n)), "gsx_mcache_ids")
        out = np.empty(n.value, dtype=np.uint64)
        self._chk(self.lib.gsx_mcache_ids(self.h, node, topic, n_windows, _ptr(out, C.c_uint64), len(out),
                                          C.byref(n)), "gsx_mcache_ids")
        return out

    # -- the gossipTracer's promises (gossip_tracer.go:48-185) ------------------------------
    def promise_add(self, pair: int, handles, expire: int, seed: int = 0):
        """AddPromise(p, msgIDs): one of `handles` (Int31n, draws h(seed, 9, pair, k)) expiring at `expire`."""
        h = np.ascontiguousarray(handles, dtype=np.uint64)
        self._chk(self.lib.gsx_promise_add(self.h, pair, _ptr(h, C.c_uint64), len(h), expire, seed), "gsx_promise_add")

    def promise_broken(self, now: int):
        """GetBrokenPromises: -> (per-pair counts [n_pairs] u32, total); the broken ones are dropped."""
        cnt = np.zeros(self.n_pairs, dtype=np.uint32)
        tot = C.c_uint64()
        self._chk(self.lib.gsx_promise_broken(self.h, now, _ptr(cnt, C.c_uint32), C.byref(tot)), "gsx_promise_broken")
        return cnt, tot.value

    def promise_fulfill(self, node: int, handle: int):
        self._chk(self.lib.gsx_promise_fulfill(self.h, node, handle), "gsx_promise_fulfill")

    def promise_throttle(self, pair: int):
        self._chk(self.lib.gsx_promise_throttle(self.h, pair), "gsx_promise_throttle")

    def promise_count(self) -> int:
        n = C.c_uint64()
        self._chk(self.lib.gsx_promise_count(self.h, C.byref(n)), "gsx_promise_count")
        return n.value

    def timing_begin(self, max_launches: int):
        self._chk(self.lib.gsx_timing_begin(self.h, max_launches), "gsx_timing_begin")

    def timing_end(self):
        """-> (total_ms, min_ms, max_ms, n_launches) of the fused kernel over the region."""
        tot, lo, hi, n = C.c_double(), C.c_double(), C.c_double(), C.c_uint32()
        self._chk(
            self.lib.gsx_timing_end(self.h, C.byref(tot), C.byref(lo), C.byref(hi), C.byref(n)), "gsx_timing_end"
        )
        return tot.value, lo.value, hi.value, n.value

    # -- state ---------------------------------------------------------------------------
    def _view(self, arrays: Dict[str, np.ndarray]) -> abi.StateView:
        sv = abi.StateView()
        for f in abi.STATE_FIELDS:
            a = arrays.get(f)
            ct = _CTYPES[abi.STATE_DTYPES[f]]
            setattr(sv, f, _ptr(a, ct))
        return sv

    def import_state(self, st: Dict[str, np.ndarray]):
        arrays = {f: np.ascontiguousarray(st[f], dtype=abi.STATE_DTYPES[f]).reshape(-1) for f in abi.STATE_FIELDS}
        R = self.n_topics * self.n_pairs
        for f in abi.RECORD_FIELDS:
            assert arrays[f].size == R, (f, arrays[f].size, R)
        for f in abi.PAIR_FIELDS:
            assert arrays[f].size == self.n_pairs, f
        sv = self._view(arrays)
        sv.last_refresh_ns = int(st.get("last_refresh_ns", 0))
        self._chk(self.lib.gsx_import_state(self.h, C.byref(sv)), "gsx_import_state")

    def synthesize_state(self, spec: abi.SynthSpec):
        self._chk(self.lib.gsx_synthesize_state(self.h, C.byref(spec)), "gsx_synthesize_state")

    def snapshot(self) -> Dict[str, np.ndarray]:
        """gsx_peer_score_snapshot (inspectScoresExtended, score.go:463-493): per pair and
        per [topic][pair] record, the PeerScoreSnapshot / TopicScoreSnapshot fields."""
        out = {f: np.empty(self.n_pairs, dtype=d) for f, d in abi.SNAPSHOT_PAIR.items()}
        out.update({f: np.empty(self.n_topics * self.n_pairs, dtype=d) for f, d in abi.SNAPSHOT_RECORD.items()})
        sv = abi.ScoreSnapshot(**{f: out[f].ctypes.data_as(dict(abi.ScoreSnapshot._fields_)[f]) for f in out})
        self._chk(self.lib.gsx_peer_score_snapshot(self.h, C.byref(sv)), "gsx_peer_score_snapshot")
        return out

    def export_state(self) -> Dict[str, np.ndarray]:
        R = self.n_topics * self.n_pairs
        out = {}
        for f in abi.STATE_FIELDS:
            n = R if f in abi.RECORD_FIELDS else self.n_pairs
            out[f] = np.empty(n, dtype=abi.STATE_DTYPES[f])
        sv = self._view(out)
        self._chk(self.lib.gsx_export_state(self.h, C.byref(sv)), "gsx_export_state")
        out["last_refresh_ns"] = int(sv.last_refresh_ns)
        return out
