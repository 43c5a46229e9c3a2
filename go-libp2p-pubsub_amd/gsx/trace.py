"""Trace export: engine results as ``pb.TraceEvent`` records.

The reference's tracer builds one ``TraceEvent`` per router action
(``trace.go:105-134`` RejectMessage, ``trace.go:136-164`` DuplicateMessage, ``trace.go:166-194`` DeliverMessage,
``trace.go:468-520`` Graft / Prune) and ``PBTracer`` writes them to a file as
varint-length-delimited protobufs (``tracer.go:131-170``), so existing trace
tooling reads a stream of such records.  This module turns what the engine
already computes on the GPU into that stream:

* ``mesh_trace``     — GRAFT / PRUNE events of one heartbeat from the round's
  tracer words (``hb_trace_words()``, gsx_hb_trace_words): every graftPeer /
  prunePeer of the maintenance (gossipsub.go:1346, :1355), every GRAFT a
  receiver accepts (:795) and every PRUNE a node handles, including the PRUNE
  answers to rejected GRAFTs (:822).  A GRAFT answered with PRUNE therefore
  yields GRAFT (sender) + PRUNE (sender, handling the answer), as in the
  reference; the counts are grafts + graft_accepted and prunes +
  prunes_handled.  The order within a heartbeat follows Go map iteration in
  the reference and is not observable; here it is (pair, kind, topic).
* ``delivery_trace`` — per message: PUBLISH_MESSAGE at its source
  (validation.go:217) and DELIVER_MESSAGE there with receivedFrom = the source
  itself (pubsub.go:1124-1125, publishMessage delivers locally published
  messages too) — or, for a message validation does not accept, REJECT_MESSAGE
  there with its reason (PushLocal's validation, validation.go:216-342); then one
  DELIVER_MESSAGE (or REJECT_MESSAGE with its reason) per (node, message) first
  receipt, ``receivedFrom`` = the first deliverer; then, given the call's
  duplicate rows (gsx_prop_duplicates), one DUPLICATE_MESSAGE per further copy
  a node pushed (pushMsg's seenMessage branch, pubsub.go:1052-1056 ->
  trace.go:136-164), ``receivedFrom`` = the copy's sender, stamped with its
  arrival.  Copies dropped by AcceptFrom (graylisted senders) are never
  pushed and yield nothing, as in pubsub.go:1014-1017.

Field numbers and wire types follow ``pb/trace.proto:5-104``; fields are
written in field-number order, as the gogo marshaller does.  This is host-side
formatting of device results (I/O, not the data-parallel path): nothing here
computes scores or forwarding.
"""
from __future__ import annotations

from typing import Callable, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .abi import (
    GSX_REC_IN_MESH,
    GSX_VALIDATION_ACCEPT,
    GSX_VALIDATION_IGNORE,
    GSX_VALIDATION_REJECT,
    GSX_VALIDATION_THROTTLE,
)

# TraceEvent.Type (pb/trace.proto:24-38)
PUBLISH_MESSAGE = 0
REJECT_MESSAGE = 1
DUPLICATE_MESSAGE = 2
DELIVER_MESSAGE = 3
GRAFT = 11
PRUNE = 12

# TraceEvent sub-message field numbers (pb/trace.proto:10-22)
_SUB_FIELD = {PUBLISH_MESSAGE: 4, REJECT_MESSAGE: 5, DUPLICATE_MESSAGE: 6, DELIVER_MESSAGE: 7, GRAFT: 15, PRUNE: 16}

# RejectMessage reasons of the validation outcomes (tracer.go:26-38, validation.go:320-383)
REJECT_REASON = {
    GSX_VALIDATION_REJECT: "validation failed",
    GSX_VALIDATION_IGNORE: "validation ignored",
    GSX_VALIDATION_THROTTLE: "validation throttled",
}


def _varint(n: int) -> bytes:
    if n < 0:  # int64 / enum: two's complement in ten bytes
        n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _len_field(field: int, payload: bytes) -> bytes:
    return _varint(field << 3 | 2) + _varint(len(payload)) + payload


def _varint_field(field: int, v: int) -> bytes:
    return _varint(field << 3) + _varint(v)


def _s(x) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


def encode_event(etype: int, peer_id: bytes, timestamp: int, sub: bytes) -> bytes:
    """One TraceEvent{type, peerID, timestamp, <sub-message>} (pb/trace.proto:5-22)."""
    return (
        _varint_field(1, etype)
        + _len_field(2, _s(peer_id))
        + _varint_field(3, timestamp)
        + _len_field(_SUB_FIELD[etype], sub)
    )


def graft_event(observer: bytes, peer: bytes, topic: str, timestamp: int) -> bytes:
    """trace.go:468-493: Graft{peerID = p, topic}, emitted by the grafting node."""
    return encode_event(GRAFT, observer, timestamp, _len_field(1, _s(peer)) + _len_field(2, _s(topic)))


def prune_event(observer: bytes, peer: bytes, topic: str, timestamp: int) -> bytes:
    """trace.go:495-520: Prune{peerID = p, topic}."""
    return encode_event(PRUNE, observer, timestamp, _len_field(1, _s(peer)) + _len_field(2, _s(topic)))


def publish_event(node: bytes, msg_id: bytes, topic: str, timestamp: int) -> bytes:
    """trace.go:76-103: PublishMessage{messageID, topic} (proto :40-43)."""
    return encode_event(PUBLISH_MESSAGE, node, timestamp, _len_field(1, _s(msg_id)) + _len_field(2, _s(topic)))


def deliver_event(node: bytes, msg_id: bytes, topic: str, received_from: bytes, timestamp: int) -> bytes:
    """trace.go:166-194: DeliverMessage{messageID, topic, receivedFrom} (proto :58-62)."""
    sub = _len_field(1, _s(msg_id)) + _len_field(2, _s(topic)) + _len_field(3, _s(received_from))
    return encode_event(DELIVER_MESSAGE, node, timestamp, sub)


def reject_event(node: bytes, msg_id: bytes, received_from: bytes, reason: str, topic: str, timestamp: int) -> bytes:
    """trace.go:105-134: RejectMessage{messageID, receivedFrom, reason, topic} (proto :45-50)."""
    sub = (_len_field(1, _s(msg_id)) + _len_field(2, _s(received_from)) + _len_field(3, _s(reason))
           + _len_field(4, _s(topic)))
    return encode_event(REJECT_MESSAGE, node, timestamp, sub)


def duplicate_event(node: bytes, msg_id: bytes, received_from: bytes, topic: str, timestamp: int) -> bytes:
    """trace.go:136-164: DuplicateMessage{messageID, receivedFrom, topic} (proto :52-56)."""
    sub = _len_field(1, _s(msg_id)) + _len_field(2, _s(received_from)) + _len_field(3, _s(topic))
    return encode_event(DUPLICATE_MESSAGE, node, timestamp, sub)


def write_delimited(events: Iterable[bytes]) -> bytes:
    """PBTracer's stream (tracer.go:156-167, protoio delimited writer): varint length + record."""
    return b"".join(_varint(len(e)) + e for e in events)


def read_delimited(buf: bytes) -> List[bytes]:
    """Split a delimited stream back into records; raises ValueError on a truncated record."""
    out, i = [], 0
    while i < len(buf):
        n, shift = 0, 0
        while True:
            if i >= len(buf):
                raise ValueError("truncated length prefix")
            b = buf[i]
            i += 1
            n |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
        if i + n > len(buf):
            raise ValueError("truncated record")
        out.append(bytes(buf[i : i + n]))
        i += n
    return out


def default_peer_id(node: int) -> bytes:
    """Simulated nodes carry no libp2p key: their id is 'gsx-' + the node index."""
    return b"gsx-%d" % node


def default_msg_id(source: int, seqno: int) -> bytes:
    """DefaultMsgIdFn (pubsub.go) is string(from) + string(seqno): source id + 8-byte big-endian seqno."""
    return default_peer_id(source) + int(seqno).to_bytes(8, "big")


def pair_endpoints(row_ptr, col) -> Tuple[np.ndarray, np.ndarray]:
    """(observer, peer) of every pair of a CSR overlay: pair p is edge p (gsx.h overlay)."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    obs = np.repeat(np.arange(len(row_ptr) - 1, dtype=np.int64), np.diff(row_ptr))
    return obs, np.asarray(col, dtype=np.int64)


def mesh_changes(before_flags, after_flags, n_topics: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(topic, pair, grafted) of every record whose inMesh flag changed, in (pair, topic) order.

    Flags are ``rec_flags`` as export_state() returns them: topic-major,
    element [t * n_pairs + p] (gsx.h state import/export).
    """
    b = np.asarray(before_flags, dtype=np.uint8).reshape(n_topics, -1) & GSX_REC_IN_MESH
    a = np.asarray(after_flags, dtype=np.uint8).reshape(n_topics, -1) & GSX_REC_IN_MESH
    pair, topic = np.nonzero((a != b).T)
    return topic, pair, a[topic, pair] != 0


def mesh_trace(
    words,
    row_ptr,
    col,
    topics: Sequence[str],
    timestamp: int,
    peer_id: Callable[[int], bytes] = default_peer_id,
) -> Iterator[bytes]:
    """GRAFT / PRUNE events of one heartbeat from its tracer words
    ``(sent_graft, sent_prune, acc_graft, handled_prune)`` ([E] u64 topic bits
    per pair, hb_trace_words()), ordered by (pair, kind in that order, topic);
    every event's observer is the pair's owner and its peer the pair's peer."""
    obs, peer = pair_endpoints(row_ptr, col)
    kinds = (GRAFT, PRUNE, GRAFT, PRUNE)
    w = np.stack([np.asarray(x, dtype=np.uint64) for x in words])  # [4, E]
    for p in np.nonzero(np.any(w != 0, axis=0))[0].tolist():
        o, q = peer_id(int(obs[p])), peer_id(int(peer[p]))
        for kind, bits in zip(kinds, w[:, p].tolist()):
            t = 0
            while bits:
                if bits & 1:
                    yield (graft_event if kind == GRAFT else prune_event)(o, q, topics[t], timestamp)
                bits >>= 1
                t += 1


def delivery_trace(
    hop,
    first_from,
    msgs,
    topic: str,
    now: int,
    hop_latency_ns: int,
    peer_id: Callable[[int], bytes] = default_peer_id,
    msg_id: Optional[Callable[[int, int], bytes]] = None,
    node_base: int = 0,
    validation_delay_ns: int = 0,
    dup_rows=None,
    row_ptr=None,
    col=None,
) -> Iterator[bytes]:
    """PUBLISH_MESSAGE / DELIVER_MESSAGE / REJECT_MESSAGE (and, with
    ``dup_rows``, DUPLICATE_MESSAGE) events of one propagation on ``topic``,
    ordered by (message, source first, node), the duplicates of a message
    after its first receipts, by (receiving pair).

    ``hop`` / ``first_from`` are prop_results() rows ([m, n] arrival hop, 0xFF
    = never, 0 at the source; first deliverer, global id); ``msgs`` the
    published records (gsx.h GsxMsg: ``source``, ``validation``,
    ``msg_id``).  Message ids default to ``default_msg_id(source, msg_id)``.
    Every first receipt is validated: an accepted message yields
    DELIVER_MESSAGE, one that is not yields REJECT_MESSAGE with its reason
    (validation.go:320-383; it is seen but never delivered or forwarded).  The
    event time is the end of validation: ``now + hop * (hop_latency +
    validation_delay)``.  ``node_base`` is the shard's first global node id
    for range-sharded results.  ``dup_rows`` ([n_pairs, words] u64 of
    gsx_prop_duplicates, unsharded only) with the overlay's ``row_ptr`` /
    ``col``: a duplicate copy sent by v left v when its validation ended and
    arrived one hop latency later, ``now + h * hop_latency + (h - 1) *
    validation_delay`` with h = hop(v) + 1 (no validation for duplicates).
    """
    if first_from is None:
        raise ValueError("delivery_trace needs first-deliverer rows (gsx_prop_set_tracking on)")
    hop = np.asarray(hop)
    first_from = np.asarray(first_from)
    mid = msg_id or default_msg_id
    step = hop_latency_ns + validation_delay_ns
    if dup_rows is not None:
        if node_base != 0 or row_ptr is None or col is None:
            raise ValueError("duplicate rows need the unsharded overlay (row_ptr, col)")
        dup_rows = np.asarray(dup_rows, dtype=np.uint64)
        d_obs, d_peer = pair_endpoints(row_ptr, col)
    for m in range(hop.shape[0]):
        v = int(msgs["validation"][m])
        src = int(msgs["source"][m])
        ident = mid(src, int(msgs["msg_id"][m]))
        if node_base <= src < node_base + hop.shape[1] and hop[m, src - node_base] == 0:
            # the local publish: PublishMessage, then (accepted) the local delivery
            me = peer_id(src)
            yield publish_event(me, ident, topic, now)
            if v == GSX_VALIDATION_ACCEPT:
                yield deliver_event(me, ident, topic, me, now)
            else:  # its local validation (PushLocal -> validate, validation.go:216-342) rejects it
                yield reject_event(me, ident, me, REJECT_REASON[v], topic, now)
        for u in np.nonzero((hop[m] != 0xFF) & (hop[m] != 0))[0].tolist():
            node, frm, ts = peer_id(node_base + u), peer_id(int(first_from[m, u])), now + int(hop[m, u]) * step
            if v == GSX_VALIDATION_ACCEPT:
                yield deliver_event(node, ident, topic, frm, ts)
            else:
                yield reject_event(node, ident, frm, REJECT_REASON[v], topic, ts)
        if dup_rows is not None:
            bits = (dup_rows[:, m // 64] >> np.uint64(m % 64)) & np.uint64(1)
            for q in np.nonzero(bits)[0].tolist():
                sender = int(d_peer[q])
                h = int(hop[m, sender]) + 1
                ts = now + h * hop_latency_ns + (h - 1) * validation_delay_ns
                yield duplicate_event(peer_id(int(d_obs[q])), ident, peer_id(sender), topic, ts)
