"""Trace export (gsx/trace.py).

Wire format: every encoder is checked byte-for-byte against the protobuf
library's own serializer for a TraceEvent schema built at run time from
pb/trace.proto's field numbers (stated below), and parsed back by it.
Content: GRAFT / PRUNE streams from a heartbeat and DELIVER_MESSAGE /
REJECT_MESSAGE streams from a propagation are checked against the backend's own counters and
first-deliverer rows (oracle here; GPU == oracle byte-for-byte in
test_gpu_trace.py)."""
import numpy as np
import pytest

import oracle as orc
import trace_cases as tc
from gsx import abi
from gsx import trace as tr

pb = pytest.importorskip("google.protobuf")
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory  # noqa: E402

F = descriptor_pb2.FieldDescriptorProto


def _trace_event_class():
    """TraceEvent with the fields the exporter writes (pb/trace.proto:5-104)."""
    fd = descriptor_pb2.FileDescriptorProto(name="gsx_trace_test.proto", package="gsxtest", syntax="proto2")
    ev = fd.message_type.add(name="TraceEvent")
    en = ev.enum_type.add(name="Type")
    for name, num in [("PUBLISH_MESSAGE", 0), ("REJECT_MESSAGE", 1), ("DUPLICATE_MESSAGE", 2),
                      ("DELIVER_MESSAGE", 3), ("GRAFT", 11), ("PRUNE", 12)]:
        en.value.add(name=name, number=num)

    def sub(name, fields):
        m = ev.nested_type.add(name=name)
        for fname, num, typ in fields:
            m.field.add(name=fname, number=num, type=typ, label=F.LABEL_OPTIONAL)

    B, S = F.TYPE_BYTES, F.TYPE_STRING
    sub("PublishMessage", [("messageID", 1, B), ("topic", 2, S)])
    sub("RejectMessage", [("messageID", 1, B), ("receivedFrom", 2, B), ("reason", 3, S), ("topic", 4, S)])
    sub("DuplicateMessage", [("messageID", 1, B), ("receivedFrom", 2, B), ("topic", 3, S)])
    sub("DeliverMessage", [("messageID", 1, B), ("topic", 2, S), ("receivedFrom", 3, B)])
    sub("Graft", [("peerID", 1, B), ("topic", 2, S)])
    sub("Prune", [("peerID", 1, B), ("topic", 2, S)])
    ev.field.add(name="type", number=1, type=F.TYPE_ENUM, type_name=".gsxtest.TraceEvent.Type", label=F.LABEL_OPTIONAL)
    ev.field.add(name="peerID", number=2, type=B, label=F.LABEL_OPTIONAL)
    ev.field.add(name="timestamp", number=3, type=F.TYPE_INT64, label=F.LABEL_OPTIONAL)
    for fname, num, tname in [("publishMessage", 4, "PublishMessage"), ("rejectMessage", 5, "RejectMessage"), ("duplicateMessage", 6, "DuplicateMessage"), ("deliverMessage", 7, "DeliverMessage"),
                              ("graft", 15, "Graft"), ("prune", 16, "Prune")]:
        ev.field.add(name=fname, number=num, type=F.TYPE_MESSAGE, type_name=f".gsxtest.TraceEvent.{tname}",
                     label=F.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("gsxtest.TraceEvent"))


TE = _trace_event_class()
TS = [0, 1, 1_700_000_000_123_456_789, -5, (1 << 63) - 1]


@pytest.mark.parametrize("ts", TS)
def test_graft_prune_bytes_match_protobuf(ts):
    for kind, enc, field in [(11, tr.graft_event, "graft"), (12, tr.prune_event, "prune")]:
        want = TE(type=kind, peerID=b"obs\x00\xff", timestamp=ts)
        getattr(want, field).peerID = b"peer-7"
        getattr(want, field).topic = "té"
        got = enc(b"obs\x00\xff", b"peer-7", "té", ts)
        assert got == want.SerializeToString(deterministic=True)
        assert TE.FromString(got) == want


@pytest.mark.parametrize("ts", TS)
def test_publish_bytes_match_protobuf(ts):
    mid = tr.default_msg_id(3, 7)
    want = TE(type=0, peerID=b"src", timestamp=ts)
    want.publishMessage.messageID, want.publishMessage.topic = mid, "t"
    assert tr.publish_event(b"src", mid, "t", ts) == want.SerializeToString(deterministic=True)


@pytest.mark.parametrize("ts", TS)
def test_deliver_duplicate_bytes_match_protobuf(ts):
    mid = tr.default_msg_id(12, 300)
    want = TE(type=3, peerID=b"n1", timestamp=ts)
    want.deliverMessage.messageID, want.deliverMessage.topic, want.deliverMessage.receivedFrom = mid, "x", b"n2"
    assert tr.deliver_event(b"n1", mid, "x", b"n2", ts) == want.SerializeToString(deterministic=True)
    want = TE(type=2, peerID=b"n1", timestamp=ts)
    want.duplicateMessage.messageID, want.duplicateMessage.receivedFrom, want.duplicateMessage.topic = mid, b"n3", "x"
    assert tr.duplicate_event(b"n1", mid, b"n3", "x", ts) == want.SerializeToString(deterministic=True)
    want = TE(type=1, peerID=b"n1", timestamp=ts)
    r = want.rejectMessage
    r.messageID, r.receivedFrom, r.reason, r.topic = mid, b"n4", "validation failed", "x"
    assert tr.reject_event(b"n1", mid, b"n4", "validation failed", "x", ts) == want.SerializeToString(deterministic=True)


def test_delimited_round_trip_and_truncation():
    evs = [tr.graft_event(b"a" * k, b"b", "t", k) for k in (0, 1, 200, 5000)]  # 1- and 2-byte prefixes
    buf = tr.write_delimited(evs)
    assert tr.read_delimited(buf) == evs
    assert tr.read_delimited(b"") == []
    with pytest.raises(ValueError):
        tr.read_delimited(buf[:-1])
    with pytest.raises(ValueError):
        tr.read_delimited(b"\x80")


def test_mesh_changes_ordering():
    # 3 pairs x 2 topics, topic-major flags
    before = np.array([1, 0, 1, 0, 0, 1], dtype=np.uint8)
    after = np.array([1, 1, 0, 0, 1, 1], dtype=np.uint8) | np.uint8(0x80)  # other bits ignored
    t, p, g = tr.mesh_changes(before, after, 2)
    assert list(zip(p.tolist(), t.tolist(), g.tolist())) == [(1, 0, True), (1, 1, True), (2, 0, False)]


def test_mesh_trace_from_words_ordering():
    # pairs 0 (0 -> 5), 1 (0 -> 6), 2 (1 -> 7); words: sent GRAFT, sent PRUNE, accepted GRAFT, handled PRUNE
    row_ptr, col = np.array([0, 2, 3]), np.array([5, 6, 7])
    words = [np.array(x, dtype=np.uint64) for x in ([0, 3, 0], [0, 0, 1], [2, 0, 0], [0, 1, 1])]
    ev = [TE.FromString(e) for e in tr.mesh_trace(words, row_ptr, col, ["a", "b"], 9)]
    got = [(e.type, e.peerID, (e.graft if e.type == 11 else e.prune).peerID,
            (e.graft if e.type == 11 else e.prune).topic, e.timestamp) for e in ev]
    assert got == [(11, b"gsx-0", b"gsx-5", "b", 9),                               # pair 0: accepted
                   (11, b"gsx-0", b"gsx-6", "a", 9), (11, b"gsx-0", b"gsx-6", "b", 9),  # pair 1: sent
                   (12, b"gsx-0", b"gsx-6", "a", 9),                                 # its PRUNE answer
                   (12, b"gsx-1", b"gsx-7", "a", 9), (12, b"gsx-1", b"gsx-7", "a", 9)]  # sent + handled


def test_heartbeat_trace_matches_counters():
    """GRAFT events = grafts + graft_accepted, PRUNE events = prunes +
    prunes_handled (gossipsub.go:795, :822, :1346, :1355); a GRAFT answered
    with PRUNE shows as the sender's GRAFT and then its PRUNE."""
    buf, out, links_before, words = tc.heartbeat_stream(orc.Oracle(len(tc.TOPICS)))
    ev = [TE.FromString(e) for e in tr.read_delimited(buf)]
    n_graft = sum(e.type == 11 for e in ev)
    n_prune = sum(e.type == 12 for e in ev)
    assert n_graft == out["grafts"] + out["graft_accepted"] > 0
    assert n_prune == out["prunes"] + out["prunes_handled"] > 0
    assert all(e.HasField("graft") != e.HasField("prune") for e in ev)
    sg, sp, ag, hp = words
    assert out["graft_rejected"] > 0 and int(np.count_nonzero(sg & hp)) > 0  # rejected: GRAFT then PRUNE


CASES = [  # (invalid, delay_ms, router, gray, max_hops)
    (0.0, 0.0, abi.GSX_ROUTER_GOSSIPSUB, False, 40),
    (0.3, 0.0, abi.GSX_ROUTER_GOSSIPSUB, False, 40),
    (0.3, 4.0, abi.GSX_ROUTER_GOSSIPSUB, False, 40),
    (0.3, 0.0, abi.GSX_ROUTER_GOSSIPSUB, True, 40),
    (0.0, 0.0, abi.GSX_ROUTER_FLOODSUB, False, 3),
    (0.2, 2.0, abi.GSX_ROUTER_RANDOMSUB, False, 40),
]


@pytest.mark.parametrize("invalid,delay_ms,router,gray,max_hops", CASES)
def test_delivery_trace_matches_results(invalid, delay_ms, router, gray, max_hops):
    """PUBLISH / DELIVER / REJECT events follow the first receipts; one
    DUPLICATE per further pushed copy (as many as the call's duplicates
    counter), each from a neighbour that had the message one hop earlier and
    to a node that had already seen it, stamped with the copy's arrival."""
    buf, hop, frm, ms, out, dup = tc.delivery_stream(orc.Oracle(len(tc.TOPICS)), invalid=invalid, delay_ms=delay_ms,
                                                     router=router, gray=gray, max_hops=max_hops)
    ev = [TE.FromString(e) for e in tr.read_delimited(buf)]
    recv = (hop != 0xFF) & (hop != 0)
    n_dup = [int(((dup[:, m // 64] >> np.uint64(m % 64)) & np.uint64(1)).sum()) for m in range(len(ms))]
    assert sum(n_dup) == out.duplicates > 0
    assert len(ev) == int(recv.sum()) + 2 * len(ms) + sum(n_dup)
    if gray:
        assert out.graylisted > 0
    # per message: the source's PUBLISH_MESSAGE and its own DELIVER (REJECT when not accepted) first
    pub, rest, dups = [], [], []
    k = 0
    for m in range(len(ms)):
        pub.append((m, ev[k], ev[k + 1]))
        n = int(recv[m].sum())
        rest.extend(ev[k + 2:k + 2 + n])
        dups.append(ev[k + 2 + n:k + 2 + n + n_dup[m]])
        k += 2 + n + n_dup[m]
    now = tc.pc.T0 + 3 * tc.pc.S
    lat, dly = 10 * abi.MILLISECOND, int(delay_ms * abi.MILLISECOND)
    for m, p, d in pub:
        src = tr.default_peer_id(int(ms["source"][m]))
        mid = tr.default_msg_id(int(ms["source"][m]), int(ms["msg_id"][m]))
        assert p.type == 0 and p.peerID == src and p.publishMessage.messageID == mid and p.timestamp == now
        assert p.publishMessage.topic == tc.TOPICS[1]
        if int(ms["validation"][m]) == abi.GSX_VALIDATION_ACCEPT:
            assert d.type == 3 and d.deliverMessage.receivedFrom == src and d.deliverMessage.messageID == mid
        else:
            assert d.type == 1 and d.rejectMessage.receivedFrom == src
    m_idx, u_idx = np.nonzero(recv)
    n_rej = 0
    for e, m, u in zip(rest, m_idx.tolist(), u_idx.tolist()):
        v = int(ms["validation"][m])
        mid = tr.default_msg_id(int(ms["source"][m]), int(ms["msg_id"][m]))
        assert e.peerID == tr.default_peer_id(u)
        assert e.timestamp == now + int(hop[m, u]) * (lat + dly)
        if v == abi.GSX_VALIDATION_ACCEPT:
            d = e.deliverMessage
            assert e.type == 3 and not e.HasField("rejectMessage")
        else:  # not accepted: seen one hop from its source, rejected with the reason
            d = e.rejectMessage
            assert e.type == 1 and d.reason == tr.REJECT_REASON[v] and hop[m, u] == 1
            n_rej += 1
        assert d.messageID == mid and d.receivedFrom == tr.default_peer_id(int(frm[m, u]))
        assert d.topic == tc.TOPICS[1]
    assert (n_rej > 0) == (invalid > 0)
    node = {tr.default_peer_id(i): i for i in range(hop.shape[1])}
    for m in range(len(ms)):
        mid = tr.default_msg_id(int(ms["source"][m]), int(ms["msg_id"][m]))
        for e in dups[m]:
            assert e.type == 2 and e.duplicateMessage.messageID == mid and e.duplicateMessage.topic == tc.TOPICS[1]
            u, v = node[e.peerID], node[e.duplicateMessage.receivedFrom]
            h = int(hop[m, v]) + 1  # the sender had it one hop earlier
            assert hop[m, v] != 0xFF and h <= max_hops and u != int(ms["source"][m])
            assert hop[m, u] < h or (hop[m, u] == h and frm[m, u] != v)  # u had already seen it
            assert e.timestamp == now + h * lat + (h - 1) * dly


def test_delivery_trace_needs_first_deliverers():
    with pytest.raises(ValueError):
        list(tr.delivery_trace(np.zeros((1, 2), np.uint8), None, np.zeros(1, abi.msg_dtype()), "t", 0, 1))
