"""The heartbeat on the GPU (gsx_heartbeat through the C ABI) vs the CPU
oracle: mesh membership, records, backoff, scores and round counters,
bit-exact after every round."""
import numpy as np
import pytest

import gsx
import heartbeat_cases as hc
import oracle as orc
from gsx import abi

pytestmark = pytest.mark.gpu


def _same(a, b, what):
    for f in list(abi.STATE_FIELDS) + ["backoff", "scores", "ihave_len", "ihave_digest"]:
        x, y = np.asarray(a[f]), np.asarray(b[f])
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), (what, f, np.argwhere(x != y)[:5])


CASES = [
    # n, d, T, ticks, mesh_degree, mix, direct, disconnect, prop_msgs, first_tick
    (300, 6, 1, 4, 2, False, 0.0, 0.0, 0, 1),
    (400, 9, 2, 5, 14, True, 0.03, 0.03, 0, 13),
    (600, 6, 2, 6, 6, True, 0.02, 0.05, 64, 58),
    (2000, 8, 1, 3, 3, False, 0.0, 0.0, 128, 59),
    # ~50 peers per node: a wave's 64 rows exceed the LDS stage (windows of
    # rows), meshes of ~40 are pruned through the merge sort (> 32 entries)
    (500, 25, 1, 3, 40, False, 0.02, 0.0, 64, 59),
]


@pytest.mark.parametrize("case", CASES, ids=[f"n{c[0]}-T{c[2]}-m{c[4]}-t{c[9]}" for c in CASES])
def test_heartbeat_rounds_match_oracle(gpu_ok, case):
    n, d, T, ticks, md, mix, direct, disc, pm, t0 = case
    runs = []
    for be in (gsx.Engine(T), orc.Oracle(T)):
        runs.append(hc.mesh_run(be, n, d, T, seed=n + d, ticks=ticks, mesh_degree=md, mix=mix, direct=direct,
                                disconnect=disc, prop_msgs=pm, first_tick=t0, mostly_positive=(md < 6)))
    (_, go, gs), (_, wo, ws) = runs
    for k in range(ticks):
        assert go[k] == wo[k], (k, go[k], wo[k])
        _same(gs[k], ws[k], f"tick {k}")
    assert sum(o["grafts"] + o["prunes"] for o in go) > 0


def test_opportunistic_grafting_matches_oracle(gpu_ok):
    res = []
    for be in (gsx.Engine(1), orc.Oracle(1)):
        out, _ = hc.opportunistic_graft_case(be)
        res.append((out.as_dict(), hc.snapshot(be)))
    assert res[0][0] == res[1][0]
    assert res[0][0]["grafts"] == 2 and res[0][0]["graft_accepted"] == 2
    _same(res[0][1], res[1][1], "og")


def test_graft_flood_matches_oracle(gpu_ok):
    g, _ = hc.graft_flood_case(gsx.Engine(1))
    w, _ = hc.graft_flood_case(orc.Oracle(1))
    for (go, gsc, gb), (wo, wsc, wb) in zip(g, w):
        assert go == wo
        assert gsc == wsc
        assert np.array_equal(gb, wb)
    assert [r[0]["penalties"] for r in g] == [1, 2, 2, 0]


def test_heartbeat_custom_params(gpu_ok):
    gp = orc.default_gossipsub_params()
    gp.d, gp.d_lo, gp.d_hi, gp.d_score, gp.d_out = 4, 3, 7, 2, 1
    gp.opportunistic_graft_ticks = 2
    gp.prune_backoff_ns = 2500 * abi.MILLISECOND  # whole-second rounding of the PRUNE backoff
    runs = []
    for be in (gsx.Engine(2), orc.Oracle(2)):
        runs.append(hc.mesh_run(be, 500, 7, 2, seed=77, ticks=4, mesh_degree=9, gp=gp, first_tick=14))
    (_, go, gs), (_, wo, ws) = runs
    for k in range(4):
        assert go[k] == wo[k]
        _same(gs[k], ws[k], f"tick {k}")


def test_heartbeat_rejects_bad_params_and_degree(gpu_ok):
    e = gsx.Engine(1)
    gp = orc.default_gossipsub_params()
    gp.d_score = -1
    with pytest.raises(gsx.GsxError):
        e.set_gossipsub_params(gp)
    # a hub above the per-node limit of the hub rows (HB_HUB_MAX) is refused, not truncated
    n = 12_100
    cols = [list(range(1, n))] + [[0] for _ in range(1, n)]
    row_ptr = np.cumsum([0] + [len(c) for c in cols]).astype(np.int64)
    col = np.concatenate([np.array(c, dtype=np.int32) for c in cols])
    e.set_topic_params(0, abi.TopicScoreParams(time_in_mesh_quantum_ns=abi.SECOND))
    e.load_overlay(row_ptr, col)
    with pytest.raises(gsx.GsxError):
        e.heartbeat(1, hc.T0, 1)


def test_heartbeat_full_size(gpu_ok):
    """cfg3-style 100k nodes x 4 topics from the device-synthesized state:
    one round, parity against the oracle on the exported state."""
    n, T = 100_000, 4
    ov = hc.pc.overlay(n, 6, seed=21)
    e = gsx.Engine(T)
    o = orc.Oracle(T)
    from gsx import synth

    for be in (e, o):
        be.set_peer_params(synth.bench_peer_params())
        for t in range(T):
            be.set_topic_params(t, synth.spam_test_topic_params())
        be.set_thresholds(abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                                         opportunistic_graft_threshold=5))
        be.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    e.synthesize_state(abi.SynthSpec(seed=21, now_ns=hc.T0, fmd_max=50, mmd_max=150, mfp_max=5, imd_max_sybil=0,
                                     p_in_mesh=0.5, graft_window_ns=abi.HOUR, bp_max=2, p_disconnected=0.02,
                                     p_absent=0.01, expire_jitter_ns=abi.SECOND, sybil_first_node=n))
    o.import_state(e.export_state())
    for tick in (60, 61):
        now = hc.T0 + (tick - 59) * abi.SECOND
        go = e.heartbeat(tick, now, 5).as_dict()
        wo = o.heartbeat(tick, now, 5).as_dict()
        assert go == wo
        _same(hc.snapshot(e), hc.snapshot(o), f"tick {tick}")
        assert go["grafts"] > 0 and go["prunes"] > 0


def test_message_cache_matches_reference_test(gpu_ok):
    from test_heartbeat_oracle import _check_message_cache

    _check_message_cache(hc.message_cache_case(gsx.Engine(1)))


@pytest.mark.parametrize("max_ihave,msgs", [(5000, 64), (9, 80), (5000, 3000)], ids=["plain", "truncated", "long"])
def test_gossip_matches_oracle(gpu_ok, max_ihave, msgs):
    """emitGossip on the GPU: IHAVE targets, lengths and id-list digests
    bit-exact with the oracle over rounds that see 1..3 cached batches."""
    gp = orc.default_gossipsub_params()
    gp.max_ihave_length = max_ihave
    gp.history_gossip = 3
    runs = []
    for be in (gsx.Engine(2), orc.Oracle(2)):
        runs.append(hc.mesh_run(be, 700, 9, 2, seed=msgs, ticks=4, mesh_degree=5, gp=gp, prop_msgs=msgs,
                                mostly_positive=True, first_tick=59))
    (_, go, gs), (_, wo, ws) = runs
    for k in range(4):
        assert go[k] == wo[k], (k, go[k], wo[k])
        _same(gs[k], ws[k], f"tick {k}")
    assert sum(o["ihave_msgs"] for o in go) > 0


@pytest.mark.parametrize("md", [8, 300])
def test_heartbeat_hub_nodes_match_oracle(gpu_ok, md):
    """Nodes with more than 64 peers (HB_LANE_DEG) run their maintenance, gossip
    and GRAFT handling one wave each: a hub peering with 700 nodes (with a mesh
    of ~300 at md=300: over Dhi, a 300-entry sort) plus a second hub, over
    rounds with gossip, vs the oracle."""
    from test_gpu_propagation import _hub_overlay, _overlay_from_edges

    n, T = 705, 2
    ov = _hub_overlay(n, seed=3)
    edges = set()
    for u in range(n):
        for v in ov.col[ov.row_ptr[u]:ov.row_ptr[u + 1]]:
            edges.add((min(u, int(v)), max(u, int(v))))
    edges |= {(1, k) for k in range(2, 200)}  # a second hub
    ov = _overlay_from_edges(n, sorted(edges))
    gp = orc.default_gossipsub_params()
    gp.history_gossip = 3
    runs = []
    for be in (gsx.Engine(T), orc.Oracle(T)):
        hc.pc.setup(be, ov, T, seed=11, mesh_degree=md, disconnect_frac=0.02)
        be.set_gossipsub_params(gp)
        outs, snaps = [], []
        for k in range(4):
            now = hc.T0 + (3 + k) * abi.SECOND
            outs.append(be.heartbeat(59 + k, now, 1234).as_dict())
            snaps.append(hc.snapshot(be))
            cfg = hc.pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, latency_ms=5, seed=k)
            cfg.now_ns = now + 100 * abi.MILLISECOND
            be.propagate(hc.pc.messages(n, 70, 100 + k), cfg)
            be.refresh(now + 500 * abi.MILLISECOND)
        runs.append((outs, snaps))
    (go, gs), (wo, ws) = runs
    for k in range(4):
        assert go[k] == wo[k], (k, go[k], wo[k])
        _same(gs[k], ws[k], f"tick {k}")
    assert sum(o["grafts"] + o["prunes"] for o in go) > 0 and sum(o["ihave_msgs"] for o in go) > 0
