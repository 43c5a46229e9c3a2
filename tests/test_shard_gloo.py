"""Multi-process (world_size 2 and 3, gloo on CPU) runs of the multi-GPU
propagation drivers of gsx/shard.py, checked against the global oracle.

Range sharding: every rank holds one shard (tests/shard_emulator.py stands in
for the engine on CPU); the exchange plan and the per-hop all-to-all go
through torch.distributed exactly as on the GPUs (where the backend is RCCL).
The ranks' stitched arrival hops, first deliverers and summed counters must
equal orc_propagate's over the whole overlay.

Message parallel: every rank propagates its block of the messages with the
oracle standing in for the engine; the all-reduced totals must equal the
single run's.
"""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

import oracle as orc
import propagation_cases as pc
from gsx import abi, synth

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg_dict(cfg):
    return {f: getattr(cfg, f) for f, _ in abi.PropConfig._fields_}


def _worker(rank, world, port, payload, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gsx import shard as gs
        from gsx.abi import PropConfig

        cfg = PropConfig(**payload["cfg"]) if "cfg" in payload else None
        tp = gs.DistTransport("cpu")
        if payload["mode"] == "range":
            import shard_emulator as emu

            sh = payload["shards"][rank]
            rp = payload["row_ptr"]
            be = emu.EmuShard(sh, payload["fwd"][int(rp[sh.node_lo]) : int(rp[sh.node_hi])])
            rs = gs.RangeSharded(be, payload["rank_lo"], tp, compact=payload["compact"])
            if payload.get("heartbeat"):
                be.gx_sets = payload.get("gx_sets")
                local, tot = rs.heartbeat(1, 0, 0)
                q.put((rank, local, tot, be.hb_checked, None))
            else:
                local, tot = rs.propagate(payload["msgs"], cfg)
                hop, frm = be.prop_results(len(payload["msgs"]))
                q.put((rank, local, tot, hop, frm))
        elif payload["mode"] == "reprows":
            import shard_emulator as emu

            be = emu.RepRowsToy(payload["shards"][rank], payload["n"])
            rs = gs.RangeSharded(be, payload["rank_lo"], tp, compact=False, chunk=payload["chunk"])
            local, tot = rs.propagate(payload["msgs"], cfg)
            q.put((rank, local, tot, be.hop, (rs.host_syncs, rs.hops_run, be.last, rs.last_mode)))
        elif payload["mode"] == "replica_hb":
            import gossip_cases as gc

            o = orc.Oracle(2)
            run = gs.MessageParallel(o, tp)
            _, outs, snaps, cached = gc.exchange_run(o, runner=run, **payload["kw"])
            q.put((rank, outs, snaps, cached, run.gathered_bytes))
        else:
            o = orc.Oracle(1)
            pc.setup(o, payload["ov"], 1, payload["seed"])
            mpar = gs.MessageParallel(o, tp)
            local, tot = mpar.propagate(payload["msgs"], cfg)
            q.put((rank, local, tot, None, None))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as ex:  # report instead of hanging the parent
        import traceback

        q.put((rank, "error", traceback.format_exc(), None, None))


def _run(world, payload):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, payload, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=240)
        assert r[1] != "error", r[2]
        res[r[0]] = r
    for p in ps:
        p.join(60)
    return [res[r] for r in range(world)]


def _reference(ov, T, seed, msgs, cfg):
    o = orc.Oracle(T)
    pc.setup(o, ov, T, seed)
    st = o.export_state()
    scores = o.scores()
    out, hop, frm = o.propagate(msgs, cfg, want_results=True)
    return o, st, scores, out, hop, frm


CASES = [
    # world, n, d, router, flood_publish, m, mix, compact
    (2, 240, 3, abi.GSX_ROUTER_FLOODSUB, 0, 64, False, False),
    (2, 240, 3, abi.GSX_ROUTER_FLOODSUB, 0, 64, False, True),
    (2, 200, 4, abi.GSX_ROUTER_GOSSIPSUB, 0, 100, True, True),
    (3, 180, 3, abi.GSX_ROUTER_GOSSIPSUB, 1, 40, True, True),
]


@pytest.mark.parametrize("case", CASES, ids=[f"w{c[0]}-r{c[3]}-m{c[5]}-{'compact' if c[7] else 'dense'}" for c in CASES])
def test_range_sharded_gloo_matches_oracle(case):
    import shard_emulator as emu

    world, n, d, router, fp, m, mix, compact = case
    seed = 7 * n + m
    ov = pc.overlay(n, d, seed, mix_protocols=mix, direct_frac=0.03 if mix else 0.0)
    msgs = pc.messages(n, m, seed)
    cfg = pc.config(router, flood_publish=fp, credit=0, max_hops=30)
    th = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                        accept_px_threshold=0, opportunistic_graft_threshold=0)
    o, st, scores, out, hop, frm = _reference(ov, 1, seed, msgs, cfg)
    gl = th.graylist_threshold if router == abi.GSX_ROUTER_GOSSIPSUB else float("-inf")
    fwd = emu.fwd_bytes(router, st, scores, ov.edge_flags, 0, 1, th.publish_threshold, fp, gl)
    rank_lo = synth.shard_ranges(n, world)
    shards = [synth.shard_of(ov, int(rank_lo[k]), int(rank_lo[k + 1])) for k in range(world)]
    payload = dict(mode="range", shards=shards, fwd=fwd, row_ptr=ov.row_ptr, rank_lo=rank_lo, msgs=msgs,
                   cfg=_cfg_dict(cfg), compact=compact)
    res = _run(world, payload)
    got_hop = np.concatenate([r[3] for r in res], axis=1)
    got_frm = np.concatenate([r[4] for r in res], axis=1)
    assert np.array_equal(got_hop, hop), np.argwhere(got_hop != hop)[:5]
    assert np.array_equal(got_frm, frm), np.argwhere(got_frm != frm)[:5]
    tot = res[0][2]
    assert all(r[2] == tot for r in res)  # every rank holds the same totals
    want = out.as_dict()
    assert tot["deliveries"] == want["deliveries"] and tot["duplicates"] == want["duplicates"]
    assert tot["graylisted"] == want["graylisted"] and tot["transmissions"] == want["transmissions"]
    if router == abi.GSX_ROUTER_GOSSIPSUB:
        assert want["graylisted"] > 0  # the setup's app scores put some senders below the graylist
    assert tot["hops"] == want["hops"] and tot["hop_deliveries"] == want["hop_deliveries"]
    assert sum(r[1]["deliveries"] for r in res) == want["deliveries"]
    assert want["deliveries"] > 0


def test_message_parallel_gloo_totals():
    world, n, m = 2, 300, 96
    seed = 11
    ov = pc.overlay(n, 4, seed)
    msgs = pc.messages(n, m, seed)
    cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, credit=0)
    _, _, _, out, _, _ = _reference(ov, 1, seed, msgs, cfg)
    payload = dict(mode="replica", ov=ov, seed=seed, msgs=msgs, cfg=_cfg_dict(cfg))
    res = _run(world, payload)
    tot = res[0][2]
    want = out.as_dict()
    for k in ("deliveries", "duplicates", "transmissions", "hops"):
        assert tot[k] == want[k], k
    assert tot["hop_deliveries"] == want["hop_deliveries"]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_heartbeat_exchange_gloo(world):
    """The two control exchanges of a sharded heartbeat (GRAFT/PRUNE words to
    the receivers' ranks, PRUNE answers back) deliver every cross-shard
    pair's words to exactly its reverse pair's receive slot."""
    import shard_emulator as emu

    n = 240
    ov = pc.overlay(n, 4, 3)
    rank_lo = synth.shard_ranges(n, world)
    shards = [synth.shard_of(ov, int(rank_lo[k]), int(rank_lo[k + 1])) for k in range(world)]
    cfg = pc.config(abi.GSX_ROUTER_FLOODSUB)
    payload = dict(mode="range", shards=shards, fwd=np.zeros(ov.n_pairs, np.uint8), row_ptr=ov.row_ptr,
                   rank_lo=rank_lo, msgs=pc.messages(n, 1, 3), cfg=_cfg_dict(cfg), compact=False, heartbeat=True)
    res = _run(world, payload)
    obs = ov.pair_observer()
    owner = np.searchsorted(rank_lo.astype(np.int64), np.arange(n), side="right") - 1
    cross = owner[obs] != owner[ov.col]
    assert sum(r[3] for r in res) == 2 * int(cross.sum()) > 0


@pytest.mark.parametrize("world,n_sets", [(2, 3), (3, 2), (2, 0)])
def test_sharded_gossip_exchange_gloo(world, n_sets):
    """The gossip exchange of a sharded heartbeat (RangeSharded._gx_exchange
    over gsx_gx_* / gsx_gxf_*): the common words ANDed over ranks, the IHAVE
    words and the cache-row entries of the cross pairs, then every forwarding
    run's fout words and per-hop frontier entries until the frontier count
    summed over the ranks is 0, and the OR of the got flags.  The emulator's
    receive side checks every word and entry against its pair (with no
    message sets, the collectives of the set words are skipped)."""
    n = 240
    ov = pc.overlay(n, 4, 3)
    rank_lo = synth.shard_ranges(n, world)
    shards = [synth.shard_of(ov, int(rank_lo[k]), int(rank_lo[k + 1])) for k in range(world)]
    cfg = pc.config(abi.GSX_ROUTER_FLOODSUB)
    payload = dict(mode="range", shards=shards, fwd=np.zeros(ov.n_pairs, np.uint8), row_ptr=ov.row_ptr,
                   rank_lo=rank_lo, msgs=pc.messages(n, 1, 3), cfg=_cfg_dict(cfg), compact=False, heartbeat=True,
                   gx_sets=n_sets)
    res = _run(world, payload)
    obs = ov.pair_observer()
    owner = np.searchsorted(rank_lo.astype(np.int64), np.arange(n), side="right") - 1
    cross = owner[obs] != owner[ov.col]
    tot = res[0][2]
    # GRAFT/PRUNE words, answers, IHAVE words, two runs' fout words; one set-common check per rank
    assert tot["mesh_links"] == 5 * int(cross.sum()) + world
    v, u = obs[cross].astype(np.int64), ov.col[cross].astype(np.int64)
    assert tot["iwant_ids"] == int(((7 * v + u) % 3 == 0).sum())
    want_fwd = sum(int(((v + u + h + run) % 2 == 0).sum()) for run in range(2) for h in range(1, 3 + run))
    assert tot["fwd_delivered"] == want_fwd
    assert tot["fwd_duplicates"] == world * (2 + 3)


@pytest.mark.parametrize("world", [2, 3])
def test_message_parallel_heartbeat_gloo(world):
    """Message-parallel replicas with heartbeats: each replica propagates its
    block of every gossipsub batch, the cache blocks are all-gathered and Put
    back as whole batches (gsx_mcache_put), and every replica runs the whole
    heartbeat with the gossip exchange.  Every replica's counters, records,
    backoff, scores, IHAVEs and cached ids must equal one oracle's over the
    same rounds (batches that travel two hops: most nodes learn by IHAVE)."""
    import gossip_cases as gc
    import heartbeat_cases as hc

    kw = dict(n=240, ticks=4, msgs=30, invalid=0.2, credit=0)
    _, want_outs, want_snaps, want_cached = gc.exchange_run(orc.Oracle(2), **kw)
    res = _run(world, dict(mode="replica_hb", kw=kw))
    assert sum(o["iwant_msgs"] for o in want_outs) > 0 and sum(o["gossip_delivered"] for o in want_outs) > 0
    for rank, outs, snaps, cached, gathered in res:
        assert outs == want_outs, rank
        for k, (a, b) in enumerate(zip(snaps, want_snaps)):
            for f in list(a):
                assert np.array_equal(np.asarray(a[f]).reshape(-1).view(np.uint8), np.asarray(b[f]).reshape(-1).view(np.uint8)), (rank, k, f)
        for v in range(len(cached)):
            assert np.array_equal(np.sort(cached[v]), np.sort(want_cached[v])), (rank, v)
        assert gathered > 0


def _bfs_hops(ov, msgs, max_hops):
    """Arrival hop of every (message, node) of a flood over the whole overlay (-1: never)."""
    n = len(ov.row_ptr) - 1
    hop = np.full((len(msgs), n), -1, dtype=np.int32)
    for k, s in enumerate(msgs["source"]):
        hop[k, int(s)] = 0
        front = [int(s)]
        for h in range(1, max_hops + 1):
            nxt = []
            for u in range(n):
                if hop[k, u] >= 0:
                    continue
                nb = ov.col[ov.row_ptr[u] : ov.row_ptr[u + 1]]
                if any(hop[k, int(v)] == h - 1 for v in nb):
                    hop[k, u] = h
                    nxt.append(u)
            if not nxt:
                break
            front = nxt
    return hop


@pytest.mark.parametrize("world,chunk,max_hops", [(2, 4, 30), (3, 2, 30), (2, 3, 3), (3, 1, 30)])
def test_replicated_rows_driver_gloo(world, chunk, max_hops):
    """RangeSharded._rep_rows (the replicated frontier as dense row slices:
    one all-gather + one summed occupancy row per hop, the per-hop receipts
    read once per chunk) over gloo with the RepRowsToy shards: the stitched
    arrival hops equal a BFS over the whole overlay, every rank ends on the
    same last delivering hop, and the host reads are one per chunk of hops
    (plus the max_hops cut's)."""
    n, m = 150, 70
    seed = 5 + world
    ov = pc.overlay(n, 3, seed)
    msgs = pc.messages(n, m, seed)
    cfg = pc.config(abi.GSX_ROUTER_FLOODSUB, credit=0, max_hops=max_hops)
    want = _bfs_hops(ov, msgs, max_hops)
    rank_lo = synth.shard_ranges(n, world)
    shards = [synth.shard_of(ov, int(rank_lo[k]), int(rank_lo[k + 1])) for k in range(world)]
    res = _run(world, dict(mode="reprows", shards=shards, n=n, rank_lo=rank_lo, msgs=msgs, cfg=_cfg_dict(cfg),
                           chunk=chunk))
    got = np.concatenate([r[3] for r in res], axis=1)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    last_true = int(want.max())
    syncs, hops, last, mode = res[0][4]
    assert mode == "replicated-rows"
    assert all(r[4][2] == last_true for r in res)  # gsx_prop_set_last_hop: the last hop that delivered anywhere
    assert all(r[2] == res[0][2] for r in res)
    assert res[0][2]["deliveries"] == int((want > 0).sum())
    assert hops <= min(max_hops, last_true + chunk)  # at most chunk - 1 empty hops past the end
    assert syncs <= -(-(hops - 1) // chunk) + 1  # one read per chunk (+ max_hops 1's)
