#!/usr/bin/env python3
"""Headline benchmark: peer-topic score updates/s on BASELINE.json configs[2]
(1M peers x 8 topics, full P1-P7 refreshScores()+score() on one MI355X).

A step is one gsx_refresh(): the purge pass plus the fused refresh+score
kernel over every (observer, peer, topic) record of the shard, with all state
resident in HBM.  With --gpus N (launched by torch.distributed.run, one rank
per GPU) every rank owns its own 1M-observer shard (observers are
range-partitioned; scoring needs no exchange), so scaling is weak and `value`
is the records all ranks refreshed / the slowest rank's time.

Rank 0 at N=1 also times the CPU oracle (oracle/, a single-threaded C
restatement of score.go) on the same state for `cpu_baseline`, and checks
that the GPU scores of that pass are bit-identical to it.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-libp2p-pubsub_amd"))

import gsx  # noqa: E402
from gsx import abi, synth  # noqa: E402
from gsx import engine as gsx_engine_mod  # noqa: E402
from gsx import shard as shard_mod  # noqa: E402

METRIC = "peer-topic score updates/s + msg deliveries/s @1M peers, 1-8 GPUs, %HBM BW"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0  # measured float4 copy on MI355X (MI355X_MICROARCH.md): the achievable rate
BYTES_PER_RECORD = 82  # read fmd,mmd,mfp,imd,graftTime,flags; write the same with meshTime
BYTES_PER_PAIR = 49  # read bp, app, p6, expire, connected; write bp, score
T0 = 1_700_000_000 * abi.SECOND


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_engine(n, T, d, seed, device):
    t = time.time()
    ov = synth.connect_some_overlay(n, d=d, seed=seed)
    log(f"[bench] overlay n={n} pairs={ov.n_pairs} in {time.time() - t:.1f}s")
    e = gsx.Engine(T, device=device)
    e.set_peer_params(synth.bench_peer_params())
    tp = synth.spam_test_topic_params()
    for k in range(T):
        e.set_topic_params(k, tp)
    t = time.time()
    e.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    e.synthesize_state(
        abi.SynthSpec(seed=seed, now_ns=T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0, imd_max_sybil=100.0,
                      p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0, p_disconnected=0.0, p_absent=0.0,
                      expire_jitter_ns=4 * abi.SECOND, sybil_first_node=n)
    )
    e.set_app_scores(np.zeros(ov.n_pairs))
    log(f"[bench] engine loaded + state synthesized in {time.time() - t:.1f}s")
    return ov, e


PMC_FILE = "pmc_r06.json"  # written by tools/pmc.sh (tools/pmc_bytes.py)


def load_pmc():
    """The PMC byte counts committed under profiles/ (FETCH_SIZE x 2 + WRITE_SIZE,
    gfx950 correction), or {}."""
    try:
        with open(os.path.join(ROOT, "profiles", PMC_FILE)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def pmc_bytes(section, key, workload):
    """One PMC figure of a profiled workload, only when the leg ran that same
    workload (peers, topics, messages, exchange ...); else None: the bytes of
    another shape say nothing about this leg's traffic."""
    d = load_pmc().get(section) or {}
    if d.get("workload") != workload:
        return None
    return d.get(key)


def load_traffic(cfg_key):
    """Per-launch HBM bytes of the fused kernel from the rocprofv3 PMC pass
    committed under profiles/ (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction)."""
    return pmc_bytes("k_refresh_score<8, true>", "hbm_bytes_per_launch", {"config": cfg_key})


def single_observer_leg(args, device):
    """SURVEY.md §8 secondary view: ONE router scoring 1M peers on T topics
    (R = 8e6 records at T = 8): the drop-in shape of a single gossipsub node's
    score.go, as opposed to the 1M-observer overlay of the headline."""
    n_peers, T = args.peers, args.topics
    row_ptr = np.zeros(n_peers + 2, dtype=np.int64)
    row_ptr[1:] = n_peers  # node 0 observes nodes 1..n_peers
    col = np.arange(1, n_peers + 1, dtype=np.int32)
    ef = np.full(n_peers, abi.GSX_EDGE_GOSSIPSUB, dtype=np.uint8)
    ips = np.stack([np.arange(n_peers + 1, dtype=np.uint32) + 1, np.full(n_peers + 1, 0xFFFFFFFF, np.uint32)], axis=1)
    e = gsx.Engine(T, device=device)
    e.set_peer_params(synth.bench_peer_params())
    for k in range(T):
        e.set_topic_params(k, synth.spam_test_topic_params())
    e.load_overlay(row_ptr, col, ef, ips)
    e.synthesize_state(
        abi.SynthSpec(seed=synth.SEED + 5, now_ns=T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0, imd_max_sybil=100.0,
                      p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0, p_disconnected=0.0, p_absent=0.0,
                      expire_jitter_ns=4 * abi.SECOND, sybil_first_node=n_peers + 1))
    e.set_app_scores(np.zeros(n_peers))
    now = T0
    for _ in range(3):
        now += abi.SECOND
        e.refresh(now)
    e.sync()
    steps = max(1, args.steps)
    e.timing_begin(steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        now += abi.SECOND
        e.refresh(now)
    e.sync()
    el = time.perf_counter() - t0
    k_total, _, _, k_n = e.timing_end()
    e.close()
    R = n_peers * T
    kavg = k_total / max(1, k_n)
    B = BYTES_PER_RECORD * R + BYTES_PER_PAIR * n_peers
    return {"metric": "peer-topic score updates/s", "value": R * steps / el, "records": R, "peers": n_peers,
            "topics": T, "ms_per_refresh": el / steps * 1e3, "kernel_avg_ms": kavg,
            "roofline": {"bound": "hbm", "algorithmic_bytes_per_launch": B, "achieved": B / (kavg * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": B / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBS}}


def cpu_baseline(e, T, now, passes):
    """Single-threaded oracle refresh+score on the engine's exact state; also
    checks the GPU scores of the same pass bit-for-bit."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # checker / CPU baseline only

    t = time.time()
    st = e.export_state()
    o = orc.Oracle(T)
    o.set_peer_params(synth.bench_peer_params())
    tp = synth.spam_test_topic_params()
    for k in range(T):
        o.set_topic_params(k, tp)
    log(f"[bench] state exported in {time.time() - t:.1f}s")
    return o, st


def _oracle_mod():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # checker / CPU baseline only

    return orc


PROP_KEYS = ("deliveries", "duplicates", "transmissions", "graylisted", "rejected", "ignored", "hops")


def cpu_prop_baseline(e, n, d, th, cfg, seed, budget_s=12.0):
    """SURVEY §8d's CPU column for msg deliveries/s: the C oracle's propagate
    (oracle/gsx_oracle.c orc_propagate, a message-at-a-time restatement of
    floodsub.go:76-100 / gossipsub.go:943-1013 with the same P2/P3/P4
    credits) on the propagation engine's exact state, one thread, on a bounded
    sample: calls of a few messages each until about budget_s of CPU time.
    The GPU engine runs the same calls afterwards and every call's counters
    must agree (a parity check of the sample, not part of the timing)."""
    orc = _oracle_mod()
    t = time.time()
    st = e.export_state()
    o = orc.Oracle(1)
    o.set_peer_params(synth.bench_peer_params())
    o.set_topic_params(0, synth.spam_test_topic_params())
    o.set_thresholds(th)
    o.set_gossipsub_params(gsx_engine_mod.default_gossipsub_params(gossip_exchange=0))
    ov = synth.connect_some_overlay(n, d=d, seed=seed)
    o.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    del ov
    o.import_state(st)
    o.set_app_scores(np.zeros(e.n_pairs))
    del st
    log(f"[bench] oracle propagation state in {time.time() - t:.1f}s")
    calls, secs, dl = [], 0.0, 0
    per_call = 4
    while secs < budget_s and len(calls) < 64:
        msgs = prop_messages(n, per_call, seed, first=90_000_000 + per_call * len(calls))
        t = time.perf_counter()
        out = o.propagate(msgs, cfg)[0]
        secs += time.perf_counter() - t
        d = out.as_dict()
        dl += d["deliveries"]
        calls.append((msgs, {k: d[k] for k in PROP_KEYS}))
    o.close()
    bad = 0
    for msgs, want in calls:
        d = e.propagate(msgs, cfg)[0].as_dict()
        bad += {k: d[k] for k in PROP_KEYS} != want
    return {"value": dl / secs, "unit": "msg deliveries/s", "cores": 1, "kind": "port",
            "sample": f"{len(calls)} gossipsub calls of {per_call} messages over the {n}-peer overlay of this leg, "
                      f"P2/P3 credits on ({secs:.1f}s of one core; oracle/gsx_oracle.c orc_propagate, gcc -O3; "
                      f"a message-at-a-time restatement, not reference Go: no Go on the box)",
            "nproc": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "sample_parity_vs_gpu": "bit-exact counters" if bad == 0 else f"MISMATCH in {bad} of {len(calls)} calls"}


def cpu_hb_baseline(args, local, seed, n_cpu=20_000, settle=3, timed=2):
    """The CPU column for the heartbeat: the C oracle's heartbeat (orc_heartbeat:
    gossipsub.go:1303-1564 with handleGraft/Prune and the gossip exchange,
    :615-716) on a cfg3-shaped sample (n_cpu peers x --topics, the bench's
    generator, --hb-msgs gossipsub messages propagated before every round),
    one thread.  The GPU engine runs the same sequence beside it and every
    round's counters must agree."""
    orc = _oracle_mod()
    T = args.topics
    ov, g = build_engine(n_cpu, T, args.degree, seed, local)
    g.refresh(T0 + abi.SECOND)
    st = g.export_state()
    o = orc.Oracle(T)
    o.set_peer_params(synth.bench_peer_params())
    for k in range(T):
        o.set_topic_params(k, synth.spam_test_topic_params())
    o.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
    o.import_state(st)
    o.set_app_scores(np.zeros(ov.n_pairs))
    del st
    th_hb = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                           accept_px_threshold=0, opportunistic_graft_threshold=5)
    gp = gsx_engine_mod.default_gossipsub_params(gossip_exchange=1 if args.hb_exchange else 0)
    for be in (g, o):
        be.set_thresholds(th_hb)
        be.set_gossipsub_params(gp)
    cfg = prop_config(args, n_cpu)
    now, tick = T0 + abi.SECOND, 59 - settle - timed
    secs, bad, rounds = 0.0, 0, 0
    for k in range(settle + timed):
        tick += 1
        now += abi.SECOND
        cfg.now_ns = now - abi.SECOND // 2
        msgs = prop_messages(n_cpu, args.hb_msgs, seed, first=70_000_000 + k * args.hb_msgs)
        o.propagate(msgs, cfg)
        g.propagate(msgs, cfg)
        t = time.perf_counter()
        oo = o.heartbeat(tick, now, seed).as_dict()
        if k >= settle:
            secs += time.perf_counter() - t
            rounds += 1
        bad += g.heartbeat(tick, now, seed).as_dict() != oo
    o.close()
    g.close()
    return {"value": n_cpu * T * rounds / secs, "unit": "heartbeat (node, topic) mesh units/s", "cores": 1,
            "kind": "port", "ms_per_round": secs / rounds * 1e3,
            "sample": f"{n_cpu} peers x {T} topics (cfg3's generator and parameters), {settle} settle + {timed} "
                      f"timed rounds (ticks {tick - timed + 1}-{tick}) with {args.hb_msgs} gossipsub messages "
                      f"before each, gossip exchange {'on' if args.hb_exchange else 'off'}; oracle/gsx_oracle.c "
                      f"orc_heartbeat, one core, {secs:.2f}s timed (restatement, not reference Go)",
            "nproc": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "sample_parity_vs_gpu": "bit-exact counters every round" if bad == 0 else
                                    f"MISMATCH in {bad} of {settle + timed} rounds"}


def prop_engine(n_total, lo, hi, d, seed, device, th, sharded):
    """Engine for a propagation leg: T=1, spam-test params, synthesized state
    (mesh ~ half of each node's peers), one refresh so publishThreshold tests
    read real scores."""
    t = time.time()
    e = gsx.Engine(1, device=device)
    e.set_peer_params(synth.bench_peer_params())
    e.set_topic_params(0, synth.spam_test_topic_params())
    e.set_thresholds(th)
    if sharded:
        rl = synth.shard_ranges(n_total, sharded[1])
        sh = synth.connect_some_shards(n_total, rl, d=d, seed=seed, ranks=[sharded[0]])[0]
        e.load_overlay_shard(n_total, sh.node_lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        n_pairs = sh.n_pairs
    else:
        ov = synth.connect_some_overlay(n_total, d=d, seed=seed)
        e.load_overlay(ov.row_ptr, ov.col, ov.edge_flags, ov.node_ips)
        n_pairs = ov.n_pairs
        del ov
    e.synthesize_state(
        abi.SynthSpec(seed=seed, now_ns=T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0, imd_max_sybil=100.0,
                      p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0, p_disconnected=0.0, p_absent=0.0,
                      expire_jitter_ns=4 * abi.SECOND, sybil_first_node=n_total))
    e.set_app_scores(np.zeros(n_pairs))
    e.refresh(T0 + abi.SECOND)
    # a propagation-only engine: no heartbeat runs on it, so no gossip exchange
    # reads its message sets' per-node validation times (gsx.h (D)) and the
    # calls skip building them (the heartbeat / adversarial legs keep it on)
    e.set_gossipsub_params(gsx_engine_mod.default_gossipsub_params(gossip_exchange=0))
    # throughput runs keep per-pair first-receipt counts, not first-deliverer
    # rows (gsx_prop_set_tracking; credits and duplicates are unchanged)
    e.set_prop_tracking(False)
    e.sync()
    log(f"[bench] propagation engine nodes={hi - lo}/{n_total} pairs={n_pairs} in {time.time() - t:.1f}s")
    return e


def prop_messages(n, m, seed, first=0):
    ms = np.zeros(m, dtype=abi.msg_dtype())
    k = np.arange(first, first + m)
    ms["source"] = (synth.h(seed, synth.TAG_SRC, k, 0) % np.uint64(n)).astype(np.uint32)
    ms["msg_id"] = k.astype(np.uint64)
    return ms


def prop_config(args, n):
    return abi.PropConfig(router=abi.GSX_ROUTER_GOSSIPSUB, topic=0, flood_publish=0, max_hops=args.prop_hops,
                          hop_latency_ns=10 * abi.MILLISECOND, now_ns=T0 + 2 * abi.SECOND,
                          credit_scores=abi.GSX_CREDIT_NOW, randomsub_size=n, seed=synth.SEED)


def with_traffic(roof, traffic, ms):
    """Adds the PMC-measured bytes (profiles/PMC_FILE) beside the algorithmic
    ones; traffic None (no PMC pass of this leg's workload) is reported as null."""
    if roof is None:
        return roof
    if traffic and ms:
        ach = traffic / (ms * 1e-3) / 1e9
        roof.update(traffic=traffic, achieved_traffic=ach, frac_traffic=ach / HBM_PEAK_GBS,
                    traffic_source=f"profiles/{PMC_FILE} (tools/pmc.sh)")
    else:
        roof.update(traffic=None, traffic_source=f"none: profiles/{PMC_FILE} holds no PMC pass of this workload")
    return roof


def prop_workload(n, msgs):
    """The propagation workload key shared with tools/pmc_bytes.py (tools/prop_profile.py)."""
    return {"peers": int(n), "msgs": int(msgs), "router": "gossipsub", "credit": "now"}


def hb_workload(n, T, msgs, exchange):
    """The heartbeat workload key shared with tools/pmc_bytes.py (tools/hb_micro.py)."""
    return {"peers": int(n), "topics": int(T), "msgs_between_rounds": int(msgs), "exchange": bool(exchange)}


def prop_roofline(tot, msgs, kernel_ms):
    """SURVEY.md §8d push-minimal bytes: 8 per frontier (vertex, word), 12 per
    eligible (edge, word) send, 16 per (vertex, word) gaining bits; the
    frontier words are the sources' plus every gaining word."""
    W = shard_mod.prop_words(len(msgs))
    src_words = len(set((int(s), k // 64) for k, s in enumerate(msgs["source"])))
    F = src_words + tot["new_words"]
    B = 8 * F + 12 * tot["edge_sends"] + 16 * tot["new_words"]
    ach = B / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    return {"bound": "hbm", "algorithmic_bytes_per_batch": B, "hop_kernel_ms_per_batch": kernel_ms,
            "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "words": W}


REHEARSE = False  # set by --rehearse: scalars reduce through host memory (gloo)


def reduce_scalar(x, dist, dev, op="max"):
    """MAX / SUM of a host scalar over ranks (x itself without a group)."""
    import torch

    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if REHEARSE else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def _max_over_ranks(x, dist, dev):
    return reduce_scalar(x, dist, dev, "max")


def prop_replica(args, rank, world, local, dist, dev, th):
    import torch

    n = args.peers
    e = prop_engine(n, 0, n, args.degree, synth.SEED, local, th, None)
    cfg = prop_config(args, n)
    M = args.prop_msgs * world
    tp = shard_mod.DistTransport(dev, stage_host=args.rehearse) if dist is not None else None
    # no heartbeat follows this leg: the replicas' cache blocks are not merged
    # (MessageParallel(cache=True) all-gathers them for replicated heartbeats).
    # Credits accumulate over a heartbeat epoch of --epoch-batches batches and
    # are summed over the replicas once per epoch, not per batch.
    runner = shard_mod.MessageParallel(e, tp, epoch=True, cache=False) if tp is not None else None
    eb = max(1, args.epoch_batches)

    def once(b):
        msgs = prop_messages(n, M, synth.SEED, first=b * M)
        if runner is not None:
            r = runner.propagate(msgs, cfg)
            if b % eb == 0:  # (warm-up batch 0 closes its own epoch; then every eb batches)
                runner.end_epoch()
            return r, msgs
        out = e.propagate(msgs, cfg)[0]
        d = shard_mod.out_dict(out)
        d2 = dict(d)
        d2["hop_kernel_ms_max"] = d["hop_kernel_ms"]
        return (d, d2), msgs

    once(0)  # warm-up
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    res = [once(1 + b) for b in range(args.prop_steps)]
    if runner is not None:
        runner.end_epoch()  # the last (partial) epoch's credits, inside the timed region
    e.settle_scores()  # deferred re-scores of the lazy folds (timed)
    torch.cuda.synchronize(dev)
    el = _max_over_ranks(time.perf_counter() - t0, dist, dev)
    dl = sum(r[0][1]["deliveries"] for r in res)
    (loc, tot), msgs = res[-1]
    mine = prop_messages(n, M, synth.SEED, first=args.prop_steps * M)
    mine = mine[(M * rank) // world : (M * (rank + 1)) // world]
    legs = prop_variant_legs(args, e, n) if world == 1 else None
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu:
        cpu = cpu_prop_baseline(e, n, args.degree, th, cfg, synth.SEED)
    e.close()
    return {
        "variants": legs,
        "cpu_baseline": cpu,
        "metric": "msg deliveries/s",
        "mode": ("message-parallel replicas (weak): full overlay per GPU, own messages, credits deferred and summed "
                 f"with one all-reduce per epoch of {eb} batches (cache blocks not merged: no heartbeat in this "
                 "leg)") if world > 1 else
                "one engine, full overlay (the 1-GPU point of the message-parallel leg: no collective)",
        "value": dl / el,
        "peers": n,
        "messages_per_batch_per_gpu": args.prop_msgs,
        "ms_per_batch": el / args.prop_steps * 1e3,
        "deliveries_per_batch": tot["deliveries"],
        "duplicates_per_batch": tot["duplicates"],
        "hops": tot["hops"],
        "router": "gossipsub (synthesized mesh, ~6 of ~12 peers), P2/P3 credits on",
        "roofline_rank0": with_traffic(prop_roofline(loc, mine, loc["hop_kernel_ms"]),
                                       pmc_bytes("p1024", "hop_bytes_per_batch", prop_workload(n, args.prop_msgs)),
                                       loc["hop_kernel_ms"]),
    }


def prop_leg(e, n, M, cfg, steps, seed, first):
    """Times `steps` batches of M messages on one engine (after one warm-up
    batch): deliveries/s, ms per batch, hop-kernel time and the push-minimal
    roofline of the last batch."""
    import torch

    e.propagate(prop_messages(n, M, seed, first=first), cfg)
    e.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = []
    for b in range(steps):
        msgs = prop_messages(n, M, seed, first=first + (1 + b) * M)
        outs.append(shard_mod.out_dict(e.propagate(msgs, cfg)[0]))
    e.settle_scores()  # the re-scores the credit folds deferred (lazy fold): timed, once per leg
    e.sync()
    el = time.perf_counter() - t0
    last = outs[-1]
    kms = sum(o["hop_kernel_ms"] for o in outs) / steps
    return {"value": sum(o["deliveries"] for o in outs) / el, "unit": "msg deliveries/s", "messages_per_batch": M,
            "ms_per_batch": el / steps * 1e3, "hop_kernel_ms_per_batch": kms, "hops": last["hops"],
            "deliveries_per_batch": last["deliveries"], "duplicates_per_batch": last["duplicates"],
            "graylisted_per_batch": last["graylisted"], "roofline": prop_roofline(last, msgs, kms)}


def prop_variant_legs(args, e, n):
    """BASELINE.md's other propagation shapes on the replica engine: 64-message
    batches (cfg2/cfg4's batch size), the floodsub router, and gossipsub with a
    P3 window shorter than the run (duplicates counted per hop by the general
    k_prop_hop kernel instead of the lean k_prop_hop_fast)."""
    steps = max(3, args.prop_steps)
    seed = synth.SEED + 7
    out = {}
    cfg = prop_config(args, n)
    out["gossipsub_64msg"] = prop_leg(e, n, 64, cfg, 4 * steps, seed, 10_000_000)
    with_traffic(out["gossipsub_64msg"]["roofline"], pmc_bytes("p64", "hop_bytes_per_batch", prop_workload(n, 64)),
                 out["gossipsub_64msg"]["hop_kernel_ms_per_batch"])
    fcfg = prop_config(args, n)
    fcfg.router = abi.GSX_ROUTER_FLOODSUB
    out["floodsub_1024msg"] = prop_leg(e, n, args.prop_msgs, fcfg, steps, seed, 20_000_000)
    out["floodsub_64msg"] = prop_leg(e, n, 64, fcfg, 4 * steps, seed, 30_000_000)
    tp = synth.spam_test_topic_params()
    tp.mesh_message_deliveries_window_ns = 25 * abi.MILLISECOND  # 2 hops of 10 ms: late copies fall outside
    e.set_topic_params(0, tp)
    leg = prop_leg(e, n, args.prop_msgs, cfg, steps, seed, 40_000_000)
    leg["note"] = "P3 window 25 ms < run: per-hop duplicate accounting, general k_prop_hop kernel"
    out["gossipsub_1024msg_short_window"] = leg
    e.set_topic_params(0, synth.spam_test_topic_params())
    return out


def prop_sharded(args, rank, world, local, dist, dev, th):
    import torch

    n = args.prop_peers
    rl = synth.shard_ranges(n, world)
    e = prop_engine(n, int(rl[rank]), int(rl[rank + 1]), args.degree, synth.SEED + 1, local, th,
                    (rank, world) if world > 1 else None)
    cfg = prop_config(args, n)
    M = args.shard_msgs  # 64-message batches
    steps = 4 * args.prop_steps
    runner = None
    if dist is not None:
        runner = shard_mod.RangeSharded(e, rl, shard_mod.DistTransport(dev, stage_host=args.rehearse),
                                        compact=args.shard_exchange == "compact", chunk=args.shard_chunk)

    def once(b):
        msgs = prop_messages(n, M, synth.SEED + 1, first=b * M)
        if runner is not None:
            return runner.propagate(msgs, cfg), msgs
        out = e.propagate(msgs, cfg)[0]
        d = shard_mod.out_dict(out)
        d2 = dict(d)
        d2["hop_kernel_ms_max"] = d["hop_kernel_ms"]
        return (d, d2), msgs

    once(0)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    res = [once(1 + b) for b in range(steps)]
    torch.cuda.synchronize(dev)
    el = _max_over_ranks(time.perf_counter() - t0, dist, dev)
    dl = sum(r[0][1]["deliveries"] for r in res)
    (loc, tot), msgs = res[-1]
    e.close()
    out = {
        "metric": "msg deliveries/s",
        "mode": (f"range-sharded (strong): {n} peers over {world} GPUs, per-hop all-to-all of packed cross-shard sends"
                 if world > 1 else f"one engine holding all {n} peers (the 1-GPU point of the range-sharded leg: "
                 "no cross-shard pairs, no all-to-all)"),
        "value": dl / el,
        "peers": n,
        "messages_per_batch": M,
        "ms_per_batch": el / steps * 1e3,
        "deliveries_per_batch": tot["deliveries"],
        "duplicates_per_batch": tot["duplicates"],
        "hops": tot["hops"],
        "router": "gossipsub (synthesized mesh, ~6 of ~12 peers), P2/P3 credits on",
        "hop_kernel_ms_max_rank": tot["hop_kernel_ms_max"],
    }
    if world == 1:
        out["roofline"] = prop_roofline(tot, msgs, loc["hop_kernel_ms"])
    else:
        out["exchange"] = {"mode": runner.last_mode, "compacted": runner.compact,
                           "chunk": None if runner.compact else runner.chunk,
                           "bytes_sent_per_batch_rank": runner.sent_bytes / (steps + 1),
                           "dense_bytes_per_hop_rank": runner.n_send * shard_mod.prop_words(M) * 8,
                           "hops_per_batch": runner.hops_run / (steps + 1),
                           "host_syncs_per_hop": runner.host_syncs / max(runner.hops_run, 1),
                           "ms_per_hop": el / max(runner.hops_run * steps / (steps + 1), 1) * 1e3}
    return out


def adversarial_leg(args, rank, world, local, dist, dev):
    """20 % sybils in IP groups of 50 attacking victim nodes
    (P6) with invalid-message counters (P4); observers range-sharded over the
    ranks.  Times refreshScores()+score() and reports how the scores treat the
    sybils; at N=1 also two heartbeats and the sybil mesh links they prune."""
    import torch

    n = args.adv_peers
    rl = synth.shard_ranges(n, world)
    t = time.time()
    sh = synth.adversarial_shards(n, rl, seed=synth.SEED + 2, ranks=[rank])[0]
    n_syb = int(round(0.2 * n))
    e = gsx.Engine(1, device=local)
    e.set_peer_params(synth.bench_peer_params())
    e.set_topic_params(0, synth.spam_test_topic_params())
    th = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                        accept_px_threshold=0, opportunistic_graft_threshold=5)
    e.set_thresholds(th)
    e.load_overlay_shard(n, sh.node_lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
    E = sh.n_pairs
    e.synthesize_state(
        abi.SynthSpec(seed=synth.SEED + 2, now_ns=T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0,
                      imd_max_sybil=100.0, p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0,
                      p_disconnected=0.0, p_absent=0.0, expire_jitter_ns=4 * abi.SECOND, sybil_first_node=n - n_syb))
    e.set_app_scores(np.zeros(E))
    log(f"[bench] cfg5 shard nodes={sh.node_hi - sh.node_lo}/{n} pairs={E} in {time.time() - t:.1f}s")
    now = T0
    for _ in range(2):
        now += abi.SECOND
        e.refresh(now)
    e.sync()
    if dist is not None:
        dist.barrier()
    steps = max(1, args.steps)
    e.timing_begin(steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        now += abi.SECOND
        e.refresh(now)
    e.sync()
    el = reduce_scalar(time.perf_counter() - t0, dist, dev, "max")
    k_total, _, _, k_n = e.timing_end()
    recs = reduce_scalar(float(E) * steps, dist, dev, "sum")
    sc = e.scores()
    syb = sh.sybil[sh.col]
    below = np.count_nonzero(sc[syb] < th.graylist_threshold)
    out = {
        "metric": "peer-topic score updates/s",
        "value": recs / el,
        "peers": n,
        "sybil_fraction": 0.2,
        "sybils_per_ip": 50,
        "pairs_rank0": E,
        "ms_per_refresh": el / steps * 1e3,
        "kernel_avg_ms_rank0": k_total / max(1, k_n),
        "sybil_pairs_rank0": int(syb.sum()),
        "sybil_pairs_below_graylist_rank0": int(below),
        "honest_pairs_below_graylist_rank0": int(np.count_nonzero(sc[~syb] < th.graylist_threshold)),
    }
    if args.prop_msgs > 0:
        # invalid-message spam through the router: three quarters
        # of a batch published by sybils and rejected by validation (seen, not
        # forwarded, P4 to the sybil at every receiver), the rest honest
        M = args.prop_msgs
        k = np.arange(M)
        hsh = synth.h(synth.SEED + 3, synth.TAG_SRC, k, 0)
        spam = (hsh % np.uint64(4)) != 0
        n_hon = n - n_syb
        ms = np.zeros(M, dtype=abi.msg_dtype())
        ms["source"] = np.where(spam, n_hon + (hsh >> np.uint64(8)) % np.uint64(n_syb),
                                (hsh >> np.uint64(8)) % np.uint64(n_hon)).astype(np.uint32)
        ms["msg_id"] = (k + (1 << 40)).astype(np.uint64)
        ms["validation"] = np.where(spam, abi.GSX_VALIDATION_REJECT, abi.GSX_VALIDATION_ACCEPT).astype(np.uint32)
        cfg = prop_config(args, n)
        cfg.now_ns = now + abi.SECOND // 2
        e.set_prop_tracking(False)
        sp_runner = None
        if dist is not None:
            sp_runner = shard_mod.RangeSharded(e, rl, shard_mod.DistTransport(dev, stage_host=args.rehearse))
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if sp_runner is None:
            d = shard_mod.out_dict(e.propagate(ms, cfg)[0])
        else:
            d = sp_runner.propagate(ms, cfg)[1]
        e.settle_scores()  # (the batch's deferred re-scores, timed with it)
        e.sync()
        torch.cuda.synchronize(dev)
        out["spam"] = {
            "messages": M, "rejected_by_validation": int(spam.sum()),
            "ms_per_batch": reduce_scalar(time.perf_counter() - t0, dist, dev, "max") * 1e3,
            "deliveries": d["deliveries"], "rejected_receipts_p4": d["rejected"], "duplicates": d["duplicates"],
            "graylisted_copies": d["graylisted"],
        }
        now += abi.SECOND
        e.refresh(now)
        sc = e.scores()
        out["spam"]["sybil_pairs_below_graylist_after_rank0"] = int(np.count_nonzero(sc[syb] < th.graylist_threshold))
    if args.hb_steps > 0:
        # heartbeats over the shards: GRAFT/PRUNE words of cross-shard pairs
        # go to their receivers' ranks and the answers come back (gsx_hb_*)
        runner = None
        if dist is not None:
            runner = shard_mod.RangeSharded(e, rl, shard_mod.DistTransport(dev, stage_host=args.rehearse))

        # the heartbeat's buffers, allocated once at setup (gsx_hb_reserve: the router's
        # attach-time state), so the timed first round is the round's work
        e.hb_reserve()

        def sybil_links():
            st = e.export_state()
            return reduce_scalar(float(np.count_nonzero(((st["rec_flags"] & abi.GSX_REC_IN_MESH) != 0) & syb)),
                                 dist, dev, "sum")

        before = sybil_links()
        if dist is not None:
            dist.barrier()
        hbs, ms = [], []
        for k in range(2):  # the attack's first round (the synthesized meshes' sybils pruned), then round 60 (OG)
            now += abi.SECOND
            torch.cuda.synchronize(dev)
            b0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)  # (the profiler's clock: tools/hb_api.py windows)
            t0 = time.perf_counter()
            if runner is None:
                hbs.append(e.heartbeat(59 + k, now, synth.SEED).as_dict())
            else:
                hbs.append(runner.heartbeat(59 + k, now, synth.SEED)[1])
            e.sync()
            torch.cuda.synchronize(dev)
            ms.append(reduce_scalar(time.perf_counter() - t0, dist, dev, "max") * 1e3)
            if os.environ.get("GSX_HB_WINDOWS"):
                log(f"window {59 + k} {b0} {time.clock_gettime_ns(time.CLOCK_BOOTTIME)}")
        out["heartbeat_ms_per_round"] = sum(ms) / len(ms)
        out["heartbeat_ms_rounds"] = ms
        if runner is not None:  # the gossip exchange's forwarding hops across the shards and their host round trips
            out["forwarding_exchange"] = {"hops": runner.gx_hops,
                                          "host_syncs_per_hop": runner.gx_syncs / max(runner.gx_hops, 1)}
        out["sybil_mesh_links_before"] = int(before)
        out["sybil_mesh_links_after"] = int(sybil_links())
        out["heartbeat_first_round"] = hbs[0]
    e.close()
    return out


def dropin_leg(args):
    """tools/dropin_latency.cpp (built here with g++ against libgsx.so) in a child
    process: Score() / tracer-call / refreshScores() latency of a single router's
    peerScore on the engine, the per-call path a cgo shim takes."""
    import subprocess

    root = os.path.dirname(os.path.abspath(__file__))
    src = os.path.join(root, "tools", "dropin_latency.cpp")
    libdir = os.path.join(root, "go-libp2p-pubsub_amd", "gsx")
    exe = os.path.join(root, "tools", "dropin_latency")
    try:
        if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(src):
            subprocess.run(["g++", "-std=c++17", "-O2", src, f"-L{libdir}", "-lgsx", f"-Wl,-rpath,{libdir}", "-o", exe],
                           check=True, timeout=120)
        out = {}
        for k in (100, 1000, 10000):
            r = subprocess.run([exe, str(k), "2000"], capture_output=True, text=True, timeout=120, check=True)
            out[f"peers_{k}"] = json.loads(r.stdout.strip().splitlines()[-1])
        out["note"] = ("per call through include/gsx_pubsub.hpp on one GPU engine holding one router's peers; "
                       "Score() with no change since the last is a host lookup (AppSpecificScore is called for the "
                       "scored peer only, score.go:320) or of the host-mapped score copy; after a tracer call one "
                       "k_dropin launch applies the queued events and re-scores only the pairs and rows they touched, "
                       "writing the asked scores to the mapped copy")
        return out
    except (subprocess.SubprocessError, OSError, ValueError) as ex:
        return {"error": str(ex)[:300]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--peers", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=8)
    ap.add_argument("--degree", type=int, default=6)
    ap.add_argument("--cpu-passes", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-single-observer", dest="single_observer", action="store_false",
                    help="skip the one-observer-with-1M-peers view (SURVEY §8)")
    ap.add_argument("--prop-msgs", type=int, default=1024,
                    help="messages per propagation batch (0: skip); 1024 = 16 words, one 128-B line per frontier row")
    ap.add_argument("--prop-peers", type=int, default=10_000_000, help="cfg4 overlay for the range-sharded leg (0: skip)")
    ap.add_argument("--shard-msgs", type=int, default=64, help="messages per batch of the cfg4 range-sharded leg")
    ap.add_argument("--shard-exchange", choices=("compact", "dense"), default="compact",
                    help="cfg4 range-sharded leg: compacted entries (one host round trip per hop) or every cross "
                         "pair's row with fixed splits (one host check per --shard-chunk hops)")
    ap.add_argument("--shard-chunk", type=int, default=4, help="dense exchange: hops per host check")
    ap.add_argument("--prop-steps", type=int, default=5)
    ap.add_argument("--epoch-batches", type=int, default=4,
                    help="message-parallel leg: batches per heartbeat epoch (one credit all-reduce each)")
    ap.add_argument("--prop-hops", type=int, default=24)
    ap.add_argument("--hb-steps", type=int, default=5, help="timed heartbeat rounds (0: skip)")
    ap.add_argument("--hb-msgs", type=int, default=256, help="gossipsub messages propagated before every heartbeat")
    ap.add_argument("--no-hb-exchange", dest="hb_exchange", action="store_false",
                    help="heartbeats without the gossip exchange (IHAVEs emitted, not handled)")
    ap.add_argument("--hb-settle", type=int, default=8,
                    help="untimed heartbeat rounds before the timed ones (the synthesized meshes rebalance)")
    ap.add_argument("--adv-peers", type=int, default=4_000_000, help="cfg5 adversarial overlay (0: skip)")
    ap.add_argument("--no-dropin", dest="dropin", action="store_false",
                    help="skip the drop-in scorer latency leg (tools/dropin_latency.cpp)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 rehearsal on one GPU: all ranks on device 0, gloo (host-staged) instead of RCCL")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse:  # every rank on GPU 0, gloo through host memory: the multi-GPU flow on one card
        local = 0
        global REHEARSE
        REHEARSE = True
    if world != args.gpus:
        log(f"[bench] note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if args.rehearse else "nccl")
    dev = torch.device("cuda", local)

    n, T = args.peers, args.topics
    seed = synth.SEED + rank  # shard r: its own observers (range partition)
    ov, e = build_engine(n, T, args.degree, seed, local)
    E = ov.n_pairs
    R = E * T

    now = T0
    for _ in range(args.warmup):
        now += abi.SECOND
        e.refresh(now)
    e.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    torch.cuda.synchronize(dev)
    e.sync()
    e.timing_begin(max(1, args.steps))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        now += abi.SECOND
        e.refresh(now)
    e.sync()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    k_total, k_min, k_max, k_n = e.timing_end()

    recs = float(R) * args.steps
    elapsed = reduce_scalar(elapsed, dist, dev, "max")
    recs = reduce_scalar(recs, dist, dev, "sum")

    value = recs / elapsed
    kavg_ms = k_total / max(1, k_n)
    bytes_per_launch = BYTES_PER_RECORD * R + BYTES_PER_PAIR * E
    achieved = bytes_per_launch / (kavg_ms * 1e-3) / 1e9
    cfg_key = f"n={n},T={T},d={args.degree},E={E}"
    traffic = load_traffic(cfg_key)

    # ---- SURVEY §8 secondary view: one observer with 1M neighbours x T topics ----
    single_obs = single_observer_leg(args, local) if (args.single_observer and rank == 0) else None

    # ---- secondary: message deliveries/s (gossipsub mesh forwarding, A13-A14) ----
    prop = None
    if args.prop_msgs > 0:
        prop = {}
        th = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                            accept_px_threshold=0, opportunistic_graft_threshold=0)
        # (1) message-parallel replicas (weak): the 1M-peer overlay on every rank,
        #     prop_msgs messages per rank, credits all-reduced and folded
        prop["replica"] = prop_replica(args, rank, world, local, dist, dev, th)
        # (2) range-sharded cfg4 overlay (strong): --prop-peers nodes over all ranks
        if args.prop_peers > 0:
            prop["sharded"] = prop_sharded(args, rank, world, local, dist, dev, th)

    # ---- heartbeat rounds (A10): every (node, topic) mesh maintained at once ----
    hb = None
    if args.hb_steps > 0:
        # steady state: a gossipsub batch arrives before every heartbeat (untimed),
        # so every round's emitGossip advertises the cached windows (mcache).
        # The synthesized meshes (every pair in the mesh with p = 0.5) rebalance
        # over the first rounds (~3e7 grafts + prunes in the first): --hb-settle
        # untimed rounds (reported as settle_per_round), then the timed rounds
        # through the OpportunisticGraftTicks round 60 (the "active" round)
        th_hb = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300,
                               accept_px_threshold=0, opportunistic_graft_threshold=5)
        e.set_thresholds(th_hb)
        # the reference's HandleRPC always runs handleIHave / handleIWant
        # (gossipsub.go:596-613): the gossip exchange (D) is part of the round
        e.set_gossipsub_params(gsx_engine_mod.default_gossipsub_params(gossip_exchange=1 if args.hb_exchange else 0))
        e.hb_reserve()  # (setup: the heartbeat's buffers, gsx_hb_reserve)
        tick = 58 - args.hb_settle
        hb_cfg = prop_config(args, n)
        rounds, settle = [], []
        for k in range(args.hb_settle + args.hb_steps):
            tick += 1
            now += abi.SECOND
            hb_cfg.now_ns = now - abi.SECOND // 2
            e.propagate(prop_messages(n, args.hb_msgs, seed, first=50_000_000 + k * args.hb_msgs), hb_cfg)
            e.settle_scores()  # the batch's own (deferred) re-scores finish with it, outside the round
            e.sync()
            barrier()
            torch.cuda.synchronize(dev)
            b0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)  # (the profiler's clock: tools/hb_api.py windows)
            t0 = time.perf_counter()
            o = e.heartbeat(tick, now, seed).as_dict()
            e.sync()
            ms = (time.perf_counter() - t0) * 1e3
            if os.environ.get("GSX_HB_WINDOWS") and k >= args.hb_settle:
                log(f"window {tick} {b0} {time.clock_gettime_ns(time.CLOCK_BOOTTIME)}")
            ms = reduce_scalar(ms, dist, dev, "max")
            r = {"tick": tick, "og_tick": tick % 60 == 0, "ms": ms, **o}
            (rounds if k >= args.hb_settle else settle).append(r)
        units = float(n) * T
        deg = E / n
        d_hi = 12
        bpu = 21 * deg + 4 * d_hi  # 4*deg + 8*deg + 9*deg + 4*Dhi per (node, topic)
        active = [r for r in rounds if r["og_tick"]]
        steady = [r for r in rounds if not r["og_tick"]]
        mean = lambda xs: sum(xs) / len(xs) if xs else None  # noqa: E731
        steady_ms = mean([r["ms"] for r in steady])
        active_ms = mean([r["ms"] for r in active])
        tot_ms = sum(r["ms"] for r in rounds)

        def roof(ms_):
            if not ms_:
                return None
            ach = units * bpu / (ms_ * 1e-3) / 1e9
            return {"bound": "hbm", "bytes_per_round": units * bpu, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ach / HBM_PEAK_GBS, "timing": "wall clock of gsx_heartbeat incl. launches"}

        units_all = reduce_scalar(units * len(rounds), dist, dev, "sum")
        hb = {
            "metric": "heartbeat (node, topic) mesh units/s",
            "value": units_all / (tot_ms * 1e-3),
            "ms_per_round": tot_ms / len(rounds),
            "rounds": len(rounds),
            "messages_between_rounds": args.hb_msgs,
            "gossip_exchange": bool(args.hb_exchange),
            "iwant_msgs_per_round": mean([r["iwant_msgs"] for r in rounds]),
            "iwant_ids_per_round": mean([r["iwant_ids"] for r in rounds]),
            "gossip_delivered_per_round": mean([r["gossip_delivered"] for r in rounds]),
            "steady_ms_per_round": steady_ms,
            "active_ms_per_round": active_ms,
            "roofline_steady": with_traffic(roof(steady_ms),
                                            pmc_bytes("heartbeat_last_round", "hbm_bytes",
                                                      hb_workload(n, args.topics, args.hb_msgs, args.hb_exchange)),
                                            steady_ms),
            "roofline_active": roof(active_ms),
            "per_round": rounds,
            "settle_per_round": [{k: r[k] for k in ("tick", "ms", "grafts", "prunes")} for r in settle],
        }
        if rank == 0 and world == 1 and not args.no_cpu:
            hb["cpu_baseline"] = cpu_hb_baseline(args, local, seed)

    adv = adversarial_leg(args, rank, world, local, dist, dev) if args.adv_peers > 0 else None

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        o, st = cpu_baseline(e, T, now, args.cpu_passes)
        t = time.time()
        o.load_overlay(ov.row_ptr, ov.col, None, ov.node_ips)
        log(f"[bench] oracle loaded in {time.time() - t:.1f}s")
        threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)

        def cpu_leg(parallel):
            o.import_state(st)
            o.set_app_scores(np.zeros(E))
            secs, c_now, sc = 0.0, now, None
            for _ in range(args.cpu_passes):
                c_now += abi.SECOND
                t = time.perf_counter()
                if parallel:
                    sc = o.refresh_scores_parallel(c_now, threads)
                else:
                    o.refresh(c_now)
                    sc = o.scores()
                secs += time.perf_counter() - t
            return secs, sc

        cpu_s1, want1 = cpu_leg(False)
        cpu_sp, want = cpu_leg(True)
        # the GPU on the same starting state and clock
        e.import_state(st)
        g_now = now
        for _ in range(args.cpu_passes):
            g_now += abi.SECOND
            e.refresh(g_now)
        got = e.scores()
        bad = int(np.count_nonzero(got.view(np.uint64) != want.view(np.uint64)))
        bad1 = int(np.count_nonzero(want1.view(np.uint64) != want.view(np.uint64)))
        parity = "bit-exact" if bad == 0 and bad1 == 0 else f"MISMATCH in {bad} pairs (serial vs parallel oracle: {bad1})"
        cpu = {
            "value": R * args.cpu_passes / cpu_sp,
            "unit": "peer-topic score updates/s",
            "cores": threads,
            "kind": "port",
            "single_thread_value": R * args.cpu_passes / cpu_s1,
            "nproc": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "sample": f"the full cfg3 shard ({R} records, {E} pairs), {args.cpu_passes} refresh+score passes of the "
                      f"C oracle (oracle/gsx_oracle.c, gcc -O3, OpenMP over pairs with {threads} threads: "
                      f"{cpu_sp:.2f}s; 1 thread: {cpu_s1:.2f}s; restatement, not reference Go: no Go on the box)",
        }
        del o, st

    # ---- drop-in boundary: per-call latency of one router's scorer (gsx_pubsub.hpp) ----
    dropin = dropin_leg(args) if (rank == 0 and world == 1 and args.dropin) else None

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "peer-topic score updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded counter-based generator, BASELINE.md cfg3 initialisation)",
        "config": {
            "workload": "cfg3: 1M peers x 8 topics, full P1-P7 refreshScores()+score() per DecayInterval, "
                        "connectSome d=6 overlay, spam-test topic params",
            "peers_per_gpu": n,
            "topics": T,
            "pairs_per_gpu": E,
            "records_per_gpu": R,
            "parallelism": f"observers range-sharded, {world} shard(s), no exchange",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": "k_refresh_score",
            "kernel_avg_ms": kavg_ms,
            "kernel_min_ms": k_min,
            "kernel_max_ms": k_max,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            # on the bytes the kernel actually moves (PMC traffic: the meshTime
            # stream and unchanged zero counters are never stored)
            "achieved_traffic": (traffic / (kavg_ms * 1e-3) / 1e9) if traffic else None,
            "frac_traffic": (traffic / (kavg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
            # also against the achievable copy rate the microarch guide measures
            "frac_traffic_of_copy": (traffic / (kavg_ms * 1e-3) / 1e9 / HBM_COPY_GBS) if traffic else None,
        },
        "single_observer": single_obs,
        "cpu_baseline": cpu,
        "parity_vs_oracle": parity,
        "propagation": prop,
        "heartbeat": hb,
        "adversarial": adv,
        "dropin": dropin,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    e.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
