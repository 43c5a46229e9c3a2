#!/usr/bin/env python3
"""Range-sharded cfg4 propagation (BASELINE.json configs[3]) in N shards on ONE
GPU: what each rank of an N-GPU node would spend in hop kernels.

Every shard is an engine of its own (gsx_load_overlay_shard) driven by
gsx.shard.RangeSharded over the in-process LocalTransport in serial mode: the
shards take turns between collectives and each turn is drained before the next
starts, so a shard's hop kernels never overlap another's on the shared device
and the per-shard HIP-event hop times (gsx_prop_out.hop_kernel_ms) are those
of a GPU running that shard alone.  The exchange itself goes through device
copies here, not xGMI: its bytes and host round trips are reported, its time
is not.  The single engine holding the whole overlay runs the same batches
first; every shard count must reproduce its totals (deliveries, duplicates,
per-hop deliveries, graylisted copies) exactly.

    python tools/shard_scaling.py [--peers 10000000] [--shards 1,2,4,8] [--batches 3]

Prints one JSON line per shard count (and the single engine as shards=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (before libgsx: torch's HIP runtime must be the process's first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-libp2p-pubsub_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import gsx  # noqa: E402
from gsx import abi, synth  # noqa: E402
from gsx import engine as gsx_engine_mod  # noqa: E402
from gsx import shard as shard_mod  # noqa: E402

TH = abi.Thresholds(gossip_threshold=-100, publish_threshold=-200, graylist_threshold=-300, accept_px_threshold=0,
                    opportunistic_graft_threshold=0)


def engine_for(n, sh, seed, full=None, state=None):
    """bench.prop_engine's setup on the whole overlay (full), or on a shard
    holding `state`, its slice of the single engine's exported state."""
    e = gsx.Engine(1, device=0)
    e.set_peer_params(synth.bench_peer_params())
    e.set_topic_params(0, synth.spam_test_topic_params())
    e.set_thresholds(TH)
    if full is not None:
        e.load_overlay(full.row_ptr, full.col, full.edge_flags, full.node_ips)
        e.synthesize_state(
            abi.SynthSpec(seed=seed, now_ns=bench.T0, fmd_max=1500.0, mmd_max=400.0, mfp_max=50.0,
                          imd_max_sybil=100.0, p_in_mesh=0.5, graft_window_ns=2 * abi.HOUR, bp_max=5.0,
                          p_disconnected=0.0, p_absent=0.0, expire_jitter_ns=4 * abi.SECOND, sybil_first_node=n))
        e.set_app_scores(np.zeros(full.n_pairs))
        e.refresh(bench.T0 + abi.SECOND)
    else:
        e.load_overlay_shard(n, sh.node_lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
        e.import_state(state)
        e.set_app_scores(np.zeros(sh.n_pairs))
    e.set_gossipsub_params(gsx_engine_mod.default_gossipsub_params(gossip_exchange=0))
    e.set_prop_tracking(False)
    e.sync()
    return e


def state_slice(st, a, b):
    """Pairs a..b-1 of a T = 1 state (tests/test_gpu_configs.py does the same)."""
    out = {f: st[f][a:b].copy() for f in abi.STATE_FIELDS}
    out["last_refresh_ns"] = st["last_refresh_ns"]
    return out


def config(max_hops):
    return abi.PropConfig(router=abi.GSX_ROUTER_GOSSIPSUB, topic=0, flood_publish=0, max_hops=max_hops,
                          hop_latency_ns=10 * abi.MILLISECOND, now_ns=bench.T0 + 2 * abi.SECOND,
                          credit_scores=abi.GSX_CREDIT_NOW, randomsub_size=0, seed=synth.SEED)


KEYS = ("deliveries", "duplicates", "graylisted", "hops")


def norm(d):
    """The totals a shard count must reproduce (hop_deliveries up to the last delivering hop)."""
    out = {k: int(d[k]) for k in KEYS}
    out["hop_deliveries"] = [int(x) for x in list(d["hop_deliveries"])[: out["hops"] + 1]]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=10_000_000)
    ap.add_argument("--msgs", type=int, default=64)
    ap.add_argument("--shards", default="2,4,8")
    ap.add_argument("--batches", type=int, default=3, help="timed batches after one warm-up batch")
    ap.add_argument("--exchange", choices=("compact", "dense"), default="compact")
    ap.add_argument("--chunk", type=int, default=4)
    ap.add_argument("--max-hops", type=int, default=24)
    ap.add_argument("--no-single", dest="single", action="store_false")
    ap.add_argument("--pairs", action="store_true", help="the per-pair halo exchange (GSX_SHARD_PAIRS=1), not the "
                                                         "replicated frontier")
    args = ap.parse_args()
    if args.pairs:
        os.environ["GSX_SHARD_PAIRS"] = "1"
    n, seed = args.peers, synth.SEED + 1
    cfg = config(args.max_hops)
    batches = [bench.prop_messages(n, args.msgs, seed, first=b * args.msgs) for b in range(1 + args.batches)]

    ref = None
    t = time.time()
    ov = synth.connect_some_overlay(n, d=6, seed=seed)
    e = engine_for(n, None, seed, full=ov)
    st0 = e.export_state()  # the shards start from its slices
    row_ptr = ov.row_ptr.copy()
    del ov
    print(f"[scaling] single engine ready in {time.time() - t:.1f}s", file=sys.stderr, flush=True)
    if args.single:
        ref, kms = [], []
        for b, msgs in enumerate(batches):
            d = shard_mod.out_dict(e.propagate(msgs, cfg)[0])
            ref.append(norm(d))
            if b:
                kms.append(d["hop_kernel_ms"])
        print(json.dumps({"shards": 1, "peers": n, "msgs": args.msgs, "hop_kernel_ms_per_batch": float(np.mean(kms)),
                          "per_batch": ref[1:]}), flush=True)
    e.close()

    for world in [int(x) for x in args.shards.split(",") if x]:
        t = time.time()
        rl = synth.shard_ranges(n, world)
        shs = synth.connect_some_shards(n, rl, d=6, seed=seed)
        engines = [engine_for(n, sh, seed, state=state_slice(st0, int(row_ptr[sh.node_lo]), int(row_ptr[sh.node_hi])))
                   for sh in shs]
        del shs
        print(f"[scaling] {world} shards ready in {time.time() - t:.1f}s", file=sys.stderr, flush=True)

        def run(tp, e):
            rs = shard_mod.RangeSharded(e, rl, tp, compact=args.exchange == "compact", chunk=args.chunk)
            outs = []
            for msgs in batches:
                loc, tot = rs.propagate(msgs, cfg)
                outs.append((loc["hop_kernel_ms"], tot, loc["hop_launches"]))
            return outs, rs.sent_bytes, rs.hops_run, rs.host_syncs, rs.n_send, rs.last_mode

        t = time.time()
        res = shard_mod.run_local(world, "cuda:0", run, [(e,) for e in engines], serial=True)
        wall = time.time() - t
        for e in engines:
            e.close()
        per_rank_ms = np.array([[o[0] for o in r[0][1:]] for r in res])  # [rank][batch]
        tots = [o[1] for o in res[0][0]]
        ok = None
        if ref is not None:
            ok = all(norm(tots[b]) == ref[b] for b in range(len(batches)))
        nb = len(batches)
        print(json.dumps({
            "shards": world, "peers": n, "msgs": args.msgs, "exchange": args.exchange, "mode": res[0][5],
            "hop_kernel_ms_per_batch_max_rank": float(per_rank_ms.max(0).mean()),
            "hop_kernel_ms_per_batch_per_rank": [float(x) for x in per_rank_ms.mean(1)],
            "hop_kernel_ms_per_batch_sum_ranks": float(per_rank_ms.sum(0).mean()),
            "equals_single_engine": ok,
            "bytes_sent_per_batch_max_rank": max(r[1] for r in res) / nb,
            "dense_bytes_per_hop_max_rank": max(r[4] for r in res) * shard_mod.prop_words(args.msgs) * 8,
            "hops_per_batch": res[0][2] / nb,
            "host_syncs_per_hop": res[0][3] / max(res[0][2], 1),
            "wall_s_one_gpu": wall,
            "per_batch": [norm(tots[b]) for b in range(1, nb)],
        }), flush=True)
        del engines, res


if __name__ == "__main__":
    main()
