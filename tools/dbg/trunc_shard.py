"""Debug: the w2-T2-trunc20 shard exchange case, every node's cache compared per round."""
import sys, os
ROOT = os.path.dirname(os.path.abspath(__file__)) + "/../.."
for p in ("go-libp2p-pubsub_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import torch  # noqa
import gsx
import propagation_cases as pc
import gossip_cases as gc
import heartbeat_cases as hc
from gsx import abi, shard, synth
from test_gpu_shard import _params, _slice_state

world, invalid, T, max_ihave, m = 2, 0.0, 2, int(sys.argv[1]) if len(sys.argv) > 1 else 20, 24
n, d, seed = 1200, 6, 47
ov = pc.overlay(n, d, seed)
full = gsx.Engine(T)
app = pc.setup(full, ov, T, seed, mesh_degree=6)
gp = gc.params(max_ihave_length=max_ihave)
full.set_gossipsub_params(gp)
st0 = full.export_state()
E = ov.n_pairs
rank_lo = synth.shard_ranges(n, world)
engines = []
for k in range(world):
    lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
    sh = synth.shard_of(ov, lo, hi)
    a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
    e = gsx.Engine(T)
    _params(e, T)
    e.load_overlay_shard(n, lo, sh.row_ptr, sh.col, sh.edge_flags, sh.node_ips)
    e.import_state(_slice_state(st0, T, E, a, b))
    e.set_app_scores(app[a:b])
    e.set_gossipsub_params(gp)
    engines.append((e, a, b, lo, hi))
runners = shard.run_local(world, "cuda:0", lambda tp, e: shard.RangeSharded(e, rank_lo, tp), [(x[0],) for x in engines])
for k in range(6):
    tick, now = 1 + k, pc.T0 + (3 + k) * abi.SECOND
    print("=== single round", k, flush=True)
    want = full.heartbeat(tick, now, seed * 31 + 7).as_dict()
    full.sync()
    print("=== shards round", k, flush=True)
    res = shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.heartbeat(tick, now, seed * 31 + 7))[1],
                          [(r,) for r in runners])
    diff = {x: (res[0][1][x], want[x]) for x in want if res[0][1][x] != want[x]}
    print("round", k, "diff", diff, flush=True)
    nd = 0
    for (e, a, b, lo, hi) in engines:
        for v in range(lo, hi):
            for w in range(1, 6):
                x = sorted(e.mcache_ids(v - lo, abi.GSX_ANY_TOPIC, w).tolist())
                y = sorted(full.mcache_ids(v, abi.GSX_ANY_TOPIC, w).tolist())
                if x != y:
                    if nd < 10:
                        print("  node", v, "windows", w, "shard-only", sorted(set(x) - set(y))[:8], "full-only",
                              sorted(set(y) - set(x))[:8], "dups", len(x) - len(set(x)), len(y) - len(set(y)))
                    nd += 1
                    break
    print("  nodes differing", nd, flush=True)
    if diff:
        break
    cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, max_hops=2, latency_ms=5, seed=seed + k)
    cfg.now_ns = now + 100 * abi.MILLISECOND
    ms = pc.messages(n, m, seed + 1000 * k, invalid=invalid)
    full.propagate(ms, cfg)
    shard.run_local(world, "cuda:0", lambda tp, r: (setattr(r, "tp", tp), r.propagate(ms, cfg))[1], [(r,) for r in runners])
    full.refresh(now + 500 * abi.MILLISECOND)
    for (e, _, _, _, _) in engines:
        e.refresh(now + 500 * abi.MILLISECOND)
