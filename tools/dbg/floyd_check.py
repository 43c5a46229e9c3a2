"""Debug: replay exchange_run up to tick K on both backends; before tick K's
heartbeat, recompute in Python the truncated IHAVE digest of some pairs from
each backend's cache lists (Floyd, gsx.h) and compare with what each emitted."""
import json
import sys

import numpy as np

sys.path[:0] = ["go-libp2p-pubsub_amd", "oracle", "tests"]
import gossip_cases as gc  # noqa: E402
import heartbeat_cases as hc  # noqa: E402
import propagation_cases as pc  # noqa: E402
import gsx  # noqa: E402
import oracle as orc  # noqa: E402
from gsx import abi  # noqa: E402

M = (1 << 64) - 1


def smix(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def h4(seed, tag, a, b):
    return smix((seed + 0x9E3779B97F4A7C15 * (1 + smix(tag ^ smix(a ^ smix(b))))) & M)


class Rng:
    def __init__(s, seed, tag, vertex, base):
        s.seed, s.tag, s.vertex, s.base, s.k = seed, tag, vertex, base, 0

    def int31(s):
        x = h4(s.seed, s.tag, s.vertex, s.base | s.k) >> 33
        s.k += 1
        return x

    def int31n(s, n):
        if n & (n - 1) == 0:
            return s.int31() & (n - 1)
        mx = (1 << 31) - 1 - (1 << 31) % n
        v = s.int31()
        while v > mx:
            v = s.int31()
        return v % n


def floyd(L, k, g):
    sel = set()
    for j in range(L - k, L):
        x = g.int31n(j + 1)
        if x in sel:
            x = j
        sel.add(x)
    return sel


kw = json.loads(sys.argv[1])
SNAP = kw.pop("snap", False)
LISTS = kw.pop("lists", True)
ONLY = kw.pop("only", None)  # read the lists of these nodes only
K = int(sys.argv[2])
T = kw.get("T", 2)
n, d, seed, msgs, hops, invalid = 300, 6, 5, kw.get("msgs", 24), 2, kw.get("invalid", 0.0)
BES = [orc.Oracle(T)] if len(sys.argv) > 3 else [gsx.Engine(T), orc.Oracle(T)]
for be in BES:
    ov = pc.overlay(n, d, seed)
    pc.setup(be, ov, T, seed, mesh_degree=6)
    for k in range(K + 1):
        if k == 0:
            gp = gc.params(max_ihave_length=kw["max_ihave_length"])
            be.set_gossipsub_params(gp)
        now = hc.T0 + (3 + k) * abi.SECOND
        if k == K:
            lists = {v: [be.mcache_ids(v, t, 5) for t in range(T)] for v in (ONLY or range(n))} if LISTS else None
            if ONLY is not None:
                lists = None
        o = be.heartbeat(1 + k, now, seed * 31 + 7)
        if k == K:
            break
        if SNAP:
            hc.snapshot(be)
        cfg = pc.config(abi.GSX_ROUTER_GOSSIPSUB, topic=k % T, max_hops=hops, latency_ms=5, seed=seed + k)
        cfg.now_ns = now + 100 * abi.MILLISECOND
        be.propagate(pc.messages(n, msgs, seed + 1000 * k, invalid=invalid), cfg)
        be.refresh(now + 500 * abi.MILLISECOND)
    ln, dg = be.gossip_results()
    if lists is None:
        np.save(f"gpurun_out/dg_{type(be).__name__}.npy", dg)
        continue
    maxl = kw["max_ihave_length"]
    bad = tot = 0
    for v in range(n):
        for r in range(ov.row_ptr[v], ov.row_ptr[v + 1]):
            for t in range(T):
                if ln[t][r] == 0:
                    continue
                ids = lists[v][t]
                L = len(ids)
                if L <= maxl:
                    inc = list(range(L))
                else:
                    kk = min(maxl, L - maxl)
                    g = Rng(seed * 31 + 7, 13, (v << 32) | int(ov.col[r]), ((1 + K) << 32) | (t << 24))
                    sel = floyd(L, kk, g)
                    inc = [i for i in range(L) if (i in sel) == (kk == maxl)]
                if ln[t][r] != len(inc):
                    print(type(be).__name__, "len", r, t, ln[t][r], len(inc))
                dd = sum(smix((int(ids[i]) + 0x9E3779B97F4A7C15) & M) for i in inc) & M
                tot += 1
                if dd != int(dg[t][r]):
                    bad += 1
                    if bad <= 3:
                        print(type(be).__name__, "pair", r, "topic", t, "L", L, "kk", kk, "emitted", int(dg[t][r]), "python", dd)
    print(type(be).__name__, "truncated lists checked", tot, "mismatching", bad)

if not LISTS or ONLY is not None:
    a, b = np.load("gpurun_out/dg_Engine.npy"), np.load("gpurun_out/dg_Oracle.npy")
    print("digest mismatches without the list reads:", int((a != b).sum()))
