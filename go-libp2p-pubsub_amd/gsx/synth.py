"""Seeded synthetic workloads (BASELINE.md "Configs restated").

Every draw comes from the counter-based generator h(seed, tag, a, b), a
SplitMix64 finaliser over a mixed key, so the same inputs can be regenerated
bit-for-bit anywhere (numpy here, C/Go/HIP elsewhere).  Nothing here is part
of the scoring path; it only builds inputs.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from . import abi

SEED = 0x9E3779B97F4A7C15
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)

# stream tags
TAG_OVL = 1
TAG_OVL_REDRAW = 2
TAG_SRC = 3
TAG_STATE = 4
TAG_IP = 5
TAG_EVENT = 6
TAG_VICTIM = 9


def _mix(z: np.ndarray) -> np.ndarray:
    """SplitMix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def h(seed: int, tag: int, a, b) -> np.ndarray:
    """h(seed, tag, a, b) = mix(seed + golden * (1 + mix(tag ^ mix(a ^ mix(b)))))."""
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    with np.errstate(over="ignore"):
        inner = _mix(np.uint64(tag) ^ _mix(a ^ _mix(b)))
        return _mix(np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (np.uint64(1) + inner))


def uniform(seed, tag, a, b) -> np.ndarray:
    """U[0,1) doubles from the top 53 bits."""
    return (h(seed, tag, a, b) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


@dataclass
class Overlay:
    n: int
    row_ptr: np.ndarray  # int64 [n+1]
    col: np.ndarray  # int32 [E]
    edge_flags: np.ndarray  # uint8 [E]
    node_ips: np.ndarray  # uint32 [n, 2]
    sybil: np.ndarray  # bool [n]

    @property
    def n_pairs(self) -> int:
        return int(self.row_ptr[-1])

    def pair_observer(self) -> np.ndarray:
        return np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self.row_ptr))


def _connect_some_keys(n: int, d: int, seed: int):
    """Sorted undirected connection keys lo*n+hi and sorted dial keys
    dialer*n+target of connectSome (floodsub_test.go:73-87): node i dials d
    targets h(seed, OVL, i, k) mod n, a self draw is redrawn once (then i+1);
    duplicate connections collapse."""
    i = np.repeat(np.arange(n, dtype=np.uint64), d)
    k = np.tile(np.arange(d, dtype=np.uint64), n)
    j = h(seed, TAG_OVL, i, k) % np.uint64(n)
    del k
    self_ = j == i
    if self_.any():
        j2 = h(seed, TAG_OVL_REDRAW, i[self_], np.nonzero(self_)[0].astype(np.uint64) % np.uint64(d)) % np.uint64(n)
        j2 = np.where(j2 == i[self_], (i[self_] + np.uint64(1)) % np.uint64(n), j2)
        j[self_] = j2
    i = i.astype(np.int64)
    j = j.astype(np.int64)
    dial_key = np.unique(i * n + j)  # (dialer, target)
    und = np.unique(np.minimum(i, j) * n + np.maximum(i, j))
    return und, dial_key


def _rows(n, und, dial_key, lo, hi, flags):
    """CSR rows lo..hi-1 (col = global ids, ascending) of the undirected keys;
    the dialer's pair is outbound."""
    a = und // n
    b = und % n
    m1 = (a >= lo) & (a < hi)
    m2 = (b >= lo) & (b < hi)
    key = np.concatenate([und[m1], b[m2] * n + a[m2]])
    key.sort()
    src = key // n
    dst = key % n
    row_ptr = np.zeros(hi - lo + 1, dtype=np.int64)
    np.cumsum(np.bincount(src - lo, minlength=hi - lo), out=row_ptr[1:])
    pos = np.searchsorted(dial_key, key)
    pos = np.minimum(pos, len(dial_key) - 1)
    outbound = dial_key[pos] == key
    ef = np.full(len(key), flags, dtype=np.uint8)
    ef[outbound] |= abi.GSX_EDGE_OUTBOUND
    return row_ptr, dst.astype(np.int32), ef


def _ips(n, sybil_frac, sybils_per_ip):
    """One unique IPv4 per honest node; the last sybil_frac*n nodes are
    sybils sharing one IP per sybils_per_ip."""
    sybil = np.zeros(n, dtype=bool)
    n_syb = int(round(sybil_frac * n))
    if n_syb:
        sybil[n - n_syb :] = True
    ips = np.full((n, 2), abi.GSX_NO_IP, dtype=np.uint32)
    ips[:, 0] = np.arange(n, dtype=np.uint32)
    if n_syb:
        sid = np.arange(n_syb, dtype=np.int64) // sybils_per_ip
        ips[n - n_syb :, 0] = (n + sid).astype(np.uint32)
    return ips, sybil


def _adversarial_keys(n: int, d: int, seed: int, sybil_frac: float, sybils_per_ip: int, victims: int):
    """honest nodes dial like connectSome over all n nodes;
    the sybils (the last sybil_frac*n nodes, sybils_per_ip of them per IP)
    attack in IP groups: every sybil of group g dials the same `victims`
    honest nodes h(seed, VICTIM, g, k) mod n_honest, so each victim sees a
    whole group on one IP (P6, score.go:337-381)."""
    n_syb = int(round(sybil_frac * n))
    n_h = n - n_syb
    i = np.repeat(np.arange(n_h, dtype=np.uint64), d)
    k = np.tile(np.arange(d, dtype=np.uint64), n_h)
    j = h(seed, TAG_OVL, i, k) % np.uint64(n)
    self_ = j == i
    j[self_] = (i[self_] + np.uint64(1)) % np.uint64(n)
    si = np.repeat(np.arange(n_h, n, dtype=np.uint64), victims)
    grp = (si - np.uint64(n_h)) // np.uint64(sybils_per_ip)
    kk = np.tile(np.arange(victims, dtype=np.uint64), n_syb)
    sj = h(seed, TAG_VICTIM, grp, kk) % np.uint64(max(n_h, 1))
    i = np.concatenate([i, si]).astype(np.int64)
    j = np.concatenate([j, sj]).astype(np.int64)
    dial_key = np.unique(i * n + j)
    und = np.unique(np.minimum(i, j) * n + np.maximum(i, j))
    return und, dial_key


def adversarial_overlay(n: int, d: int = 6, seed: int = SEED, sybil_frac: float = 0.2, sybils_per_ip: int = 50,
                        victims: int = 6, flags: int = abi.GSX_EDGE_GOSSIPSUB) -> Overlay:
    """cfg5 overlay (see _adversarial_keys); IPs as in connect_some_overlay."""
    und, dial_key = _adversarial_keys(n, d, seed, sybil_frac, sybils_per_ip, victims)
    row_ptr, col, ef = _rows(n, und, dial_key, 0, n, flags)
    ips, sybil = _ips(n, sybil_frac, sybils_per_ip)
    return Overlay(n, row_ptr, col, ef, ips, sybil)


def adversarial_shards(n: int, rank_lo, d: int = 6, seed: int = SEED, sybil_frac: float = 0.2,
                       sybils_per_ip: int = 50, victims: int = 6, flags: int = abi.GSX_EDGE_GOSSIPSUB, ranks=None):
    und, dial_key = _adversarial_keys(n, d, seed, sybil_frac, sybils_per_ip, victims)
    ips, sybil = _ips(n, sybil_frac, sybils_per_ip)
    out = []
    for k in range(len(rank_lo) - 1) if ranks is None else ranks:
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        row_ptr, col, ef = _rows(n, und, dial_key, lo, hi, flags)
        out.append(OverlayShard(n, lo, hi, row_ptr, col, ef, ips, sybil))
    return out


def connect_some_overlay(
    n: int, d: int = 6, seed: int = SEED, sybil_frac: float = 0.0, sybils_per_ip: int = 50, flags: int = abi.GSX_EDGE_GOSSIPSUB
) -> Overlay:
    """connectSome-style random overlay (floodsub_test.go:73-87): node i dials d
    targets h(seed, OVL, i, k) mod n, a self draw is redrawn once (then i+1);
    duplicate connections collapse; both ends get a pair; the dialer's pair is
    outbound."""
    und, dial_key = _connect_some_keys(n, d, seed)
    row_ptr, col, ef = _rows(n, und, dial_key, 0, n, flags)
    ips, sybil = _ips(n, sybil_frac, sybils_per_ip)
    return Overlay(n, row_ptr, col, ef, ips, sybil)


@dataclass
class OverlayShard:
    """Rows node_lo .. node_hi-1 of an n-node overlay (col = global ids)."""
    n: int
    node_lo: int
    node_hi: int
    row_ptr: np.ndarray
    col: np.ndarray
    edge_flags: np.ndarray
    node_ips: np.ndarray  # all n nodes
    sybil: np.ndarray  # all n nodes

    @property
    def n_pairs(self) -> int:
        return int(self.row_ptr[-1])


def shard_ranges(n: int, world: int) -> np.ndarray:
    """Balanced contiguous node ranges: rank k owns rank_lo[k] .. rank_lo[k+1]-1."""
    return np.array([(n * k) // world for k in range(world + 1)], dtype=np.uint32)


def connect_some_shards(n: int, rank_lo, d: int = 6, seed: int = SEED, sybil_frac: float = 0.0,
                        sybils_per_ip: int = 50, flags: int = abi.GSX_EDGE_GOSSIPSUB, ranks=None):
    """The shards (for `ranks`, default all) of connect_some_overlay(n, ...):
    the connection draw is global, each shard keeps its rows."""
    und, dial_key = _connect_some_keys(n, d, seed)
    ips, sybil = _ips(n, sybil_frac, sybils_per_ip)
    out = []
    for k in range(len(rank_lo) - 1) if ranks is None else ranks:
        lo, hi = int(rank_lo[k]), int(rank_lo[k + 1])
        row_ptr, col, ef = _rows(n, und, dial_key, lo, hi, flags)
        out.append(OverlayShard(n, lo, hi, row_ptr, col, ef, ips, sybil))
    return out


def shard_of(ov: Overlay, lo: int, hi: int) -> OverlayShard:
    """Rows lo..hi-1 of an existing overlay."""
    a, b = int(ov.row_ptr[lo]), int(ov.row_ptr[hi])
    return OverlayShard(ov.n, lo, hi, ov.row_ptr[lo : hi + 1] - a, ov.col[a:b].copy(), ov.edge_flags[a:b].copy(),
                        ov.node_ips, ov.sybil)


def spam_test_topic_params() -> abi.TopicScoreParams:
    """Topic params of TestGossipsubAttackInvalidMessageSpam (gossipsub_spam_test.go:636-654)."""
    S = abi.SECOND
    return abi.TopicScoreParams(
        topic_weight=0.25,
        time_in_mesh_weight=0.0027,
        time_in_mesh_quantum_ns=S,
        time_in_mesh_cap=3600,
        first_message_deliveries_weight=0.664,
        first_message_deliveries_decay=0.9916,
        first_message_deliveries_cap=1500,
        mesh_message_deliveries_weight=-0.25,
        mesh_message_deliveries_decay=0.97,
        mesh_message_deliveries_cap=400,
        mesh_message_deliveries_threshold=100,
        mesh_message_deliveries_activation_ns=30 * S,
        mesh_message_deliveries_window_ns=5 * abi.MINUTE,
        mesh_failure_penalty_weight=-0.25,
        mesh_failure_penalty_decay=0.997,
        invalid_message_deliveries_weight=-99,
        invalid_message_deliveries_decay=0.9994,
    )


def bench_peer_params() -> abi.PeerScoreParams:
    """cfg3 global params: TopicScoreCap 100, AppWeight 1,
    P6 weight -10 threshold 1, P7 weight -10 threshold 0 decay
    ScoreParameterDecay(10 min), DecayInterval 1 s, DecayToZero 0.01."""
    # ScoreParameterDecay(10 min) = 0.01 ** (1/600), computed by the engine's twin
    # of score_params.go:282-287 at run time where the library is loaded; the
    # closed form here is the same expression.
    d7 = 0.01 ** (1.0 / 600.0)
    return abi.PeerScoreParams(
        topic_score_cap=100.0,
        app_specific_weight=1.0,
        app_specific_score_set=1,
        ip_colocation_factor_threshold=1,
        ip_colocation_factor_weight=-10.0,
        behaviour_penalty_weight=-10.0,
        behaviour_penalty_threshold=0.0,
        behaviour_penalty_decay=d7,
        decay_interval_ns=abi.SECOND,
        decay_to_zero=0.01,
        retain_score_ns=10 * abi.SECOND,
    )


def synthetic_state(ov: Overlay, n_topics: int, now_ns: int, seed: int = SEED, p_disconnected: float = 0.0,
                    p_absent: float = 0.0) -> Dict[str, np.ndarray]:
    """Counter initialisation of BASELINE.md cfg3: fmd~U[0,1500), mmd~U[0,400),
    mfp~U[0,50), imd=0 honest / U[0,100) for pairs whose peer is a sybil,
    inMesh~Bern(0.5), graftTime=now-U[0,2h), bp~U[0,5).  Optional fractions of
    retained (disconnected) and absent pairs exercise the purge path."""
    E = ov.n_pairs
    R = n_topics * E
    r = np.arange(R, dtype=np.uint64)
    p = np.arange(E, dtype=np.uint64)
    st: Dict[str, np.ndarray] = {}
    st["first_message_deliveries"] = uniform(seed, TAG_STATE, r, 1) * 1500.0
    st["mesh_message_deliveries"] = uniform(seed, TAG_STATE, r, 2) * 400.0
    st["mesh_failure_penalty"] = uniform(seed, TAG_STATE, r, 3) * 50.0
    syb_pair = np.tile(ov.sybil[ov.col], n_topics)
    imd = uniform(seed, TAG_STATE, r, 4) * 100.0
    st["invalid_message_deliveries"] = np.where(syb_pair, imd, 0.0)
    in_mesh = uniform(seed, TAG_STATE, r, 5) < 0.5
    graft = now_ns - (uniform(seed, TAG_STATE, r, 6) * float(2 * abi.HOUR)).astype(np.int64)
    st["graft_time_ns"] = graft
    st["mesh_time_ns"] = np.where(in_mesh, now_ns - graft, 0).astype(np.int64)
    st["rec_flags"] = np.where(in_mesh, abi.GSX_REC_IN_MESH, 0).astype(np.uint8)
    pf = np.full(E, abi.GSX_PAIR_PRESENT | abi.GSX_PAIR_CONNECTED, dtype=np.uint8)
    if p_disconnected > 0:
        u = uniform(seed, TAG_STATE, p, 7)
        pf[u < p_disconnected] = abi.GSX_PAIR_PRESENT
    if p_absent > 0:
        u = uniform(seed, TAG_STATE, p, 8)
        pf[u < p_absent] = 0
    st["pair_flags"] = pf
    # retained pairs: expiry within now +- 2 s (half expire at the first refresh)
    st["expire_ns"] = now_ns + ((uniform(seed, TAG_STATE, p, 9) - 0.5) * float(4 * abi.SECOND)).astype(np.int64)
    st["behaviour_penalty"] = uniform(seed, TAG_STATE, p, 10) * 5.0
    st["last_refresh_ns"] = now_ns  # meshTime above is what a refresh at `now` wrote
    return st
