"""CPU stand-in for one range shard of the engine's stepped propagation
(gsx.h "range sharding": gsx_shard_recv_plan / send_plan, gsx_prop_begin /
pack / step / end), TEST INFRASTRUCTURE ONLY.

It restates the split of a hop into the sender-side pack (eligibility, the
`from` exclusion) and the receiver-side merge (origin exclusion, lowest
sender first) in plain Python over numpy words, so that the multi-process
driver (gsx/shard.py) can be run over gloo on CPU and its stitched result
compared with the global oracle (oracle/gsx_oracle.c: orc_propagate).  The
GPU tests run the same driver over the HIP engine.
"""
from __future__ import annotations

import numpy as np

from gsx import abi
from gsx.shard import prop_words

M64 = (1 << 64) - 1
FWD, PUB = 1, 2
GIN = 8  # the pair's observer drops its neighbour's RPCs (gossipsub AcceptFrom, graylist)


def fwd_bytes(router, state, scores, edge_flags, topic, n_topics, publish_threshold, flood_publish,
              graylist_threshold=float("-inf")):
    """fwd[r] of every pair (v -> u) (gsx_propagate.hip k_prop_fwd) from an exported state."""
    E = len(edge_flags)
    pf = state["pair_flags"]
    inn = (pf & (abi.GSX_PAIR_PRESENT | abi.GSX_PAIR_CONNECTED)) == (abi.GSX_PAIR_PRESENT | abi.GSX_PAIR_CONNECTED)
    out = np.zeros(E, dtype=np.uint8)
    if router == abi.GSX_ROUTER_FLOODSUB:
        out[inn] = FWD | PUB
        return out
    assert router == abi.GSX_ROUTER_GOSSIPSUB
    direct = (edge_flags & abi.GSX_EDGE_DIRECT) != 0
    above = scores >= publish_threshold
    fwd = direct | (((edge_flags & abi.GSX_EDGE_GOSSIPSUB) == 0) & above)
    mesh = (state["rec_flags"].reshape(n_topics, E)[topic] & abi.GSX_REC_IN_MESH) != 0
    fwd = fwd | mesh
    pub = (direct | above) if flood_publish else fwd
    out = np.where(fwd, FWD, 0) | np.where(pub, PUB, 0)
    out = np.where(inn, out, 0)
    gin = ~direct & (scores < graylist_threshold)  # gossipsub.go:583-594
    return (out | np.where(gin, GIN, 0)).astype(np.uint8)


def _elig(fw, own):
    m = fw & 3
    if m == 3:
        return M64
    if m == FWD:
        return ~own & M64
    if m == PUB:
        return own
    return 0


class EmuShard:
    def __init__(self, shard, fwd_local):
        self.sh = shard
        self.lo = shard.node_lo
        self.n = shard.node_hi - shard.node_lo
        self.row_ptr = shard.row_ptr
        self.col = shard.col.astype(np.int64)
        self.fwd = fwd_local
        self.obs = np.repeat(np.arange(self.n), np.diff(self.row_ptr))
        E = len(self.col)
        self.rev = [None] * E  # ("local", r) | ("halo", slot) | None
        for q in range(E):
            v = int(self.col[q])
            if self.lo <= v < self.lo + self.n:
                lv = v - self.lo
                row = self.col[self.row_ptr[lv] : self.row_ptr[lv + 1]]
                i = np.searchsorted(row, self.obs[q] + self.lo)
                if i < len(row) and row[i] == self.obs[q] + self.lo:
                    self.rev[q] = ("local", int(self.row_ptr[lv] + i))

    def _find(self, lv, u):
        row = self.col[self.row_ptr[lv] : self.row_ptr[lv + 1]]
        i = np.searchsorted(row, u)
        return int(self.row_ptr[lv] + i) if i < len(row) and row[i] == u else None

    # -- plan ---------------------------------------------------------------------
    def shard_recv_plan(self, rank_lo):
        rank_lo = np.asarray(rank_lo, dtype=np.int64)
        self.rank_lo = rank_lo
        world = len(rank_lo) - 1
        owner = np.searchsorted(rank_lo, self.col, side="right") - 1
        remote = (self.col < self.lo) | (self.col >= self.lo + self.n)
        counts = np.zeros(world, dtype=np.uint64)
        ru, rv = [], []
        slot = 0
        for k in range(world):
            for q in np.nonzero(remote & (owner == k))[0]:
                self.rev[q] = ("halo", slot)
                ru.append(self.obs[q] + self.lo)
                rv.append(self.col[q])
                slot += 1
            counts[k] = int((remote & (owner == k)).sum())
        return counts, np.array(ru, dtype=np.uint32), np.array(rv, dtype=np.uint32)

    def shard_send_plan(self, send_counts, req_u, req_v):
        self.send_pair = [self._find(int(v) - self.lo, int(u)) for u, v in zip(req_u, req_v)]
        self.send_counts = np.asarray(send_counts, dtype=np.int64)
        self.send_base = np.concatenate([[0], np.cumsum(self.send_counts)])
        self.n_recv = sum(1 for r in self.rev if r is not None and r[0] == "halo")

    def shard_set_halo_bases(self, bases):
        self.halo_base = np.asarray(bases, dtype=np.int64)

    # -- stepped heartbeat: exchange plumbing only ---------------------------------------
    # The control words a pair carries are stand-ins naming the pair
    # ((sender << 32 | receiver) for GRAFT, its complement for PRUNE, the
    # answer as (receiver << 32 | sender)); hb_recv / hb_end check that every
    # receive slot got exactly the words of its pair's reverse.
    def _pair_ids(self, r):
        return int(self.obs[r]) + self.lo, int(self.col[r])

    def hb_begin(self, tick, now, seed):
        self.hb_checked = 0

    def hb_pack_ctl(self, send):
        a = np.zeros((len(self.send_pair), 2), dtype=np.uint64)
        for j, r in enumerate(self.send_pair):
            if r is not None:
                v, u = self._pair_ids(r)
                a[j] = (v << 32 | u, ~(v << 32 | u) & M64)
        send[: len(a)].copy_(_as_tensor(a.view(np.int64)))

    def _halo_pairs(self):
        for q, rv in enumerate(self.rev):
            if rv is not None and rv[0] == "halo":
                yield q, rv[1]

    def hb_recv(self, halo):
        h = halo.numpy().view(np.uint64)
        for q, slot in self._halo_pairs():
            u, v = self._pair_ids(q)
            assert int(h[slot, 0]) == (v << 32 | u) and int(h[slot, 1]) == (~(v << 32 | u) & M64), (q, slot)
            self.hb_checked += 1

    def hb_pack_resp(self, send):
        a = np.zeros(len(self.send_pair), dtype=np.uint64)
        for j, r in enumerate(self.send_pair):
            if r is not None:
                u, v = self._pair_ids(r)  # r = (u -> v) answers v's GRAFT
                a[j] = u << 32 | v
        send[: len(a)].copy_(_as_tensor(a.view(np.int64)))

    def hb_end(self, halo):
        h = halo.numpy().view(np.uint64)
        for r, slot in self._halo_pairs():
            v, u = self._pair_ids(r)  # r = (v -> u): u's answer to v
            assert int(h[slot]) == (u << 32 | v), (r, slot)
            self.hb_checked += 1
        out = abi.HeartbeatOut()
        out.mesh_links = self.hb_checked
        return out

    # -- the sharded gossip exchange (gsx_gx_*, gsx_gxf_*): plumbing only ---------------
    # With gx_sets set, hb_end leaves an exchange of that many message sets
    # pending.  Every stand-in word names its pair (or the rank), every
    # receive side checks it got exactly what its senders packed: the common
    # words (rank k clears bit k of word 0, so the AND clears bits 0..world-1),
    # IHAVE/answer words per cross pair, variable row entries for the send
    # slots with (7v + u) % 3 == 0, per-run fout words, and per-hop frontier
    # entries for the slots with (v + u + hop + run) even; run k forwards for
    # exactly 2 + k hops (the frontier count is 0 from then on), the got flags
    # of rank k mark set k % n_sets.
    gx_sets = None
    gx_runs = 2

    def _rank(self):
        return int(np.searchsorted(self.rank_lo, self.lo, side="right") - 1)

    def gx_pending(self):
        return self.gx_sets

    def gx_common(self, n_sets):
        assert n_sets == self.gx_sets
        c = np.full(64 * n_sets, M64, dtype=np.uint64)
        if n_sets:
            c[0] = np.uint64(M64 & ~(1 << self._rank()))
        return c

    def gx_set_common(self, c):
        world = len(self.rank_lo) - 1
        assert len(c) == 64 * self.gx_sets
        if self.gx_sets:
            assert int(c[0]) == M64 & ~((1 << world) - 1) and all(int(x) == M64 for x in c[1:])
        self.hb_checked += 1

    def _send_ids(self):
        for j, r in enumerate(self.send_pair):
            if r is not None:
                v, u = self._pair_ids(r)
                yield j, v, u

    def gx_pack_ihave(self, send):
        a = np.zeros((len(self.send_pair), 2), dtype=np.uint64)
        for j, v, u in self._send_ids():
            a[j] = ((v << 32 | u) ^ 0x1111, u << 32 | v)
        send[: len(a)].copy_(_as_tensor(a.view(np.int64)))

    def gx_recv_ihave(self, recv):
        h = recv.numpy().view(np.uint64)
        for q, slot in self._halo_pairs():
            u, v = self._pair_ids(q)
            assert int(h[slot, 0]) == (v << 32 | u) ^ 0x1111 and int(h[slot, 1]) == (u << 32 | v), (q, slot)
            self.hb_checked += 1

    def _entries(self, keep, words, out):
        cnt = np.zeros(len(self.send_counts), dtype=np.uint64)
        rows = []
        for d in range(len(self.send_counts)):
            for j in range(int(self.send_base[d]), int(self.send_base[d + 1])):
                r = self.send_pair[j]
                if r is None:
                    continue
                v, u = self._pair_ids(r)
                if keep(v, u):
                    rows.append([int(self.halo_base[d] + j - self.send_base[d])] + words(v, u))
                    cnt[d] += 1
        if out is not None and rows:
            out[: len(rows)].copy_(_as_tensor(np.array(rows, dtype=np.uint64).view(np.int64)))
        return cnt

    def _check_entries(self, entries, n, keep, words):
        e = entries[:n].numpy().view(np.uint64)
        want = {slot: q for q, slot in self._halo_pairs()}
        seen = set()
        for row in e:
            slot = int(row[0])
            u, v = self._pair_ids(want[slot])
            assert keep(v, u) and [int(x) for x in row[1:]] == words(v, u), (slot, row)
            assert slot not in seen
            seen.add(slot)
        assert seen == {s for s, q in want.items() if keep(*self._pair_ids(q)[::-1])}
        return len(seen)

    @staticmethod
    def _row_keep(v, u):
        return (7 * v + u) % 3 == 0

    def gx_rows_words(self):
        return 3

    def gx_rows_pack(self, n_ranks, out=None):
        return self._entries(self._row_keep, lambda v, u: [v << 32 | u, 0xABC], out)

    def gx_rows_recv(self, entries, n):
        self.gx_rows = self._check_entries(entries, n, self._row_keep, lambda v, u: [v << 32 | u, 0xABC])

    def gx_exchange(self):
        self.gx_hops = []
        self.gx_fwd = 0
        return self.gx_runs

    def gxf_begin(self, run):
        assert run == len(self.gx_hops)
        self.gx_run = run
        self.gx_hops.append(0)

    def gxf_entry_words(self):
        return 4

    def gxf_pack_fout(self, send):
        a = np.zeros(len(self.send_pair), dtype=np.uint64)
        for j, v, u in self._send_ids():
            a[j] = (v << 32 | u) + self.gx_run
        send[: len(a)].copy_(_as_tensor(a.view(np.int64)))

    def gxf_recv_fout(self, recv):
        h = recv.numpy().view(np.uint64)
        for q, slot in self._halo_pairs():
            u, v = self._pair_ids(q)
            assert int(h[slot]) == (v << 32 | u) + self.gx_run, (q, slot)
            self.hb_checked += 1

    def _fwd_keep(self, hop):
        return lambda v, u: (v + u + hop + self.gx_run) % 2 == 0

    def gxf_pack(self, hop, n_ranks, out=None):
        return self._entries(self._fwd_keep(hop), lambda v, u: [v << 32 | u, hop, self.gx_run], out)

    def gxf_pack_dev(self, hop, out, d_counts):
        """gsx_gxf_pack_dev: destination d's entries from entry send_base[d] on, and
        (entries for rank d, this rank's frontier of hop - 1) per destination."""
        keep, words = self._fwd_keep(hop), (lambda v, u: [v << 32 | u, hop, self.gx_run])
        cnt = np.zeros(len(self.send_counts), dtype=np.int64)
        a = np.zeros((max(len(self.send_pair), 1), 4), dtype=np.uint64)
        for d in range(len(self.send_counts)):
            for j in range(int(self.send_base[d]), int(self.send_base[d + 1])):
                r = self.send_pair[j]
                if r is None:
                    continue
                v, u = self._pair_ids(r)
                if keep(v, u):
                    a[int(self.send_base[d]) + cnt[d]] = [int(self.halo_base[d] + j - self.send_base[d])] + words(v, u)
                    cnt[d] += 1
        out[: len(a)].copy_(_as_tensor(a.view(np.int64)))
        front = 1 if hop == 1 else (1 if hop - 1 < 2 + self.gx_run else 0)
        d_counts.copy_(_as_tensor(np.stack([cnt, np.full(len(cnt), front, dtype=np.int64)], 1)))

    def gxf_step(self, hop, entries, n, sync=True):
        assert hop == self.gx_hops[-1] + 1
        self.gx_hops[-1] = hop
        self.gx_fwd += self._check_entries(entries, n, self._fwd_keep(hop), lambda v, u: [v << 32 | u, hop, self.gx_run])
        f = 1 if hop < 2 + self.gx_run else 0
        return f if sync else None

    def gxf_end(self):
        assert self.gx_hops[-1] == 2 + self.gx_run

    def gx_got(self, n_sets):
        g = np.zeros(n_sets, dtype=np.uint8)
        if n_sets:
            g[self._rank() % n_sets] = 1
        return g

    def gx_end(self, got_all):
        world = len(self.rank_lo) - 1
        n = self.gx_sets
        want = np.zeros(n, dtype=np.uint8)
        for k in range(world):
            if n:
                want[k % n] = 1
        assert list(got_all) == list(want)
        assert len(self.gx_hops) == self.gx_runs
        out = abi.HeartbeatOut()
        out.mesh_links = self.hb_checked
        out.fwd_delivered = self.gx_fwd
        out.fwd_duplicates = sum(self.gx_hops)
        out.iwant_ids = self.gx_rows
        return out

    # -- stepped propagation ----------------------------------------------------------
    def prop_begin(self, msgs, cfg):
        self.cfg = cfg
        self.m = len(msgs)
        self.W = prop_words(self.m)
        n, E, W = self.n, len(self.col), self.W
        self.seen = [[0] * W for _ in range(n)]
        self.origin = [[0] * W for _ in range(n)]
        self.front = [[0] * W for _ in range(n)]
        self.frm = [[0] * W for _ in range(E)]
        self.hop = np.full((n, W * 64), 0xFF, dtype=np.uint8)
        self.h = 0
        self.stats = dict(deliveries=0, duplicates=0, graylisted=0, hop=[0] * (abi.GSX_MAX_HOPS + 1))
        for k, s in enumerate(msgs["source"]):
            s = int(s)
            if self.lo <= s < self.lo + n:
                u = s - self.lo
                b = 1 << (k % 64)
                self.origin[u][k // 64] |= b
                self.seen[u][k // 64] |= b
                self.front[u][k // 64] |= b
                self.hop[u, k] = 0

    def _send_row(self, r):
        v = int(self.obs[r])
        return [self.front[v][w] & _elig(int(self.fwd[r]), self.origin[v][w]) & ~self.frm[r][w] & M64
                for w in range(self.W)]

    def prop_pack(self, send):
        rows = [self._send_row(r) if r is not None else [0] * self.W for r in self.send_pair]
        a = np.array(rows, dtype=np.uint64).reshape(-1, self.W) if rows else np.zeros((0, self.W), np.uint64)
        send[: len(rows)].copy_(_as_tensor(a.view(np.int64)))

    def prop_pack_compact(self, out):
        """Entries [receive slot at the destination][row] of the non-empty rows,
        destination d's from entry send_base[d] on (gsx_prop_pack_compact)."""
        cnt = np.zeros(len(self.send_counts), dtype=np.uint64)
        rows = []
        for d in range(len(self.send_counts)):
            for j in range(int(self.send_base[d]), int(self.send_base[d + 1])):
                r = self.send_pair[j]
                row = self._send_row(r) if r is not None else [0] * self.W
                if any(row):
                    rows.append((int(self.send_base[d] + cnt[d]), [int(self.halo_base[d] + j - self.send_base[d])] + row))
                    cnt[d] += 1
        if rows:
            a = np.zeros((len(self.send_pair), self.W + 1), dtype=np.uint64)
            for pos, e in rows:
                a[pos] = e
            out[: len(a)].copy_(_as_tensor(a.view(np.int64)))
        return cnt

    def prop_pack_compact_dev(self, out, counts):
        """gsx_prop_pack_compact_dev: (entries for rank k, first receipts of the hop just run)."""
        cnt = self.prop_pack_compact(out)
        prev = self.stats["hop"][self.h] if self.h < len(self.stats["hop"]) else 0
        a = np.stack([cnt.astype(np.int64), np.full(len(cnt), prev, dtype=np.int64)], 1)
        counts.copy_(_as_tensor(a).reshape(counts.shape))

    def prop_step_compact(self, entries, n, sync=True):
        halo = np.zeros((max(self.n_recv, 1), self.W), dtype=np.uint64)
        e = entries[:n].numpy().view(np.uint64)
        for row in e:
            halo[int(row[0])] = row[1:]
        v = self._prop_step(_as_tensor(halo.view(np.int64)))
        return v if sync else None

    def prop_hop_counts_dev(self, out):
        """gsx_prop_hop_counts_dev: this rank's first receipts per hop."""
        out.copy_(_as_tensor(np.array(self.stats["hop"], dtype=np.int64)))

    def prop_step(self, recv, sync=True):
        v = self._prop_step(recv)
        return v if sync else None

    def _prop_step(self, recv):
        halo = recv.numpy().view(np.uint64) if len(recv) else None
        self.h += 1
        h, W = self.h, self.W
        nxt = [[0] * W for _ in range(self.n)]
        n_new = 0
        for u in range(self.n):
            for w in range(W):
                seen, mine, acc = self.seen[u][w], self.origin[u][w], 0
                for q in range(self.row_ptr[u], self.row_ptr[u + 1]):
                    rv = self.rev[q]
                    if rv is None:
                        continue
                    if rv[0] == "halo":
                        c = int(halo[rv[1], w])
                    else:
                        c = self._send_row(rv[1])[w]
                    c &= ~mine & M64
                    if not c:
                        continue
                    if int(self.fwd[q]) & GIN:  # u's AcceptFrom drops v's RPCs whole
                        self.stats["graylisted"] += bin(c).count("1")
                        continue
                    newb = c & ~seen & ~acc & M64
                    self.stats["duplicates"] += bin(c & acc).count("1") + bin(c & seen).count("1")
                    acc |= newb
                    self.frm[q][w] |= newb
                nxt[u][w] = acc
                if acc:
                    self.seen[u][w] = seen | acc
                    c = bin(acc).count("1")
                    n_new += c
                    for b in range(64):
                        if acc >> b & 1:
                            self.hop[u, w * 64 + b] = h
        self.front = nxt
        self.stats["hop"][h] = n_new
        self.stats["deliveries"] += n_new
        return n_new

    def prop_set_last_hop(self, last_hop):  # (the emulator keeps no validation-time table)
        pass

    def prop_rep(self):  # (the emulator runs the per-pair exchange)
        return False

    def prop_end(self):
        out = abi.PropOut()
        out.deliveries = self.stats["deliveries"]
        out.duplicates = self.stats["duplicates"]
        out.graylisted = self.stats["graylisted"]
        out.transmissions = out.deliveries + out.duplicates + out.graylisted
        for h, c in enumerate(self.stats["hop"]):
            out.hop_deliveries[h] = c
            if c:
                out.hops = h
        return out

    def prop_results(self, n_msgs):
        hop = self.hop[:, :n_msgs].T.copy()
        frm = np.full((n_msgs, self.n), -1, dtype=np.int32)
        for u in range(self.n):
            for q in range(self.row_ptr[u], self.row_ptr[u + 1]):
                for w in range(self.W):
                    bits = self.frm[q][w]
                    for b in range(64):
                        if bits >> b & 1 and w * 64 + b < n_msgs:
                            frm[w * 64 + b, u] = self.col[q]
        return hop, frm


def _as_tensor(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a))


class RepRowsToy:
    """Stand-in for one range shard in the replicated frontier's dense-row
    exchange (gsx.h gsx_prop_rep_rows*, gsx/shard.py RangeSharded._rep_rows),
    TEST INFRASTRUCTURE ONLY: floodsub over a CSR shard (every pair forwards
    everything), arrival hops only.  Every rank keeps the frontier rows of ALL
    nodes two hops deep and its own occupancy bits per hop, exactly the state
    the driver moves (one all-gather of the ranks' row slices, one summed bit
    row per hop; the per-hop receipts read once per chunk), so the driver's
    collective sequence, its chunked end test and the max_hops cut run over
    gloo against a plain BFS."""

    def __init__(self, shard, n_total):
        self.sh = shard
        self.lo = shard.node_lo
        self.n = shard.node_hi - shard.node_lo
        self.n_nodes = self.n
        self.n_total = n_total
        self.row_ptr = shard.row_ptr
        self.col = shard.col.astype(np.int64)
        self.rows_on = False

    # the shard plan: no per-pair exchange in this mode
    def shard_recv_plan(self, rank_lo):
        return np.zeros(len(rank_lo) - 1, dtype=np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint32)

    def shard_send_plan(self, asked, u, v):
        pass

    def shard_set_halo_bases(self, b):
        pass

    def prop_begin(self, msgs, cfg):
        self.m = len(msgs)
        self.W = prop_words(self.m)
        self.max_hops = int(cfg.max_hops)
        self.ow = (self.n_total + 63) // 64 + 1
        self.front = np.zeros((2, self.n_total, self.W), dtype=np.uint64)
        self.occ = np.zeros((2, self.ow), dtype=np.uint64)
        self.seen = np.zeros((self.n, self.W), dtype=np.uint64)
        self.hop = np.full((self.m, self.n), -1, dtype=np.int32)
        self.cnt = np.zeros(abi.GSX_MAX_HOPS + 1, dtype=np.int64)
        self.h = 0
        self.last = None
        for k, s in enumerate(msgs["source"]):  # hop 0 is every rank's: the message list
            s = int(s)
            self.front[0, s, k // 64] |= np.uint64(1 << (k % 64))
            self.occ[0, s // 64] |= np.uint64(1 << (s % 64))
            if self.lo <= s < self.lo + self.n:
                self.seen[s - self.lo, k // 64] |= np.uint64(1 << (k % 64))
                self.hop[k, s - self.lo] = 0

    def prop_rep(self):
        return True

    def prop_rep_fwd_pack(self, out):
        pass

    def prop_rep_fwd_recv(self, inp):
        pass

    def prop_rep_rows(self, on=True):
        assert self.h == 0
        self.rows_on = bool(on)

    def _hop(self):
        assert self.h < self.max_hops
        self.h += 1
        p, c = (self.h - 1) & 1, self.h & 1
        self.occ[c] = 0
        for u in range(self.n):
            acc = np.zeros(self.W, dtype=np.uint64)
            for q in range(self.row_ptr[u], self.row_ptr[u + 1]):
                v = int(self.col[q])
                if int(self.occ[p, v // 64]) >> (v % 64) & 1:
                    acc |= self.front[p, v]
            new = acc & ~self.seen[u]
            self.front[c, self.lo + u] = new
            if new.any():
                g = self.lo + u
                self.occ[c, g // 64] |= np.uint64(1 << (g % 64))
                self.seen[u] |= new
                for w in range(self.W):
                    bits = int(new[w])
                    for b in range(64):
                        if bits >> b & 1:
                            self.hop[w * 64 + b, u] = self.h
                            self.cnt[self.h] += 1

    def prop_rep_step(self, parts=(), counts=()):
        assert self.h == 0 and not parts  # hop 1: no exchange
        self._hop()

    def prop_rep_rows_export(self, rows, occ):
        assert self.rows_on and self.h >= 1
        rows.copy_(_as_tensor(self.front[self.h & 1, self.lo : self.lo + self.n].view(np.int64)))
        occ.copy_(_as_tensor(self.occ[self.h & 1].view(np.int64)))

    def prop_rep_rows_step(self, parts, occ_sum):
        c = self.h & 1
        off = 0
        for part in parts:  # (the ranks' slices in rank order: contiguous ranges)
            a = part.cpu().numpy().view(np.uint64).reshape(-1, self.W)
            self.front[c, off : off + len(a)] = a
            off += len(a)
        assert off == self.n_total
        self.occ[c] = occ_sum.cpu().numpy().view(np.uint64)
        self._hop()

    def prop_hop_counts_dev(self, out):
        out.copy_(_as_tensor(self.cnt))

    def prop_rep_sends_pack(self, out):
        pass

    def prop_rep_sends_recv(self, inp):
        pass

    def prop_set_last_hop(self, last):
        self.last = int(last)

    def prop_end(self):
        out = abi.PropOut()
        out.deliveries = int(self.cnt.sum())
        out.transmissions = out.deliveries
        for h, c in enumerate(self.cnt):
            out.hop_deliveries[h] = int(c)
            if c:
                out.hops = h
        return out
