"""Multi-GPU propagation drivers, one process per GPU.

Two ways to spread GossipSub forwarding (floodsub.go:76-100,
gossipsub.go:943-1013, randomsub.go:99-160) over ranks:

* ``RangeSharded`` — the overlay is range-partitioned by node; every rank's
  engine holds its nodes' rows (gsx_load_overlay_shard).  Per hop each rank
  packs what its nodes send across shards (gsx_prop_pack), one all-to-all
  moves the packed rows (RCCL over xGMI on MI355X: torch.distributed "nccl"),
  and the hop kernel reads them in place of the local gather
  (gsx_prop_step).  The loop ends when a hop delivers nothing on any rank.
  Per-rank results are the single-engine rows of the rank's nodes, bit for bit.

* ``MessageParallel`` — every rank holds the whole overlay and propagates
  its share of the messages (messages are independent given the call's
  forwarding state); the deferred P2/P3 credit counts are summed with one
  all-reduce and folded on every rank, which equals folding them on one engine.

The exchange goes through a tiny transport interface so the same drivers run
over torch.distributed (any backend) or in-process between several engines
on one device (``LocalGroup``, tests).  Nothing here computes propagation: the
engine's HIP kernels do.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from . import abi
from .abi import prop_words  # noqa: F401  (re-exported)

_STAT_KEYS = ("deliveries", "duplicates", "transmissions", "edge_sends", "new_words", "rejected", "ignored",
              "graylisted")




def _torch():
    import torch

    return torch


class DistTransport:
    """torch.distributed transport (RCCL for "nccl", gloo on CPU).

    stage_host: device tensors go through host memory around each
    collective (a gloo group driving GPU buffers, e.g. several ranks
    rehearsing the multi-GPU flow on one card)."""

    def __init__(self, device, group=None, stage_host=False):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.device = device
        self.stage = stage_host
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def _h(self, t):
        return t.cpu() if self.stage and t.is_cuda else t

    def all_to_all(self, recv, send, recv_splits, send_splits):
        r, s = self._h(recv), self._h(send)
        self.dist.all_to_all_single(r, s, list(map(int, recv_splits)), list(map(int, send_splits)), group=self.group)
        if r is not recv:
            recv.copy_(r)

    def all_to_all_parts(self, recv, recv_splits, send_parts):
        """send_parts[k] (contiguous rows) -> rank k; recv gets rank k's rows at
        the k-th split.  One gather copy on the device, then the same
        all_to_all_single every backend runs (the list form would skip the
        copy on RCCL, but this path is the one the tests and the rehearsal
        exercise; the copy is small next to the exchange itself)."""
        _parts_via_single(self, recv, recv_splits, send_parts)

    def all_gather(self, t):
        """-> [rank k's t] (equal shapes on every rank)."""
        h = self._h(t)
        out = [h.new_empty(h.shape) for _ in range(self.world)]
        self.dist.all_gather(out, h, group=self.group)
        if h is not t:
            out = [o.to(t.device) for o in out]
        return out

    def all_reduce_sum(self, t):
        h = self._h(t)
        self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM, group=self.group)
        if h is not t:
            t.copy_(h)

    def all_reduce_max(self, t):
        h = self._h(t)
        self.dist.all_reduce(h, op=self.dist.ReduceOp.MAX, group=self.group)
        if h is not t:
            t.copy_(h)


def _parts_via_single(tp, recv, recv_splits, send_parts) -> None:
    """all_to_all_parts for transports without a list all-to-all: one gather copy."""
    torch = _torch()
    send = torch.cat(list(send_parts), 0)
    tp.all_to_all(recv, send, recv_splits, [len(p) for p in send_parts])


def exchange_plan(backend, rank_lo, transport) -> None:
    """Build the per-hop exchange: this rank's receive list goes to the owners
    of the remote neighbours, which resolve it to their local pairs."""
    torch = _torch()
    counts, ru, rv = backend.shard_recv_plan(rank_lo)
    W = transport.world
    dev = transport.device
    send_cnt = torch.tensor(counts.astype(np.int64), dtype=torch.int64, device=dev)  # what I ask of rank k
    recv_cnt = torch.empty(W, dtype=torch.int64, device=dev)
    transport.all_to_all(recv_cnt, send_cnt, [1] * W, [1] * W)
    asked = recv_cnt.cpu().numpy()  # how many rows rank k asks of me
    req = torch.tensor(np.stack([ru, rv], 1).astype(np.int64).reshape(-1, 2), dtype=torch.int64, device=dev)
    got = torch.empty((int(asked.sum()), 2), dtype=torch.int64, device=dev)
    transport.all_to_all(got, req, asked, counts)
    g = got.cpu().numpy()
    backend.shard_send_plan(asked.astype(np.uint64), g[:, 0].astype(np.uint32), g[:, 1].astype(np.uint32))
    backend._plan_counts = (asked.astype(np.int64), counts.astype(np.int64))
    # compacted exchange: tell every source where its rows start in my halo
    base = np.concatenate([[0], np.cumsum(counts.astype(np.int64))[:-1]])
    mine = torch.tensor(base, dtype=torch.int64, device=dev)
    theirs = torch.empty(W, dtype=torch.int64, device=dev)
    transport.all_to_all(theirs, mine, [1] * W, [1] * W)
    backend.shard_set_halo_bases(theirs.cpu().numpy().astype(np.uint64))


class RangeSharded:
    """Range-sharded propagation over one engine per rank.

    compact=True (default): per hop only the non-empty cross-shard rows
    travel, as (receive slot, row) entries — one small all-to-all of the
    entry counts, then the entries (one host round trip per hop: the entry
    splits are host lists); compact=False moves every cross pair's row with
    fixed splits, so hops run back to back with no host sync: every `chunk`
    hops one all-reduce of the per-hop delivery counts (device) and one read
    find the hop that delivered nothing on any rank — the hops after it were
    empty and changed nothing (1 / chunk host syncs per hop).

    The lean calls take the replicated frontier (gsx_prop_rep_*): compact=True
    moves every rank's new frontier rows as (global id, row) entries, padded
    to the largest rank's count (one host read per hop sizes the all-gather);
    compact=False moves every rank's dense slice of the rows and a summed
    occupancy-bit row per hop, chunked like the dense exchange (_rep_rows)."""

    def __init__(self, backend, rank_lo, transport, compact=True, chunk=4):
        self.be = backend
        self.compact = compact
        self.chunk = max(1, int(chunk))  # dense exchange: hops per host check of the global frontier
        self.rank_lo = np.asarray(rank_lo, dtype=np.uint32)
        self.tp = transport
        exchange_plan(backend, self.rank_lo, transport)
        self.send_counts, self.recv_counts = backend._plan_counts  # rows I send to / receive from rank k
        self.n_send = int(self.send_counts.sum())
        self.n_recv = int(self.recv_counts.sum())
        self._bufs = {}
        self.sent_bytes = 0  # exchange volume this rank sent (cumulative)
        self.hops_run = 0  # hops run (cumulative) and host round trips they took
        self.host_syncs = 0
        self.last_mode = None  # the exchange the last call ran: "replicated" | "compact" | "dense"
        self.gx_hops = 0  # heartbeat forwarding hops (gossip exchange) and their host round trips
        self.gx_syncs = 0
        dev = getattr(transport, "device", None)
        self._stream = None
        if hasattr(backend, "set_stream") and dev is not None and _torch().device(dev).type == "cuda":
            # engine kernels and the collectives on one stream: pack -> all-to-all -> step in order.
            # A stream of our own, made current around every round: torch's default stream has
            # handle 0, which the engine reads as "its own (non-blocking) stream", unordered
            # with the copies and collectives torch issues.
            torch = _torch()
            self._stream = torch.cuda.Stream(device=dev)
            backend.set_stream(self._stream.cuda_stream)

    def _on_stream(self):
        import contextlib

        return _torch().cuda.stream(self._stream) if self._stream is not None else contextlib.nullcontext()

    def _buffers(self, W):
        torch = _torch()
        if W not in self._bufs:
            dev = self.tp.device
            self._bufs = {W: (torch.zeros((max(self.n_send, 1), W), dtype=torch.int64, device=dev),
                              torch.zeros((max(self.n_recv, 1), W), dtype=torch.int64, device=dev))}
        return self._bufs[W]

    def _compact_buffers(self, W):
        torch = _torch()
        key = ("c", W)
        if key not in self._bufs:
            dev = self.tp.device
            self._bufs = {key: (torch.zeros((max(self.n_send, 1), W + 1), dtype=torch.int64, device=dev),
                                torch.zeros((max(self.n_recv, 1), W + 1), dtype=torch.int64, device=dev),
                                torch.zeros((self.tp.world, 2), dtype=torch.int64, device=dev),
                                torch.zeros((self.tp.world, 2), dtype=torch.int64, device=dev))}
        return self._bufs[key]

    def _hop_compact(self, W, first: bool):
        """One hop of the compacted exchange with ONE host round trip: the pack
        leaves (entries for rank k, this rank's receipts of the hop before) on
        the device, one all-to-all of those pairs, one copy of both count
        vectors to the host (the entry splits must be host lists); the
        entries go out as per-destination views of the pack buffer, and the
        hop runs without a sync.  -> (whether this hop ran: False when the hop
        before delivered nothing on any rank, the call is over; the first
        receipts of the hop before summed over the ranks)."""
        torch = _torch()
        be, tp = self.be, self.tp
        out, recv, sc, rc = self._compact_buffers(W)
        be.prop_pack_compact_dev(out, sc)
        tp.all_to_all(rc, sc, [1] * tp.world, [1] * tp.world)
        hc = torch.cat([sc, rc], 0).cpu().numpy()  # the hop's one host sync
        self.host_syncs += 1
        cnt, rcnt = hc[: tp.world, 0], hc[tp.world :, 0]
        got = int(hc[tp.world :, 1].sum())
        if not first and got == 0:
            return False, 0
        sb = np.concatenate([[0], np.cumsum(self.send_counts)[:-1]])
        parts = [out[int(sb[d]) : int(sb[d] + cnt[d])] for d in range(tp.world)]
        n = int(rcnt.sum())
        tp.all_to_all_parts(recv[:n], rcnt, parts)
        self.sent_bytes += int(cnt.sum()) * (W + 1) * 8
        be.prop_step_compact(recv, n, sync=False)
        self.hops_run += 1
        return True, got

    def propagate(self, msgs, cfg: abi.PropConfig):
        """-> (this rank's PropOut as a dict, global totals dict)."""
        with self._on_stream():
            return self._propagate(msgs, cfg)

    def _propagate(self, msgs, cfg: abi.PropConfig):
        torch = _torch()
        be, tp = self.be, self.tp
        W = prop_words(len(msgs))
        if not self.compact:
            send, recv = self._buffers(W)
        be.prop_begin(msgs, cfg)
        last = 0  # the last hop that delivered on any rank (gsx_prop_set_last_hop)
        if getattr(be, "prop_rep", None) is not None and be.prop_rep():
            self.last_mode = "replicated" if self.compact else "replicated-rows"
            last = self._propagate_rep(W, cfg)
        elif self.compact:
            self.last_mode = "compact"
            ran = 0
            for h in range(cfg.max_hops):
                more, got = self._hop_compact(W, h == 0)
                if h and got:
                    last = h
                if not more:
                    break
                ran += 1
            if ran == cfg.max_hops and ran:  # cut by max_hops: the last hop's receipts, summed
                cnt = torch.zeros(abi.GSX_MAX_HOPS + 1, dtype=torch.int64, device=tp.device)
                be.prop_hop_counts_dev(cnt)
                tp.all_reduce_sum(cnt)
                if int(cnt[ran].item()):
                    last = ran
                self.host_syncs += 1
        else:
            self.last_mode = "dense"
            cnt = torch.zeros(abi.GSX_MAX_HOPS + 1, dtype=torch.int64, device=tp.device)
            h = 0
            while h < cfg.max_hops:
                k = min(self.chunk, cfg.max_hops - h)
                for _ in range(k):  # no host sync inside the chunk
                    be.prop_pack(send)
                    tp.all_to_all(recv[: self.n_recv], send[: self.n_send], self.recv_counts, self.send_counts)
                    self.sent_bytes += self.n_send * W * 8
                    be.prop_step(recv, sync=False)
                    self.hops_run += 1
                h += k
                be.prop_hop_counts_dev(cnt)
                tp.all_reduce_sum(cnt)
                c = cnt.cpu().numpy()  # the chunk's one host sync
                self.host_syncs += 1
                nz = np.nonzero(c[1 : h + 1])[0]
                last = int(nz[-1]) + 1 if len(nz) else 0
                if (c[h - k + 1 : h + 1] == 0).any():
                    break
        be.prop_set_last_hop(last)
        out = be.prop_end()
        return out_dict(out), totals(out, tp)


    def _propagate_rep(self, W, cfg) -> int:
        """The replicated frontier (gsx.h gsx_prop_rep_*): the cross pairs' fwd
        bytes once, hop 1 with no exchange (hop 0 is the message list), then per
        hop one all-gather of the ranks' new frontier rows (padded to the
        largest rank's count, which the one host read per hop gives along with
        the hop's receipts summed over the ranks), and the cross pairs' sends of
        the call at its end.  -> the last hop that delivered on any rank."""
        torch = _torch()
        be, tp = self.be, self.tp
        dev, R = tp.device, tp.world
        sf = torch.zeros(max(self.n_send, 1), dtype=torch.uint8, device=dev)
        rf = torch.zeros(max(self.n_recv, 1), dtype=torch.uint8, device=dev)
        be.prop_rep_fwd_pack(sf)
        tp.all_to_all(rf[: self.n_recv], sf[: self.n_send], self.recv_counts, self.send_counts)
        be.prop_rep_fwd_recv(rf)
        last = 0
        if cfg.max_hops >= 1 and not self.compact:
            last = self._rep_rows(W, cfg)
        elif cfg.max_hops >= 1:
            be.prop_rep_step()
            self.hops_run += 1
            n_local = max(int(getattr(be, "n_nodes", 0) or 0), 1)
            out = self._bufs.get(("rep", W, n_local))
            if out is None:
                out = torch.empty((n_local, W + 1), dtype=torch.int64, device=dev)
                self._bufs = {("rep", W, n_local): out}
            cnt = torch.zeros(2, dtype=torch.int64, device=dev)
            h, cut = 1, True
            while h < cfg.max_hops:
                be.prop_rep_pack_dev(out, cnt)
                c = torch.stack(tp.all_gather(cnt)).cpu().numpy()  # the hop's one host sync
                self.host_syncs += 1
                if int(c[:, 1].sum()) == 0:
                    cut = False
                    break
                last = h
                m = int(c[:, 0].max())
                parts = tp.all_gather(out[:m]) if m else []
                others = [(parts[k], int(c[k, 0])) for k in range(R) if k != tp.rank and c[k, 0]]
                self.sent_bytes += m * (W + 1) * 8 * (R - 1)  # (an all-gather delivers the padded rows to R - 1 ranks)
                be.prop_rep_step([p for p, _ in others], [n for _, n in others])
                self.hops_run += 1
                h += 1
            if cut:  # the last hop ran without a look at its receipts: sum them
                hc = torch.zeros(abi.GSX_MAX_HOPS + 1, dtype=torch.int64, device=dev)
                be.prop_hop_counts_dev(hc)
                tp.all_reduce_sum(hc)
                self.host_syncs += 1
                if int(hc[h].item()):
                    last = h
        ss = torch.zeros(max(self.n_send, 1), dtype=torch.int64, device=dev)
        rs = torch.zeros(max(self.n_recv, 1), dtype=torch.int64, device=dev)
        be.prop_rep_sends_pack(ss)
        tp.all_to_all(rs[: self.n_recv], ss[: self.n_send], self.recv_counts, self.send_counts)
        be.prop_rep_sends_recv(rs)
        return last

    def _rep_rows(self, W, cfg) -> int:
        """The replicated frontier as dense row slices (compact=False;
        gsx_prop_rep_rows): hop 1 from the message list, then per hop one
        all-gather of every rank's slice of the hop's rows (n_local x W words,
        padded to the largest range) and one all-reduce of the occupancy-bit
        rows (the ranks own disjoint bits: their sum is their union) — no host
        read inside a chunk; every `chunk` hops one all-reduce of the per-hop
        receipts and one read find the end (the hops after a hop that delivered
        nothing on any rank run empty and change nothing: 1 / chunk host syncs
        per hop, up to chunk - 1 empty hops).  -> the last hop that delivered."""
        torch = _torch()
        be, tp = self.be, self.tp
        dev, R = tp.device, tp.world
        lens = np.diff(self.rank_lo.astype(np.int64))
        L = max(int(lens.max()), 1)
        n_total = int(self.rank_lo[-1])
        ow = (n_total + 63) // 64 + 1
        key = ("rows", W, L, ow)
        bufs = self._bufs.get(key)
        if bufs is None:
            bufs = (torch.zeros((L, W), dtype=torch.int64, device=dev), torch.zeros(ow, dtype=torch.int64, device=dev),
                    torch.zeros(abi.GSX_MAX_HOPS + 1, dtype=torch.int64, device=dev))
            self._bufs = {key: bufs}
        rows, occ, cnt = bufs
        n_local = int(lens[tp.rank])
        be.prop_rep_rows(True)
        be.prop_rep_step()  # hop 1: hop 0's rows are every rank's already
        self.hops_run += 1
        h, last = 1, 0
        while h < cfg.max_hops:
            k = min(self.chunk, cfg.max_hops - h)
            for _ in range(k):  # no host sync inside the chunk
                be.prop_rep_rows_export(rows[:n_local], occ)
                parts = tp.all_gather(rows)
                tp.all_reduce_sum(occ)
                self.sent_bytes += L * W * 8 * (R - 1) + ow * 8
                be.prop_rep_rows_step([parts[j][: int(lens[j])] for j in range(R)], occ)
                self.hops_run += 1
                h += 1
            be.prop_hop_counts_dev(cnt)
            tp.all_reduce_sum(cnt)
            c = cnt.cpu().numpy()  # the chunk's one host sync
            self.host_syncs += 1
            nz = np.nonzero(c[1 : h + 1])[0]
            last = int(nz[-1]) + 1 if len(nz) else 0
            if (c[h - k + 1 : h + 1] == 0).any():
                break
        else:
            if h == 1:  # (max_hops 1: no chunk ran, hop 1's receipts decide `last`)
                be.prop_hop_counts_dev(cnt)
                tp.all_reduce_sum(cnt)
                c = cnt.cpu().numpy()
                self.host_syncs += 1
                nz = np.nonzero(c[1 : h + 1])[0]
                last = int(nz[-1]) + 1 if len(nz) else 0
        return last

    def heartbeat(self, tick: int, now: int, seed: int):
        """One heartbeat round of every node on every rank (gossipsub.go:1303-1564
        with handleGraft / handlePrune): the GRAFT/PRUNE words of the
        cross-shard pairs go to the receivers' ranks (one all-to-all), the
        PRUNE answers come back (a second, smaller one).  -> (this rank's
        counters, summed counters)."""
        with self._on_stream():
            return self._heartbeat(tick, now, seed)

    def _heartbeat(self, tick: int, now: int, seed: int):
        torch = _torch()
        be, tp = self.be, self.tp
        dev = tp.device
        s2 = torch.zeros((max(self.n_send, 1), 2), dtype=torch.int64, device=dev)
        r2 = torch.zeros((max(self.n_recv, 1), 2), dtype=torch.int64, device=dev)
        px = getattr(be, "hb_px_enabled", lambda: False)()
        be.hb_begin(tick, now, seed)
        if px:  # the (A) PRUNEs' PX lists to the receivers' ranks, before their (B)
            self._px_exchange(0)
        be.hb_pack_ctl(s2)
        tp.all_to_all(r2[: self.n_recv], s2[: self.n_send], self.recv_counts, self.send_counts)
        be.hb_recv(r2)
        if px:  # the (B) answers' PX lists, before the GRAFT senders' (C)
            self._px_exchange(1)
        s1 = torch.zeros(max(self.n_send, 1), dtype=torch.int64, device=dev)
        r1 = torch.zeros(max(self.n_recv, 1), dtype=torch.int64, device=dev)
        be.hb_pack_resp(s1)
        tp.all_to_all(r1[: self.n_recv], s1[: self.n_send], self.recv_counts, self.send_counts)
        out = be.hb_end(r1)
        n_sets = be.gx_pending() if hasattr(be, "gx_pending") else None
        if n_sets is not None:  # the gossip exchange (D) across the ranks
            out = self._gx_exchange(n_sets)
        d = out.as_dict()
        t = torch.tensor([d[k] for k, _ in abi.HeartbeatOut._fields_], dtype=torch.int64, device=dev)
        tp.all_reduce_sum(t)
        t = t.cpu().numpy()
        return d, {k: int(t[i]) for i, (k, _) in enumerate(abi.HeartbeatOut._fields_)}


    def _entries(self, counts, words, pack):
        """Variable entry all-to-all: counts[k] entries of `words` u64 for rank
        k (pack(out) writes them, destination by destination) -> (the received
        entries, their number)."""
        torch = _torch()
        tp = self.tp
        sc = torch.tensor(counts.astype(np.int64), dtype=torch.int64, device=tp.device)
        rc = torch.empty(tp.world, dtype=torch.int64, device=tp.device)
        tp.all_to_all(rc, sc, [1] * tp.world, [1] * tp.world)
        rcnt = rc.cpu().numpy()
        n_out, n_in = int(counts.sum()), int(rcnt.sum())
        send = torch.zeros((max(n_out, 1), words), dtype=torch.int64, device=tp.device)
        pack(send)
        recv = torch.zeros((max(n_in, 1), words), dtype=torch.int64, device=tp.device)
        tp.all_to_all(recv[:n_in], send[:n_out], rcnt, counts.astype(np.int64))
        return recv, n_in

    def _gx_exchange(self, n_sets: int):
        """The gossip exchange of a sharded heartbeat (gsx.h, gsx_gx_*): the
        common words ANDed over ranks, the IHAVE bits and answer bits of the
        cross-shard pairs (fixed words per pair), the senders' cache rows
        (entries), the exchange at the receivers, then the forwarding of the
        recovered messages hop by hop (frontier entries, a frontier count
        summed over ranks per hop), and the round's end with every rank's
        got flags.  -> this rank's counters."""
        torch = _torch()
        be, tp = self.be, self.tp
        dev = tp.device
        W = tp.world
        c = be.gx_common(n_sets)
        if n_sets:  # (the set count is the same on every rank: the cache is global)
            parts = tp.all_gather(torch.tensor(c.view(np.int64), dtype=torch.int64, device=dev))
            c = np.bitwise_and.reduce(np.stack([p.cpu().numpy().view(np.uint64) for p in parts]), axis=0)
        be.gx_set_common(c)
        s2 = torch.zeros((max(self.n_send, 1), 2), dtype=torch.int64, device=dev)
        r2 = torch.zeros((max(self.n_recv, 1), 2), dtype=torch.int64, device=dev)
        be.gx_pack_ihave(s2)
        tp.all_to_all(r2[: self.n_recv], s2[: self.n_send], self.recv_counts, self.send_counts)
        be.gx_recv_ihave(r2)
        rows, n_rows = self._entries(be.gx_rows_pack(W), be.gx_rows_words(), lambda out: be.gx_rows_pack(W, out))
        be.gx_rows_recv(rows, n_rows)
        n_runs = be.gx_exchange()
        del rows
        for run in range(n_runs):
            be.gxf_begin(run)
            s1 = torch.zeros(max(self.n_send, 1), dtype=torch.int64, device=dev)
            r1 = torch.zeros(max(self.n_recv, 1), dtype=torch.int64, device=dev)
            be.gxf_pack_fout(s1)
            tp.all_to_all(r1[: self.n_recv], s1[: self.n_send], self.recv_counts, self.send_counts)
            be.gxf_recv_fout(r1)
            words = be.gxf_entry_words()
            if not hasattr(be, "gxf_pack_dev"):  # (a backend without the device-count pack)
                hop = 1
                while True:
                    ent, n_ent = self._entries(be.gxf_pack(hop, W), words, lambda out, h=hop: be.gxf_pack(h, W, out))
                    front = be.gxf_step(hop, ent, n_ent)
                    t = torch.tensor([front], dtype=torch.int64, device=dev)
                    tp.all_reduce_sum(t)
                    self.gx_hops += 1
                    self.gx_syncs += 4
                    if int(t.item()) == 0:
                        break
                    hop += 1
                be.gxf_end()
                continue
            # one host round trip per hop: the pack leaves (entries for rank k, this
            # rank's frontier of the hop before) on the device; one all-to-all of the
            # pairs, one read; the run ends at the pack after a hop that left no
            # frontier on any rank
            out = torch.zeros((max(self.n_send, 1), words), dtype=torch.int64, device=dev)
            sc = torch.zeros((W, 2), dtype=torch.int64, device=dev)
            rc = torch.zeros((W, 2), dtype=torch.int64, device=dev)
            sb = np.concatenate([[0], np.cumsum(self.send_counts)[:-1]])
            hop, held = 1, None
            while hop < abi.GXF_MAX_HOPS:
                be.gxf_pack_dev(hop, out, sc)
                tp.all_to_all(rc, sc, [1] * W, [1] * W)
                hc = torch.cat([sc, rc], 0).cpu().numpy()  # the hop's one host sync
                self.gx_syncs += 1
                if hop > 1 and int(hc[W:, 1].sum()) == 0:
                    break
                cnt, rcnt = hc[:W, 0], hc[W:, 0]
                n_in = int(rcnt.sum())
                recv = torch.zeros((max(n_in, 1), words), dtype=torch.int64, device=dev)
                tp.all_to_all_parts(recv[:n_in], rcnt, [out[int(sb[d]) : int(sb[d] + cnt[d])] for d in range(W)])
                last = hop == abi.GXF_MAX_HOPS - 1
                front = be.gxf_step(hop, recv, n_in, sync=last)
                held = recv  # (read by the hop's kernels: alive until the next sync)
                self.gx_hops += 1
                hop += 1
                if last:  # the engine runs no hop past this one: a frontier left anywhere is an error
                    t = torch.tensor([front], dtype=torch.int64, device=dev)
                    tp.all_reduce_sum(t)
                    self.gx_syncs += 1
                    if int(t.item()):
                        raise abi.GsxError(abi.GSX_ERANGE, f"heartbeat forwarding still has a frontier after "
                                                           f"{abi.GXF_MAX_HOPS - 1} hops: gsx_gxf_step")
            del held
            be.gxf_end()
        got = be.gx_got(n_sets)
        if n_sets:
            g = torch.tensor(got.astype(np.int64), dtype=torch.int64, device=dev)
            tp.all_reduce_max(g)
            got = g.cpu().numpy().astype(np.uint8)
        return be.gx_end(got)

    def _px_exchange(self, kind: int):
        """Peer exchange across shards (gsx_hb_px_*): the PX lists of this rank's
        cross-shard PRUNEs go to the receivers' ranks (one count all-to-all,
        one entry all-to-all), which handle them."""
        torch = _torch()
        be, tp = self.be, self.tp
        w = be.hb_px_entry_words()
        cnt = be.hb_px_count(kind, tp.world).astype(np.int64)
        send = torch.zeros((max(int(cnt.sum()), 1), w), dtype=torch.int32, device=tp.device)
        be.hb_px_pack(kind, send)
        sc = torch.tensor(cnt, dtype=torch.int64, device=tp.device)
        rc = torch.empty(tp.world, dtype=torch.int64, device=tp.device)
        tp.all_to_all(rc, sc, [1] * tp.world, [1] * tp.world)
        rcnt = rc.cpu().numpy()
        n = int(rcnt.sum())
        recv = torch.zeros((max(n, 1), w), dtype=torch.int32, device=tp.device)
        tp.all_to_all(recv[:n], send[: int(cnt.sum())], rcnt, cnt)
        be.hb_px_recv(kind, recv, n)


class MessageParallel:
    """Every rank propagates its block of the messages over the full overlay.

    The engine runs on a torch stream of its own (set_stream), so its kernels,
    the credit copies and the collectives are ordered on one stream with no
    host synchronisation between them.  epoch=False (default): each batch's
    deferred P2/P3/P4 counts are summed over ranks and folded right away (the
    single engine with GSX_CREDIT_NOW, batch by batch).  epoch=True: batches
    only accumulate their counts on every rank; end_epoch() (before a
    heartbeat) sums them with one all-reduce and folds them:
    equal to one engine propagating the same batches with GSX_CREDIT_DEFER and
    folding once.

    cache=True (default): after a gossipsub batch every replica takes its
    block out of its message cache, the blocks are all-gathered and every
    replica Puts the whole batch back (gsx_mcache_put), so every replica's
    cache — and with it emitGossip and the gossip exchange of its heartbeats —
    equals one engine's (gossipsub.go:943-944, mcache.go:55-59).  heartbeat()
    then runs the same round on every replica with no exchange: the replicas'
    states are equal, so are their decisions (the round is replicated, not
    split)."""

    def __init__(self, engine, transport, epoch: bool = False, cache: bool = True):
        self.e = engine
        self.tp = transport
        self.epoch = epoch
        self.cache = cache
        self.pending = False
        self.gathered_bytes = 0  # cache blocks received (cumulative)
        self._stream = None
        dev = getattr(transport, "device", None)
        if hasattr(engine, "set_stream") and dev is not None and _torch().device(dev).type == "cuda":
            torch = _torch()
            self._stream = torch.cuda.Stream(device=dev)
            engine.set_stream(self._stream.cuda_stream)

    def _on_stream(self):
        import contextlib

        return _torch().cuda.stream(self._stream) if self._stream is not None else contextlib.nullcontext()

    def bounds(self, m: int):
        r, w = self.tp.rank, self.tp.world
        return (m * r) // w, (m * (r + 1)) // w

    def share(self, msgs):
        lo, hi = self.bounds(len(msgs))
        return msgs[lo:hi]

    def propagate(self, msgs, cfg: abi.PropConfig):
        with self._on_stream():
            mine = self.share(msgs)
            credit = cfg.credit_scores
            c = abi.PropConfig()
            for f, _ in abi.PropConfig._fields_:
                setattr(c, f, getattr(cfg, f))
            if credit:
                c.credit_scores = abi.GSX_CREDIT_DEFER
            out = self.e.propagate(mine, c)[0]
            tot = totals(out, self.tp)
            if self.cache and cfg.router == abi.GSX_ROUTER_GOSSIPSUB and len(msgs):
                # the merged set keeps the validation times of hops 0 .. the last hop that
                # delivered on any replica, as one engine propagating every message does
                cm = abi.PropConfig()
                for f, _ in abi.PropConfig._fields_:
                    setattr(cm, f, getattr(cfg, f))
                cm.max_hops = tot["hops"]
                self._merge_cache(msgs, cm, len(mine))
            if credit:
                self.pending = True
                if not self.epoch:
                    self.end_epoch()
            return out_dict(out), tot

    def _merge_cache(self, msgs, cfg, n_mine: int):
        """One all-gather of the replicas' cache blocks; every replica Puts the whole batch."""
        m, w = len(msgs), self.tp.world
        counts = [(m * (k + 1)) // w - (m * k) // w for k in range(w)]
        pad = max(self.e.mcache_part_size(n, cfg) for n in counts)
        if n_mine:
            mine, got = self.e.mcache_take_block(pad, self.tp.device, cfg)
            if got != n_mine:
                raise RuntimeError(f"the newest cached batch holds {got} messages, not this replica's {n_mine}")
        else:
            mine = self.e.mcache_empty_block(pad, self.tp.device)
        blocks = self.tp.all_gather(mine)
        self.gathered_bytes += (w - 1) * mine.numel() * mine.element_size()
        self.e.mcache_put(msgs, cfg, blocks, counts)

    def end_epoch(self):
        """Sum every rank's pending first receipts, in-window duplicates and
        invalid deliveries (P4) and fold them (one all-reduce of 3 x E x 4 B)."""
        if not self.pending:
            return
        with self._on_stream():
            torch = _torch()
            E = self.e.n_pairs
            cnt = torch.empty((3, max(E, 1)), dtype=torch.int32, device=self.tp.device)
            self.e.pending_credits(cnt[0].data_ptr(), cnt[1].data_ptr())
            self.e.pending_invalid(cnt[2].data_ptr())
            self.tp.all_reduce_sum(cnt)
            self.e.replace_pending_invalid(cnt[2].data_ptr())
            self.e.fold_credits(cnt[0].data_ptr(), cnt[1].data_ptr())
        self.pending = False

    def heartbeat(self, tick: int, now: int, seed: int):
        """One heartbeat (gossipsub.go:1303-1564, with the gossip exchange when
        on) on every replica: pending credits are folded first, then each
        replica runs the whole round on its equal state.  -> (this replica's
        counters, the round's counters) — the same dict: the round is not split."""
        self.end_epoch()
        with self._on_stream():
            d = self.e.heartbeat(tick, now, seed).as_dict()
        return d, dict(d)


def out_dict(out) -> dict:
    d = out.as_dict()
    d.update(edge_sends=int(out.edge_sends), new_words=int(out.new_words), hop_kernel_ms=float(out.hop_kernel_ms),
             hop_launches=int(out.hop_launches))
    return d


def totals(out, tp) -> dict:
    """Sums over ranks (max for hops and kernel time)."""
    torch = _torch()
    v = [int(getattr(out, k)) for k in _STAT_KEYS] + [int(x) for x in out.hop_deliveries]
    t = torch.tensor(v, dtype=torch.int64, device=tp.device)
    tp.all_reduce_sum(t)
    mx = torch.tensor([int(out.hops), int(round(out.hop_kernel_ms * 1e6))], dtype=torch.int64, device=tp.device)
    tp.all_reduce_max(mx)
    t = t.cpu().numpy()
    mx = mx.cpu().numpy()
    d = {k: int(t[i]) for i, k in enumerate(_STAT_KEYS)}
    d["hops"] = int(mx[0])
    d["hop_deliveries"] = [int(x) for x in t[len(_STAT_KEYS) :][: d["hops"] + 1]]
    d["hop_kernel_ms_max"] = float(mx[1]) / 1e6
    return d


# ---- in-process transport: several engines (shards) in one process ------------------
class LocalGroup:
    """Lock-step in-process stand-in for a process group over `world` members
    (used to run every shard of a test overlay on one GPU).  Member k calls the
    collectives through LocalTransport(group, k); a collective completes when
    all members have called it, which happens because the members run as
    Python threads."""

    def __init__(self, world: int, device, serial: bool = False):
        import threading

        self.world = world
        self.device = device
        self.barrier = threading.Barrier(world)
        self.slots: List[Optional[object]] = [None] * world
        # serial: the members take turns between collectives, each turn drained
        # before the next starts, so one member's kernels never overlap
        # another's on the shared device (per-shard kernel times as if each
        # shard had a GPU of its own: tools/shard_scaling.py)
        self.turn = threading.Lock() if serial else None


class LocalTransport:
    def __init__(self, group: LocalGroup, rank: int):
        self.g = group
        self.rank = rank
        self.world = group.world
        self.device = group.device

    def _gather(self, obj):
        turn = self.g.turn
        if turn is not None:  # end of this member's turn: drain its work, let the next one run
            torch = _torch()
            if torch.device(self.device).type == "cuda":
                torch.cuda.synchronize(self.device)
            turn.release()
        try:
            self.g.slots[self.rank] = obj
            self.g.barrier.wait()
            vals = list(self.g.slots)
            self.g.barrier.wait()
        finally:
            if turn is not None:
                turn.acquire()
        return vals

    def all_to_all(self, recv, send, recv_splits, send_splits):
        torch = _torch()
        if send.is_cuda:
            torch.cuda.synchronize(send.device)
        so = np.concatenate([[0], np.cumsum(np.asarray(send_splits, dtype=np.int64))])
        vals = self._gather((send, so))
        parts = [vals[k][0][vals[k][1][self.rank] : vals[k][1][self.rank + 1]] for k in range(self.world)]
        if parts:
            recv.copy_(torch.cat(parts, 0).reshape(recv.shape))
        if recv.is_cuda:
            torch.cuda.synchronize(recv.device)
        self._gather(None)  # senders may reuse their buffers only after everyone copied

    def all_to_all_parts(self, recv, recv_splits, send_parts):
        _parts_via_single(self, recv, recv_splits, send_parts)

    def all_gather(self, t):
        torch = _torch()
        c = t.clone()
        if c.is_cuda:
            torch.cuda.synchronize(c.device)
        vals = self._gather(c)
        self._gather(None)
        return vals

    def _settled(self, t):
        """A copy of t whose values are final (members run on streams of their own)."""
        torch = _torch()
        c = t.clone()
        if c.is_cuda:
            torch.cuda.synchronize(c.device)
        return c

    def all_reduce_sum(self, t):
        vals = self._gather(self._settled(t))
        acc = vals[0].clone()
        for v in vals[1:]:
            acc += v
        t.copy_(acc)
        if t.is_cuda:
            _torch().cuda.synchronize(t.device)
        self._gather(None)

    def all_reduce_max(self, t):
        vals = self._gather(self._settled(t))
        acc = vals[0].clone()
        for v in vals[1:]:
            acc = acc.maximum(v)
        t.copy_(acc)
        if t.is_cuda:
            _torch().cuda.synchronize(t.device)
        self._gather(None)


def run_local(world: int, device, fn: "callable", args: Sequence, serial: bool = False) -> list:
    """Run fn(transport, *args[k]) for k in range(world) as lock-step threads
    (serial: one member's work at a time between collectives, LocalGroup)."""
    import threading

    torch = _torch()  # import and initialise the device runtime on the calling (main) thread
    if torch.device(device).type == "cuda":
        torch.cuda.init()
        torch.zeros(1, device=device)
    g = LocalGroup(world, device, serial=serial)
    res: List[object] = [None] * world
    err: List[BaseException] = []

    def body(k):
        if g.turn is not None:
            g.turn.acquire()
        try:
            res[k] = fn(LocalTransport(g, k), *args[k])
            if g.turn is not None and torch.device(device).type == "cuda":
                torch.cuda.synchronize(device)
        except BaseException as ex:  # surface the first failure, release the others
            err.append(ex)
            g.barrier.abort()
        finally:
            if g.turn is not None:
                g.turn.release()

    th = [threading.Thread(target=body, args=(k,)) for k in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise err[0]
    return res
