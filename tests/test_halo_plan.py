"""Multi-rank halo exchange logic on the CPU (no GPU needed).

The library's host-only entries roms_gpu_halo_plan / roms_gpu_halo_map expose
the neighbour table and the exact cell order its pack/unpack kernels use.
These tests check the plan's symmetry on many processor grids, then run the
exchange itself between world_size 2 and 4 gloo processes -- pack with the
library's maps, send/recv with the same per-peer ordering the RCCL transport
uses, unpack -- and require every halo cell to hold the global field's value
(mpi_exchanges.F semantics: a subdomain's halo equals its neighbours'
interior / the periodic wrap / the closed-edge ghost row).
"""
import itertools
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import romsgpu as R

GRIDS = [(1, 1), (2, 1), (1, 2), (2, 2), (3, 2), (2, 3), (3, 3)]


def _local_plan(LLm, MMm, npx, npe, rank, ewp, nsp):
    jn, inn = divmod(rank, npx)
    Lm, _ = R.rank_extent(LLm, npx, inn)
    Mm, _ = R.rank_extent(MMm, npe, jn)
    return (Lm, Mm, inn, jn) + R.halo_plan(Lm, Mm, npx, npe, inn, jn, ewp, nsp)


@pytest.mark.parametrize("npx,npe", GRIDS)
@pytest.mark.parametrize("ewp,nsp", list(itertools.product([0, 1], [0, 1])))
def test_plan_is_symmetric(npx, npe, ewp, nsp):
    LLm, MMm = 23, 17   # uneven split: exercises the off_xi/off_eta corrections
    plans = [_local_plan(LLm, MMm, npx, npe, r, ewp, nsp) for r in range(npx * npe)]
    assert sum(R.rank_extent(LLm, npx, i)[0] for i in range(npx)) == LLm
    assert sum(R.rank_extent(MMm, npe, j)[0] for j in range(npe)) == MMm
    for r, (Lm, Mm, inn, jn, peer, cnt, strip) in enumerate(plans):
        for d in range(8):
            p = peer[d]
            if p < 0:
                assert cnt[d] == 0
                continue
            o = R.HALO_OPP[d]
            assert plans[p][4][o] == r, (r, d, p)          # neighbour points back
            assert plans[p][5][o] == cnt[d], (r, d, p)     # message sizes agree
        # a closed physical edge has no neighbour, a periodic or interior one does
        assert (peer[0] >= 0) == bool(ewp or inn > 0)
        assert (peer[3] >= 0) == bool(nsp or jn < npe - 1)


def _global_field(LLm, MMm, ewp, nsp, seed, H=2):
    """Global (MMm+2H, LLm+2H) field with H-deep halos (global cell (i, j) at
    [j+H-1, i+H-1]): periodic wrap, or random physical ghost rows at closed
    edges (the rows beyond stay NaN)."""
    rng = np.random.default_rng(seed)
    G = np.full((MMm + 2 * H, LLm + 2 * H), np.nan)
    G[H:MMm + H, H:LLm + H] = rng.standard_normal((MMm, LLm))
    if not ewp:
        G[H - 1:MMm + H + 1, H - 1] = rng.standard_normal(MMm + 2)
        G[H - 1:MMm + H + 1, LLm + H] = rng.standard_normal(MMm + 2)
    if not nsp:
        G[H - 1, H - 1:LLm + H + 1] = rng.standard_normal(LLm + 2)
        G[MMm + H, H - 1:LLm + H + 1] = rng.standard_normal(LLm + 2)
    if ewp:
        G[:, 0:H] = G[:, LLm:LLm + H]
        G[:, LLm + H:LLm + 2 * H] = G[:, H:2 * H]
    if nsp:
        G[0:H, :] = G[MMm:MMm + H, :]
        G[MMm + H:MMm + 2 * H, :] = G[H:2 * H, :]
    return G


def _exchange_worker(rank, world, port, LLm, MMm, npx, npe, ewp, nsp, nlev, q, H=2):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        jn, inn = divmod(rank, npx)
        Lm, iSW = R.rank_extent(LLm, npx, inn)
        Mm, jSW = R.rank_extent(MMm, npe, jn)
        peer, cnt, _ = R.halo_plan(Lm, Mm, npx, npe, inn, jn, ewp, nsp)
        if H != 2:
            cnt = [len(R.halo_map(Lm, Mm, npx, npe, inn, jn, ewp, nsp, d, False, width=H)[0]) for d in range(8)]
        Gs = [_global_field(LLm, MMm, ewp, nsp, 100 + k, H) for k in range(nlev)]
        # local windows: local (i,j) <-> global (iSW+i, jSW+j); array index +H-1
        o = H - 1
        win = [G[jSW:jSW + Mm + 2 * H, iSW:iSW + Lm + 2 * H] for G in Gs]
        A = [np.full_like(w, np.nan) for w in win]
        # cells this rank owns: interior plus its physical (closed-edge) ghost
        # row/column, which the BC code -- not the exchange -- sets
        i_lo = 0 if (not ewp and inn == 0) else 1
        i_hi = Lm + 1 if (not ewp and inn == npx - 1) else Lm
        j_lo = 0 if (not nsp and jn == 0) else 1
        j_hi = Mm + 1 if (not nsp and jn == npe - 1) else Mm
        for a, w in zip(A, win):
            a[j_lo + o:j_hi + o + 1, i_lo + o:i_hi + o + 1] = w[j_lo + o:j_hi + o + 1, i_lo + o:i_hi + o + 1]
        maps = [R.halo_map(Lm, Mm, npx, npe, inn, jn, ewp, nsp, d, False, width=H) for d in range(8)]
        umaps = [R.halo_map(Lm, Mm, npx, npe, inn, jn, ewp, nsp, d, True, width=H) for d in range(8)]
        send = {}
        for d in range(8):
            if peer[d] < 0:
                continue
            iv, jv = maps[d]
            send[d] = torch.from_numpy(np.concatenate([a[jv + o, iv + o] for a in A]))
        reqs, recv = [], {}
        # the transport's ordering: messages to a peer in direction order,
        # receives for halo opp(d) in the same order (tag = sender's direction)
        for d in range(8):
            if peer[d] >= 0 and peer[d] != rank:
                reqs.append(dist.isend(send[d], dst=peer[d], tag=d))
        for d in range(8):
            h = R.HALO_OPP[d]
            if peer[h] >= 0:
                if peer[h] == rank:
                    recv[h] = send[d].clone()
                else:
                    recv[h] = torch.empty(nlev * cnt[h], dtype=torch.float64)
                    reqs.append(dist.irecv(recv[h], src=peer[h], tag=d))
        for r_ in reqs:
            r_.wait()
        for h, buf in recv.items():
            iv, jv = umaps[h]
            parts = buf.numpy().reshape(nlev, cnt[h])
            for a, part in zip(A, parts):
                a[jv + o, iv + o] = part
        bad = 0
        for a, w in zip(A, win):
            defined = ~np.isnan(w)
            bad += int(np.sum(a[defined] != w[defined]))
        q.put((rank, bad))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("npx,npe,ewp,nsp", [(2, 1, 1, 1), (1, 2, 0, 0), (2, 1, 0, 1), (2, 2, 1, 1), (2, 2, 0, 0),
                                             (2, 2, 1, 0)])
def test_gloo_exchange_fills_every_halo(npx, npe, ewp, nsp):
    world = npx * npe
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, 13, 11, npx, npe, ewp, nsp, 3, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == 0 for v in res.values()), res


@pytest.mark.parametrize("H,L,M,npx,npe,ewp,nsp",
                         [(H, 23, 19) + c for H in (4, 8)
                          for c in ((2, 1, 1, 1), (2, 2, 1, 1), (2, 2, 0, 0), (2, 2, 1, 0), (1, 2, 1, 0))] +
                         [(H, 40, 36, 2, 2, 1, 1) for H in (12, 16)] + [(16, 40, 36, 2, 2, 1, 0)])
def test_gloo_wide_exchange_fills_every_halo(H, L, M, npx, npe, ewp, nsp):
    """The fast loop's H-deep exchange (H = 2K, roms_gpu_halo_map_wide; K up
    to 8): every cell of the H-deep frame that has a neighbour, a periodic
    image or a closed-edge ghost row holds the global field's value after
    the swap."""
    world = npx * npe
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, L, M, npx, npe, ewp, nsp, 2, q, H))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == 0 for v in res.values()), res
