"""Edge-sharded BA protocol (m3s.dist_ba.run_sharded) at world_size 2 over gloo, on CPU.

The product shard (HipShard) needs a GPU; here each rank drives the same protocol with an oracle
shard: linearise only its contiguous edge range into rows of a per-edge table (zeros elsewhere),
all-reduce(sum) the table, then assemble/factorise/retract identically on every rank — the exact
structure of HipShard's edge-sum table, with the oracle's per-edge blocks (4x49 H + 2x7 g) as rows.
Checks: (1) every rank ends with bit-identical poses, (2) the 2-rank result is bit-identical to
the 1-rank result of the same shard type (a sum with zeros is exact), (3) it agrees with the
oracle's single-process gauss_newton (gn_kernels.cu:1181-1225 restated) to 1e-5.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O

ROW = 4 * 49 + 2 * 7


class OracleShard:
    """CPU stand-in for m3s.dist_ba.HipShard with the same linearize / edge_sums / solve surface."""

    def __init__(self, mode, Twc, Xs, Cs, ii, jj, idx, valid, Q, params, delta_thresh, e0, e1):
        self.mode, self.params, self.delta = mode, params, float(delta_thresh)
        self.Twc = np.array(Twc, np.float32, copy=True)
        self.Xs, self.Cs, self.idx, self.valid, self.Q = Xs, Cs, idx, valid, Q
        u = np.unique(np.concatenate((ii, jj)))  # torch.unique(cat([ii, jj])) ranks (gn_kernels.cu)
        self.ie, self.je = np.searchsorted(u, ii), np.searchsorted(u, jj)
        self.E, self.e0, self.e1 = ii.shape[0], e0, e1
        self.edge_sums = torch.zeros((self.E, ROW), dtype=torch.float64)
        self.done = False
        self.iters = 0

    def linearize(self):
        self.edge_sums.zero_()
        if self.done or self.e1 <= self.e0:
            return
        s = slice(self.e0, self.e1)
        Hs, gs = O.ba_linearize(self.mode, self.Twc, self.Xs, self.Cs, self.ie[s], self.je[s], self.idx[s],
                                self.valid[s], self.Q[s], self.params)
        n = self.e1 - self.e0
        rows = np.concatenate((Hs.transpose(1, 0, 2, 3).reshape(n, 4 * 49), gs.transpose(1, 0, 2).reshape(n, 14)), 1)
        self.edge_sums[s] = torch.from_numpy(rows)

    def solve(self):
        if self.done:
            return
        K = self.Twc.shape[0]
        n = (K - 1) * 7
        tab = self.edge_sums.numpy()
        A = np.zeros((n, n))
        b = np.zeros(n)
        for e in range(self.E):  # fixed assembly order on every rank
            io, jo = self.ie[e] - 1, self.je[e] - 1
            Hs = tab[e, :196].reshape(4, 7, 7)
            for blk, (r, c) in enumerate(((io, io), (io, jo), (jo, io), (jo, jo))):
                if r >= 0 and c >= 0:
                    A[r * 7:r * 7 + 7, c * 7:c * 7 + 7] += Hs[blk]
            if io >= 0:
                b[io * 7:io * 7 + 7] += tab[e, 196:203]
            if jo >= 0:
                b[jo * 7:jo * 7 + 7] += tab[e, 203:210]
        L = np.linalg.cholesky(A)
        dx = (-np.linalg.solve(L.T, np.linalg.solve(L, b))).astype(np.float32).reshape(K - 1, 7)
        self.Twc = O.pose_retr(self.Twc, dx, 1)
        self.iters += 1
        if float(np.sqrt((dx.astype(np.float64) ** 2).sum())) < self.delta:
            self.done = True


def _problem():
    from m3s.synthetic import make_graph, two_way

    G = make_graph(n_kf=12, H=16, W=24, loops_per_kf=1, seed=3)
    ii, jj, idx, valid, Q = two_way(G)  # global_opt.py:106-112 two-way edges
    params = O.ba_params("rays", 0.003, 10.0, 0.0, 1.5)
    return (G["Twc0"].numpy(), G["Xs"].numpy(), G["Cs"][..., 0].numpy(), ii.numpy(), jj.numpy(), idx.numpy(),
            valid[..., 0].numpy().astype(np.uint8), Q[..., 0].numpy(), params)


def _rank_main(rank, world, port, out_dir, max_iter):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from m3s.dist_ba import run_sharded, shard_range

        Twc, Xs, Cs, ii, jj, idx, valid, Q, params = _problem()
        e0, e1 = shard_range(ii.shape[0], rank, world)
        sh = OracleShard("rays", Twc, Xs, Cs, ii, jj, idx, valid, Q, params, 1e-8, e0, e1)
        run_sharded(sh, max_iter)
        np.save(os.path.join(out_dir, f"T_w{world}_r{rank}.npy"), sh.Twc)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, out_dir, max_iter):
    mp.spawn(_rank_main, args=(world, _free_port(), str(out_dir), max_iter), nprocs=world, join=True)
    return [np.load(os.path.join(out_dir, f"T_w{world}_r{r}.npy")) for r in range(world)]


@pytest.mark.timeout(300)
def test_sharded_ba_protocol_gloo_world2(tmp_path):
    max_iter = 4
    T2 = _run(2, tmp_path, max_iter)
    T1 = _run(1, tmp_path, max_iter)
    assert np.array_equal(T2[0], T2[1]), "ranks diverged"
    assert np.array_equal(T2[0], T1[0]), "2-rank result differs from 1-rank result"
    Twc, Xs, Cs, ii, jj, idx, valid, Q, params = _problem()
    Tref, _, _ = O.gauss_newton("rays", Twc, Xs, Cs, ii, jj, idx, valid, Q, params, max_iter, 1e-8)
    np.testing.assert_allclose(T2[0], Tref, atol=1e-5)
    assert not np.array_equal(T2[0], Twc), "BA did not move the poses"


class _StallShard:
    """A shard whose factor schedule stalled on rank 1 only (HipShard.stalled() == M3S_ESTALL there)."""

    def __init__(self, rank):
        self.rank = rank
        self.edge_sums = torch.zeros((4, ROW), dtype=torch.float64)

    def linearize(self):
        pass

    def solve(self):
        pass

    def stalled(self):
        return self.rank == 1


def _stall_main(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from m3s.dist_ba import run_sharded

        try:
            run_sharded(_StallShard(rank), 3)
            msg = "no error"
        except RuntimeError as e:
            msg = str(e)
        # a collective after the failed solve: no rank is left waiting for another
        t = torch.ones(1)
        dist.all_reduce(t)
        with open(os.path.join(out_dir, f"stall_r{rank}.txt"), "w") as f:
            f.write(f"{msg}|{t.item()}")
    finally:
        dist.destroy_process_group()


class _ErrorShard(_StallShard):
    """A shard whose status readback failed on rank 1 with a non-stall error (it must not raise
    before the collective)."""

    def status(self):
        return -2 if self.rank == 1 else 0


def _error_main(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from m3s.dist_ba import run_sharded

        try:
            run_sharded(_ErrorShard(rank), 2)
            msg = "no error"
        except RuntimeError as e:
            msg = str(e)
        t = torch.ones(1)
        dist.all_reduce(t)
        with open(os.path.join(out_dir, f"err_r{rank}.txt"), "w") as f:
            f.write(f"{msg}|{t.item()}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_sharded_ba_error_raises_on_every_rank(tmp_path):
    mp.spawn(_error_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        msg, tot = open(os.path.join(tmp_path, f"err_r{r}.txt")).read().split("|")
        assert "m3s error -2" in msg, f"rank {r}: {msg}"
        assert float(tot) == 2.0


@pytest.mark.timeout(120)
def test_sharded_ba_stall_raises_on_every_rank(tmp_path):
    """a stall on one rank (its loop stopped, its edge-sum rows zero) is a global decision: one MAX
    all-reduce of the flag after the loop makes every rank raise M3S_ESTALL, and the ranks stay in step."""
    mp.spawn(_stall_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        msg, tot = open(os.path.join(tmp_path, f"stall_r{r}.txt")).read().split("|")
        assert "stall" in msg, f"rank {r}: {msg}"
        assert float(tot) == 2.0
