"""world_size-2 gloo tests of the N>1 path on CPU.

The multi-GPU path (gol_runtime.cpp one_step/exchange, bench.py) cuts the
global grid into row slabs with gol_slab_plan, and every k generations sends
each slab's first/last k rows to rank-1/rank+1 and receives the neighbours'
edge rows into k-row halos (ncclSend/ncclRecv on the GPU).  Here the same
protocol runs over torch.distributed gloo between two CPU processes, with the
oracle standing in for the kernel, and the gathered result must equal the
single-grid oracle — i.e. the decomposition, halo depth and dead outer edges
are right for every k.  The bench's control-plane steps (RCCL unique-id
broadcast, max-over-ranks timing) are exercised the same way.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import golcpu as g


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _slab_protocol(rank, world, port, rows, cols, k, gens, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from mpi_amd import golhip
        r0, H = golhip.slab_plan(rows, world, rank)
        # storage: k halo rows, H slab rows, k halo rows (zero = dead outside the grid)
        buf = np.zeros((H + 2 * k, cols), np.uint8)
        buf[k:k + H] = g.init_dead(H, cols, seed, row0=r0, full_cols=cols)
        done = 0
        while done < gens:
            kk = min(k, gens - done)
            ops = []
            up_recv = torch.zeros((kk, cols), dtype=torch.uint8)
            dn_recv = torch.zeros((kk, cols), dtype=torch.uint8)
            if rank > 0:
                ops.append(dist.P2POp(dist.isend, torch.from_numpy(buf[k:k + kk].copy()), rank - 1))
                ops.append(dist.P2POp(dist.irecv, up_recv, rank - 1))
            if rank < world - 1:
                ops.append(dist.P2POp(dist.isend, torch.from_numpy(buf[k + H - kk:k + H].copy()), rank + 1))
                ops.append(dist.P2POp(dist.irecv, dn_recv, rank + 1))
            for r in (dist.batch_isend_irecv(ops) if ops else []):
                r.wait()
            buf[k - kk:k] = up_recv.numpy()
            buf[k + H:k + H + kk] = dn_recv.numpy()
            # kk generations on slab + halos; rows beyond the global grid stay dead
            lo = 0 if rank > 0 else k
            hi = H + 2 * k if rank < world - 1 else k + H
            win = buf[lo:hi]
            win = g.run(win, kk, g.DEAD)
            new = np.zeros_like(buf)
            new[lo:hi] = win
            # only the slab rows are kept (the halo rows' results are outside the light cone)
            buf[k:k + H] = new[k:k + H]
            buf[:k] = 0
            buf[k + H:] = 0
            done += kk
        # bench control plane: max over ranks, uid broadcast
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        blob = [bytes(range(128)) if rank == 0 else None]
        dist.broadcast_object_list(blob, src=0)
        parts = [None] * world
        dist.all_gather_object(parts, (r0, buf[k:k + H].copy()))
        if rank == 0:
            q.put((parts, float(t.item()), blob[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("rows,cols,k,gens", [(64, 80, 1, 9), (64, 80, 4, 13), (97, 70, 8, 24), (40, 33, 3, 7)])
def test_row_slab_halo_protocol_world2(rows, cols, k, gens):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slab_protocol, args=(r, 2, port, rows, cols, k, gens, 1, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts, tmax, blob = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.zeros((rows, cols), np.uint8)
    for r0, slab in parts:
        got[r0:r0 + slab.shape[0]] = slab
    ref = g.run(g.init_dead(rows, cols, 1), gens, g.DEAD)
    assert (got == ref).all()
    assert tmax == 2.0 and blob == bytes(range(128))
