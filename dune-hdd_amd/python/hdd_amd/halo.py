"""Transports for the face halo of a sharded (Block)SWIPDG assembly.

Each rank owns a contiguous range of subdomains (block-swipdg.hh:355-382: the owner of subdomain ss writes
A_ss and A_ss,nn) and assembles only its own rows; the C++ step hdd_block_assemble_sharded packs the element
records the peers need, moves them through an hdd_comm and receives them straight into the ghost columns.
No reduction is ever needed (rows are owned), so there is no all-reduce on the data path.  This module only
builds the communicators: RCCL (one GPU per rank, the production path) or a gloo host transport (rehearsal
of several ranks on one GPU, where RCCL refuses duplicate devices).
"""
import numpy as np

from . import Comm


def gloo_host_comm(device=0, group=None):
    """hdd_comm host transport over torch.distributed point-to-point (gloo: host tensors).  The C++ step
    (hdd_block_assemble_sharded) stages the halo through pinned host memory and calls this synchronously --
    the rehearsal transport for several ranks on one GPU, where RCCL refuses duplicate devices."""
    import torch
    import torch.distributed as dist

    def exchange(peers, sends, recvs):
        # the step posts several messages per peer (one per halo row, in the same order on both sides):
        # one gloo message per peer carries them concatenated, split again on arrival
        order, by = [], {}
        for p, sv, rv in zip(peers, sends, recvs):
            if p not in by:
                by[p] = ([], [])
                order.append(p)
            by[p][0].append(sv)
            by[p][1].append(rv)
        ops, inbox = [], []
        for p in order:
            sv = np.concatenate(by[p][0]) if by[p][0] else np.empty(0)
            rbuf = torch.empty(sum(r.size for r in by[p][1]), dtype=torch.float64)
            inbox.append((p, rbuf))
            if sv.size:
                ops.append(dist.P2POp(dist.isend, torch.from_numpy(np.ascontiguousarray(sv)), p, group=group))
            if rbuf.numel():
                ops.append(dist.P2POp(dist.irecv, rbuf, p, group=group))
        for r in (dist.batch_isend_irecv(ops) if ops else []):
            r.wait()
        for p, rbuf in inbox:
            off, flat = 0, rbuf.numpy()
            for rv in by[p][1]:
                rv[:] = flat[off:off + rv.size]
                off += rv.size

    return Comm.host(exchange, device)


def rccl_comm(rank, world, device, group=None):
    """hdd_comm over RCCL (one GPU per rank): rank 0's ncclUniqueId is broadcast over the (gloo) control
    group, then every rank runs ncclCommInitRank inside the library."""
    import torch.distributed as dist
    obj = [Comm.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return Comm.rccl(obj[0], world, rank, device)


def strip_owner(n_sub, world):
    """subdomain -> rank for `world` ranks owning contiguous, near-equal subdomain ranges."""
    own = np.empty(n_sub, np.int32)
    for r in range(world):
        a, b = (r * n_sub) // world, ((r + 1) * n_sub) // world
        own[a:b] = r
    return own
