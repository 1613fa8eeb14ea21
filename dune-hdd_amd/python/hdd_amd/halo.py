"""Face-halo exchange of a sharded (Block)SWIPDG assembly.

Each rank owns a contiguous range of subdomains (block-swipdg.hh:355-382: the owner of subdomain ss writes
A_ss and A_ss,nn) and assembles only its own rows.  The rows need the element records (vertex coordinates,
diffusion tensor, per-element coefficients) of the face neighbours owned by other ranks: those ghost
columns are filled here by a pack (hdd_soa_gather) -> RCCL send/recv (torch.distributed, backend "nccl"
is RCCL on ROCm, point-to-point over xGMI) -> unpack (hdd_soa_scatter) sequence.  No reduction is ever
needed (rows are owned), so there is no all-reduce on the data path.
"""
import numpy as np

from . import Comm, soa_gather, soa_scatter


def gloo_host_comm(device=0, group=None):
    """hdd_comm host transport over torch.distributed point-to-point (gloo: host tensors).  The C++ step
    (hdd_block_assemble_sharded) stages the halo through pinned host memory and calls this synchronously --
    the rehearsal transport for several ranks on one GPU, where RCCL refuses duplicate devices."""
    import torch
    import torch.distributed as dist

    def exchange(peers, sends, recvs):
        ops = []
        for p, sv, rv in zip(peers, sends, recvs):
            if sv.size:
                ops.append(dist.P2POp(dist.isend, torch.from_numpy(sv), p, group=group))
            if rv.size:
                ops.append(dist.P2POp(dist.irecv, torch.from_numpy(rv), p, group=group))
        for r in (dist.batch_isend_irecv(ops) if ops else []):
            r.wait()

    return Comm.host(exchange, device)


def rccl_comm(rank, world, device, group=None):
    """hdd_comm over RCCL (one GPU per rank): rank 0's ncclUniqueId is broadcast over the (gloo) control
    group, then every rank runs ncclCommInitRank inside the library."""
    import torch.distributed as dist
    obj = [Comm.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return Comm.rccl(obj[0], world, rank, device)


class HaloExchange:
    """arrays: list of (device tensor [rows][n_local] contiguous, rows).  owner: subdomain -> rank map."""

    def __init__(self, ctx, local, arrays, owner, rank, host_staging=False):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.ctx = ctx
        self.local = local
        self.arrays = [a for a, _ in arrays]
        self.rows = [int(r) for _, r in arrays]
        self.total_rows = sum(self.rows)
        self.ld = local.n_local
        self.host_staging = host_staging
        dev = self.arrays[0].device
        self.plan = local.halo_plan(owner, rank)
        self.peers = []
        for p in self.plan:
            send_idx = torch.from_numpy(p["send"]).to(dev)
            sbuf = torch.empty((self.total_rows, len(p["send"])), dtype=torch.float64, device=dev)
            rbuf = torch.empty((self.total_rows, p["recv_count"]), dtype=torch.float64, device=dev)
            hs = hr = None
            if host_staging:
                hs = torch.empty(sbuf.shape, dtype=torch.float64)
                hr = torch.empty(rbuf.shape, dtype=torch.float64)
            self.peers.append(dict(peer=p["peer"], idx=send_idx, sbuf=sbuf, rbuf=rbuf, off=p["recv_offset"],
                                   n_recv=p["recv_count"], hs=hs, hr=hr))

    @property
    def halo_bytes(self):
        return sum(8 * self.total_rows * (p["idx"].numel() + p["n_recv"]) for p in self.peers)

    def pack(self, p):
        soa_gather(self.ctx, self.arrays, self.rows, self.ld, p["idx"], p["sbuf"])

    def unpack(self, p):
        soa_scatter(self.ctx, self.arrays, self.rows, self.ld, p["off"], p["n_recv"], p["rbuf"])

    def start(self):
        """Pack the send lists and post the RCCL send/recv.  Device work queued on the current stream after
        this call (the interior tiles) overlaps the transfer; finish() orders the stream after it."""
        dist = self.dist
        for p in self.peers:
            if p["idx"].numel():
                self.pack(p)
        ops = []
        if self.host_staging:      # gloo rehearsal: host-staged and synchronous, nothing to overlap
            for p in self.peers:
                p["hs"].copy_(p["sbuf"])
            for p in self.peers:
                ops.append(dist.P2POp(dist.isend, p["hs"], p["peer"]))
                ops.append(dist.P2POp(dist.irecv, p["hr"], p["peer"]))
            for r in dist.batch_isend_irecv(ops):
                r.wait()
            for p in self.peers:
                p["rbuf"].copy_(p["hr"])
            self.pending = []
            return
        for p in self.peers:
            ops.append(dist.P2POp(dist.isend, p["sbuf"], p["peer"]))
            ops.append(dist.P2POp(dist.irecv, p["rbuf"], p["peer"]))
        self.pending = dist.batch_isend_irecv(ops) if ops else []

    def finish(self):
        """Make the current stream wait for the transfer (no host block for RCCL) and unpack the ghosts."""
        for r in self.pending:
            r.wait()
        self.pending = []
        for p in self.peers:
            if p["n_recv"]:
                self.unpack(p)

    def exchange(self):
        self.start()
        self.finish()


def strip_owner(n_sub, world):
    """subdomain -> rank for `world` ranks owning contiguous, near-equal subdomain ranges."""
    own = np.empty(n_sub, np.int32)
    for r in range(world):
        a, b = (r * n_sub) // world, ((r + 1) * n_sub) // world
        own[a:b] = r
    return own
