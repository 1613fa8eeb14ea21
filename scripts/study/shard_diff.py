"""Where a sharded schedule differs from the single-GPU assembly (debug aid for tests/test_device_transport.py):
per schedule and rank, the number of differing values, the differing owned elements, how many of them are
ghost-adjacent, and the first few (element, tile, lane) positions.
usage: python scripts/study/shard_diff.py [n] [two]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "dune-hdd_amd", "python"))
import hdd_amd as H  # noqa: E402
import test_device_transport as T  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    two = len(sys.argv) > 2 and sys.argv[2] == "two"
    grid = H.Grid.structured(H.CUBE, 3520, 1200, T.LOWER, T.UPPER, px=8, py=8)
    sched = {"default": 0, "inplace": H.SHARD_FIX_INPLACE, "serial": H.SHARD_NO_OVERLAP}
    got, infos = T.run_device_ranks(grid, n, H.TENSOR_ISO_PER_ELEM, two, sched, steps=2)
    ref = T._single_gpu(grid, H.TENSOR_ISO_PER_ELEM, two)
    # per-rank nnz ranges and element ptrs (Q1: 16 (1 + interior faces) values per element)
    bounds = np.cumsum([0] + [i.nnz for i in infos])
    for name, v in got.items():
        bad = v.view(np.int64) != ref.view(np.int64)
        print("%s: %d differing values of %d" % (name, int(bad.sum()), bad.size), flush=True)
        if not bad.any():
            continue
        for r in range(n):
            b = bad[:, bounds[r]:bounds[r + 1]].any(0)
            if not b.any():
                continue
            sh = grid.local(infos[r].s_begin, infos[r].s_end)   # the shard's local numbering
            nbr = sh.neighbors
            o0, o1 = sh.own_begin, sh.own_end
            assert o1 - o0 == infos[r].own_end - infos[r].own_begin
            nint = (nbr[:, o0:o1] >= 0).sum(0)
            ep = np.concatenate([[0], np.cumsum(16 * (1 + nint))])
            el = np.unique(np.searchsorted(ep, np.nonzero(b)[0], side="right") - 1)
            ghost_adj = ((nbr[:, o0:o1] >= 0) & ((nbr[:, o0:o1] < o0) | (nbr[:, o0:o1] >= o1))).any(0)
            tiles = np.unique(el // 64)
            full = [int((nint[t * 64:(t + 1) * 64] == 4).all()) for t in tiles[:8]]
            print("  rank %d: %d values, %d elements (%d ghost-adjacent), %d tiles; first elements %s tiles %s full %s"
                  % (r, int(b.sum()), el.size, int(ghost_adj[el].sum()), tiles.size, el[:8].tolist(),
                     tiles[:8].tolist(), full), flush=True)
            for e in el[:3]:
                row = slice(bounds[r] + ep[e], bounds[r] + ep[e + 1])
                d = np.nonzero(bad[0, row])[0]
                print("    element %d (ghost-adj %d, nint %d): %d of %d values differ, positions %s; got %s ref %s"
                      % (e, ghost_adj[e], nint[e], d.size, ep[e + 1] - ep[e], d[:10].tolist(),
                         v[0, row][d[:3]].tolist(), ref[0, row][d[:3]].tolist()), flush=True)


if __name__ == "__main__":
    main()
