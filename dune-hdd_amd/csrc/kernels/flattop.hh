// dune-hdd_amd/csrc/kernels/flattop.hh -- HDD_FN_FLATTOP: c + b * sum_k v_k phi_k(x) phi_k(y), the sum of
// dune-stuff FlatTop functions that Spe10::Model1 builds its channel from when channel_boundary_layer != 0
// (problems/spe10.hh:139-148, 213-222).  FlatTop is third-party (dune-stuff, absent here): this is the
// restated Brenner-Scott flat-top, per coordinate 1 on [l + d, u - d], 0 outside [l - d, u + d] and the C^1
// cubic transitions (1 + t)^2 (1 - 2t), t = (x - (l + d)) / 2d in [-1, 0), and (1 - t)^2 (1 + 2t),
// t = (x - (u - d)) / 2d in [0, 1) -- parity against oracle/swipdg_oracle.c's restatement, unpinned.
// Box record (HDD_FLATTOP_REC doubles): lx, ly, ux, uy, dx, dy, value.
#pragma once
#include <hip/hip_runtime.h>

#include "hdd.h"

namespace hdd {
namespace dev {

__device__ __forceinline__ double flattop_1d(double x, double l, double u, double d)
{
  const double tl = (x - (l + d)) / (2.0 * d);
  const double tr = (x - (u - d)) / (2.0 * d);
  const double vl = (1.0 + tl) * (1.0 + tl) * (1.0 - 2.0 * tl);
  const double vr = (1.0 - tr) * (1.0 - tr) * (1.0 + 2.0 * tr);
  return x < l - d ? 0.0 : (x < l + d ? vl : (x < u - d ? 1.0 : (x < u + d ? vr : 0.0)));
}

// The boxes are wave-uniform data (scalar loads); a box no active lane's point reaches is skipped by a
// wave-uniform branch, so a tile pays only for the few channel boxes near it.  Summation order = box order
// (skipped boxes add exact zeros in the restatement).
__device__ __forceinline__ double flattop_sum(const double* table, int n, double c, double b, double x, double y)
{
  double s = 0.0;
  for (int k = 0; k < n; ++k) {
    const double* r = table + HDD_FLATTOP_REC * k;
    const double lx = r[0], ly = r[1], ux = r[2], uy = r[3], dx = r[4], dy = r[5];
    const bool near = x >= lx - dx && x < ux + dx && y >= ly - dy && y < uy + dy;
    if (!__any(near)) continue;
    s += r[6] * flattop_1d(x, lx, ux, dx) * flattop_1d(y, ly, uy, dy);
  }
  return c + b * s;
}

}  // namespace dev
}  // namespace hdd
