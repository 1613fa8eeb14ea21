// dune-hdd_amd/csrc/kernels/swipdg_q1.hip -- Q1 (parallelograms) instantiations of the persistent tile driver:
// closed-form piecewise-constant stiffness (the C1 / C4 kernel), the smooth-kappa quadrature policy, the
// SWIPDG penalty product.
#include "swipdg_device.hh"

namespace hdd {
namespace dev {

// The C1 / C4 kernel.  With the mesh's vertex-indexed geometry: the half-image kernel (two waves per SIMD, 20 KB
// image; round 5: every element computed once at full width, swapped between the wave's halves) -- the two waves
// per SIMD hide the second gather stage that made vertex-indexed geometry lose at one wave per SIMD (0.600 -> 0.690
// ms, round 2).  Element-major meshes keep the whole-tile kernel (the half-image kernel on element-major coords
// measured 0.630 ms, round 4).  HDD_VARIANT_Q1_WHOLE_TILE: the whole-tile kernel on every mesh (the tests' bitwise
// cross-check).  The sharded step's full-range SKIP launch uses the half-image kernel too (round 5): its full tiles
// stay on the rotated image and drop the skipped elements' chunks at the store (profiles/r05/c_study/).
hipError_t launch_q1_pwc(const AssembleArgs& a, hipStream_t s)
{
  const bool half = a.ev && !(a.variant & HDD_VARIANT_Q1_WHOLE_TILE);
  if (half) return dispatch_kinds_vx<Q1PwcH2, true>(a, s, false);
  return dispatch_kinds_vx<Q1Pwc, false>(a, s, false);
}
hipError_t launch_q1_smooth(const AssembleArgs& a, hipStream_t s) { return dispatch_kinds<Q1Smooth3>(a, s, true); }

// The sharded Q1 step's side buffer into place (after the join): one wave per listed element writes the element's
// CSR row block contiguously (lane = CSR position), fetching each value from the value-major buffer the element
// pass wrote in canonical order (list_elements == 4: value k = row i, block b, column c at k fix_ld + list entry).
// The inverse of the block placement -- which canonical (b, c) a CSR position holds -- is recomputed from the
// element's neighbour ids and face info (Q1PwcPolicy::positions / role_slot).
__global__ void __launch_bounds__(64) fix_scatter_q1_kernel(const double* __restrict__ buf, int64_t ld,
                                                            const int32_t* __restrict__ list, int64_t n,
                                                            const int64_t* __restrict__ elem_ptr,
                                                            const int32_t* __restrict__ nbrs,
                                                            const uint32_t* __restrict__ finfo, int64_t n_local,
                                                            int64_t own_begin, double* vals)
{
  for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const int64_t el = list[i], e = own_begin + el;
    int32_t nb[4];
    int pf[4], nint = 0;   // (the own block: every CSR block no face claims)
#pragma unroll
    for (int f = 0; f < 4; ++f) nb[f] = nbrs[f * n_local + e];
    const uint32_t fi = finfo[e];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      nint += nb[f] >= 0;
      int p = (e < nb[f]) ? 1 : 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) p += (nb[q] >= 0 && nb[q] < nb[f]);
      pf[f] = p;
    }
    const int rowlen = 4 * (1 + nint);
    const int64_t b0 = elem_ptr[el];
    for (int p = threadIdx.x; p < 4 * rowlen; p += 64) {
      const int row = p / rowlen, q = p - row * rowlen, blk = q >> 2, col = q & 3;
      int k = row * 20 + col;   // the element's own block
#pragma unroll
      for (int f = 0; f < 4; ++f)
        if (nb[f] >= 0 && pf[f] == blk) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (role_slot<Cube>(fi, f, r) == col) k = row * 20 + (1 + f) * 4 + r;
        }
      vals[b0 + p] = buf[int64_t(k) * ld + i];
    }
  }
}

hipError_t launch_q1_scatter_soa(const AssembleArgs& a, const double* buf, int64_t ld, double* vals, hipStream_t s)
{
  if (a.n_tile_list <= 0) return hipSuccess;
  const unsigned grid = unsigned(std::min<int64_t>(a.n_tile_list, int64_t(a.n_cu) * 8));
  hipLaunchKernelGGL(fix_scatter_q1_kernel, dim3(grid), dim3(64), 0, s, buf, ld, a.tile_list, a.n_tile_list, a.elem_ptr,
                     a.nbrs, a.finfo, a.n_local, a.own_begin, vals);
  return hipGetLastError();
}

template <int TK, int KK> using Q1Pen = Q1PwcPolicy<TK, KK, true>;
hipError_t launch_q1_penalty(const AssembleArgs& a, hipStream_t s) { return dispatch_pwc<Q1Pen>(a, s); }

}  // namespace dev
}  // namespace hdd
