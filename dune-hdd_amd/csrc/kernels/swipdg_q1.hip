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
// cross-check).  The sharded step's full-range launch (skip_ghost) keeps the whole-tile kernel: beside the in-place
// element pass it cost +10 % over one launch at C4 N = 8 against +22 % for the half-image kernel, whose waves fill
// every SIMD (profiles/r04/c_shard/).
hipError_t launch_q1_pwc(const AssembleArgs& a, hipStream_t s)
{
  // (ablation bit 16777216: the half-image kernel on the SKIP launch too, for the sharded-step study)
  const bool half = a.ev && !(a.variant & HDD_VARIANT_Q1_WHOLE_TILE) && (!a.skip_ghost || HDD_ABL(a, 16777216));
  if (half) return dispatch_kinds_vx<Q1PwcH2, true>(a, s, false);
  return dispatch_kinds_vx<Q1Pwc, false>(a, s, false);
}
hipError_t launch_q1_smooth(const AssembleArgs& a, hipStream_t s) { return dispatch_kinds<Q1Smooth3>(a, s, true); }

template <int TK, int KK> using Q1Pen = Q1PwcPolicy<TK, KK, true>;
hipError_t launch_q1_penalty(const AssembleArgs& a, hipStream_t s) { return dispatch_pwc<Q1Pen>(a, s); }

}  // namespace dev
}  // namespace hdd
