// dune-hdd_amd/csrc/kernels/swipdg_q1.hip -- Q1 (parallelograms) instantiations of the persistent tile driver:
// closed-form piecewise-constant stiffness (the C1 / C4 kernel), the smooth-kappa quadrature policy, the
// SWIPDG penalty product.
#include "swipdg_device.hh"

namespace hdd {
namespace dev {

// The C1 / C4 kernel.  With the mesh's vertex-indexed geometry: the half-image kernel (two waves per SIMD, 20 KB
// image) -- C4 0.547-0.555 ms against 0.595-0.599 for the whole-tile image on element-major coords, same box
// (profiles/r04/b_sweep/).  The two waves per SIMD hide the second gather stage that made vertex-indexed
// geometry lose at one wave per SIMD (0.600 -> 0.690 ms, round 2).  Element-major meshes keep the whole-tile
// kernel (the half-image kernel on element-major coords measured 0.630 ms).
// A/B switches (HDD_DEBUG_FLAGS): 1048576 = the whole-tile kernel always, 2097152 = the half-image kernel on
// element-major coords.
// The sharded step's full-range launch (skip_ghost) keeps the whole-tile kernel: beside the in-place element pass
// it costs +10 % over one launch at C4 N = 8 against +22 % for the half-image kernel, whose waves fill every SIMD
// (profiles/r04/c_shard/; bit 16777216 selects the half-image kernel there too).
hipError_t launch_q1_pwc(const AssembleArgs& a, hipStream_t s)
{
  if (a.debug_flags & 2097152) return dispatch_kinds_vx<Q1PwcH2, false>(a, s, false);
  const bool half = a.ev && !(a.debug_flags & 1048576) && (!a.skip_ghost || (a.debug_flags & 16777216));
  if (half) return dispatch_kinds_vx<Q1PwcH2, true>(a, s, false);
  return dispatch_kinds_vx<Q1Pwc, false>(a, s, false);
}
hipError_t launch_q1_smooth(const AssembleArgs& a, hipStream_t s) { return dispatch_kinds<Q1Smooth3>(a, s, true); }

template <int TK, int KK> using Q1Pen = Q1PwcPolicy<TK, KK, true>;
hipError_t launch_q1_penalty(const AssembleArgs& a, hipStream_t s) { return dispatch_pwc<Q1Pen>(a, s); }

}  // namespace dev
}  // namespace hdd
