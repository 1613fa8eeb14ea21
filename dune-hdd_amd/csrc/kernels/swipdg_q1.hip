// dune-hdd_amd/csrc/kernels/swipdg_q1.hip -- Q1 (parallelograms) instantiations of the persistent tile driver:
// closed-form piecewise-constant stiffness (the C1 / C4 kernel), the smooth-kappa quadrature policy, the
// SWIPDG penalty product.
#include "swipdg_device.hh"

namespace hdd {
namespace dev {

// HDD_DEBUG_FLAGS bit 1048576: the half-image kernel (two waves per SIMD) instead of the whole-tile image;
// + bit 2097152: with the vertex-indexed geometry (mesh elem_vertices / vertex_coords)
hipError_t launch_q1_pwc(const AssembleArgs& a, hipStream_t s)
{
  if (!(a.debug_flags & 1048576)) return dispatch_kinds<Q1Pwc>(a, s, false);
  if ((a.debug_flags & 2097152) && a.ev) return dispatch_kinds_vx<Q1PwcH2, true>(a, s, false);
  return dispatch_kinds_vx<Q1PwcH2, false>(a, s, false);
}
hipError_t launch_q1_smooth(const AssembleArgs& a, hipStream_t s) { return dispatch_kinds<Q1Smooth3>(a, s, true); }

template <int TK, int KK> using Q1Pen = Q1PwcPolicy<TK, KK, true>;
hipError_t launch_q1_penalty(const AssembleArgs& a, hipStream_t s) { return dispatch_pwc<Q1Pen>(a, s); }

}  // namespace dev
}  // namespace hdd
