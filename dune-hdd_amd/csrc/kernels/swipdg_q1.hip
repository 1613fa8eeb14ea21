// dune-hdd_amd/csrc/kernels/swipdg_q1.hip -- Q1 (parallelograms) instantiations of the persistent tile driver:
// closed-form piecewise-constant stiffness (the C1 / C4 kernel), the smooth-kappa quadrature policy, the
// SWIPDG penalty product.
#include "swipdg_device.hh"

namespace hdd {
namespace dev {

// HDD_DEBUG_FLAGS bit 1048576: the half-image kernel (two waves per SIMD) instead of the whole-tile image
hipError_t launch_q1_pwc(const AssembleArgs& a, hipStream_t s)
{
  return (a.debug_flags & 1048576) ? dispatch_kinds<Q1PwcH2>(a, s, false) : dispatch_kinds<Q1Pwc>(a, s, false);
}
hipError_t launch_q1_smooth(const AssembleArgs& a, hipStream_t s) { return dispatch_kinds<Q1Smooth3>(a, s, true); }

template <int TK, int KK> using Q1Pen = Q1PwcPolicy<TK, KK, true>;
hipError_t launch_q1_penalty(const AssembleArgs& a, hipStream_t s) { return dispatch_pwc<Q1Pen>(a, s); }

}  // namespace dev
}  // namespace hdd
