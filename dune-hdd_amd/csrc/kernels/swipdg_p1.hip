// dune-hdd_amd/csrc/kernels/swipdg_p1.hip -- P1 (triangles) instantiations of the persistent tile driver:
// closed-form piecewise-constant stiffness (the C2 kernel), the smooth-kappa moments policy (C3), the
// SWIPDG penalty product.
#include "swipdg_device.hh"

namespace hdd {
namespace dev {

static hipError_t dispatch_smooth_p1(const AssembleArgs& a, hipStream_t s)
{
  if (a.variant & HDD_VARIANT_P1_SMOOTH_QUADRATURE) return dispatch_kinds<P1Smooth3>(a, s, true);
  const int tk = a.tkind;
  if (a.kappa[0].kind == HDD_FN_FLATTOP) {   // (the SPE10 FlatTop channel: not a BASELINE kernel, VX only)
    if (!a.ev) return dispatch_kinds<P1Smooth3>(a, s, true);
    if (tk == HDD_TENSOR_CONST) return launch_persistent<P1SmoothPolicy<HDD_TENSOR_CONST, true, HDD_FN_FLATTOP>>(a, s);
    if (tk == HDD_TENSOR_ISO_PER_ELEM)
      return launch_persistent<P1SmoothPolicy<HDD_TENSOR_ISO_PER_ELEM, true, HDD_FN_FLATTOP>>(a, s);
    return launch_persistent<P1SmoothPolicy<HDD_TENSOR_SYM_PER_ELEM, true, HDD_FN_FLATTOP>>(a, s);
  }
  if (a.ev) {
    if (tk == HDD_TENSOR_CONST) return launch_persistent<P1SmoothPolicy<HDD_TENSOR_CONST, true>>(a, s);
    if (tk == HDD_TENSOR_ISO_PER_ELEM) return launch_persistent<P1SmoothPolicy<HDD_TENSOR_ISO_PER_ELEM, true>>(a, s);
    return launch_persistent<P1SmoothPolicy<HDD_TENSOR_SYM_PER_ELEM, true>>(a, s);
  }
  if (tk == HDD_TENSOR_CONST) return launch_persistent<P1SmoothPolicy<HDD_TENSOR_CONST>>(a, s);
  if (tk == HDD_TENSOR_ISO_PER_ELEM) return launch_persistent<P1SmoothPolicy<HDD_TENSOR_ISO_PER_ELEM>>(a, s);
  return launch_persistent<P1SmoothPolicy<HDD_TENSOR_SYM_PER_ELEM>>(a, s);
}

hipError_t launch_p1_pwc(const AssembleArgs& a, hipStream_t s) { return dispatch_kinds<P1Pwc>(a, s, false); }
hipError_t launch_p1_smooth(const AssembleArgs& a, hipStream_t s) { return dispatch_smooth_p1(a, s); }
// two components (OS2014, C3): both emitted in one pass over the geometry (P1SmoothFusedPolicy<.., TWO>); tile lists
// and the sharded SKIP launch included.  More components: one image, emitted one after the other.
hipError_t launch_p1_smooth_fused(const AssembleArgs& a, hipStream_t s)
{
  const int tk = a.tkind;
  if (a.n_comp == 2) {
    if (tk == HDD_TENSOR_CONST) return launch_persistent<P1SmoothFusedPolicy<HDD_TENSOR_CONST, true, true>>(a, s);
    if (tk == HDD_TENSOR_ISO_PER_ELEM)
      return launch_persistent<P1SmoothFusedPolicy<HDD_TENSOR_ISO_PER_ELEM, true, true>>(a, s);
    return launch_persistent<P1SmoothFusedPolicy<HDD_TENSOR_SYM_PER_ELEM, true, true>>(a, s);
  }
  if (tk == HDD_TENSOR_CONST) return launch_persistent<P1SmoothFusedPolicy<HDD_TENSOR_CONST, true>>(a, s);
  if (tk == HDD_TENSOR_ISO_PER_ELEM) return launch_persistent<P1SmoothFusedPolicy<HDD_TENSOR_ISO_PER_ELEM, true>>(a, s);
  return launch_persistent<P1SmoothFusedPolicy<HDD_TENSOR_SYM_PER_ELEM, true>>(a, s);
}

template <int TK, int KK> using P1Pen = P1PwcPolicy<TK, KK, true>;
template <int TK, int KK> using P1PenVX = P1PwcPolicy<TK, KK, true, 1>;
hipError_t launch_p1_penalty(const AssembleArgs& a, hipStream_t s)
{
  return a.ev ? dispatch_pwc<P1PenVX>(a, s) : dispatch_pwc<P1Pen>(a, s);   // vertex-indexed geometry as the stiffness
}

}  // namespace dev
}  // namespace hdd
