// dune-hdd_amd/csrc/kernels/swipdg_assemble.hip -- dispatch of the SWIPDG stiffness / product kernels
// (swipdg_device.hh) and the wave-per-row fallback kernels for the remaining quadrature rules.
#include "swipdg_device.hh"

namespace hdd {
namespace dev {

// one launch per component: components of one call may differ in kind (affine part const, component
// per-element, ...) -- the kinds are compile-time inside the kernels
static hipError_t launch_components(const AssembleArgs& a, int nqv, int nqf, hipStream_t s, bool* supported)
{
  // C3: sinusoid components sharing one phase (OS2014's affine part and mu-component) -> one fused launch that
  // evaluates the sines once per element (P1, vertex-indexed geometry; HDD_VARIANT_C3_PER_COMPONENT: per component)
  if (a.elem_type == HDD_SIMPLEX && nqv == 6 && nqf == 3 && a.ev && a.n_comp > 1 &&
      !(a.variant & HDD_VARIANT_C3_PER_COMPONENT)) {
    bool same = true;
    for (int c = 0; c < a.n_comp; ++c)
      same = same && a.kappa[c].kind == HDD_FN_SINUSOID && a.kappa[c].kx == a.kappa[0].kx &&
             a.kappa[c].ky == a.kappa[0].ky;
    if (same) return launch_p1_smooth_fused(a, s);
  }
  for (int c = 0; c < a.n_comp; ++c) {
    AssembleArgs ac = a;
    ac.n_comp = 1;
    ac.kappa[0] = a.kappa[c];
    ac.vals[0] = a.vals[c];
    const bool smooth = smooth_kind(ac.kappa[0].kind);
    hipError_t e = hipSuccess;
    if (ac.elem_type == HDD_SIMPLEX && nqv == 1 && nqf == 2 && !smooth) e = launch_p1_pwc(ac, s);
    else if (ac.elem_type == HDD_SIMPLEX && nqv == 6 && nqf == 3 && smooth) e = launch_p1_smooth(ac, s);
    else if (ac.elem_type == HDD_CUBE && nqv == 1 && nqf == 2 && !smooth) e = launch_q1_pwc(ac, s);
    else if (ac.elem_type == HDD_CUBE && nqv == 4 && nqf == 3 && smooth) e = launch_q1_smooth(ac, s);
    else {
      *supported = false;
      return hipSuccess;
    }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// ------------------------------------------------------------------------------------------------
// products (hdd_product_assemble) on the persistent driver: P1 / Q1 with piecewise-constant kappa; the
// caller falls back to the generic product kernel (rhs.hip) for smooth kappa and hexahedra
// ------------------------------------------------------------------------------------------------
hipError_t launch_product_fast(const AssembleArgs& a, int product, hipStream_t s, bool* supported)
{
  *supported = true;
  const int kk = a.kappa[0].kind;
  const bool uses_kappa = product == HDD_PRODUCT_ELLIPTIC || product == HDD_PRODUCT_PENALTY;
  if ((uses_kappa && kk != HDD_FN_CONST && kk != HDD_FN_PER_ELEM) ||
      (a.elem_type != HDD_SIMPLEX && a.elem_type != HDD_CUBE)) {
    *supported = false;
    return hipSuccess;
  }
  if (product != HDD_PRODUCT_PENALTY) return launch_vol_products(a, product, s);
  return a.elem_type == HDD_SIMPLEX ? launch_p1_penalty(a, s) : launch_q1_penalty(a, s);
}

int volume_points(int elem_type, int order)
{
  if (elem_type == HDD_SIMPLEX) return order <= 1 ? 1 : (order == 2 ? 3 : (order <= 4 ? 6 : -1));
  const int n = (order + 2) / 2;
  return n <= 3 ? n * n : -1;
}
int face_points(int order)
{
  const int n = (order + 2) / 2;
  return n <= 3 ? n : -1;
}

hipError_t launch_assemble(const AssembleArgs& a, int nqv, int nqf, hipStream_t s, bool* supported)
{
  *supported = true;
  if (!(a.variant & HDD_VARIANT_WAVE_PER_ROW)) {
    const hipError_t e = launch_components(a, nqv, nqf, s, supported);
    if (*supported || a.tile_list || a.skip_ghost) return e;
    *supported = true;   // fall through to the wave-per-row kernels for the remaining rules
  }
  if (a.tile_list || a.skip_ghost) {   // (the wave-per-row kernels take neither lists nor skipped elements)
    *supported = false;
    return hipSuccess;
  }
  bool pwc = true;
  for (int c = 0; c < a.n_comp; ++c) pwc &= !smooth_kind(a.kappa[c].kind);
  if (a.elem_type == HDD_SIMPLEX) {
    if (nqv == 1 && nqf == 2) return pwc ? launch_t<Simplex, 1, 2, true>(a, s) : launch_t<Simplex, 1, 2, false>(a, s);
    if (nqv == 6 && nqf == 3) return launch_t<Simplex, 6, 3, false>(a, s);
    if (nqv == 3 && nqf == 2) return launch_t<Simplex, 3, 2, false>(a, s);
    if (nqv == 3 && nqf == 3) return launch_t<Simplex, 3, 3, false>(a, s);   // smooth kappa of order 2
  } else {
    if (nqv == 1 && nqf == 2) return launch_t<Cube, 1, 2, false>(a, s);
    if (nqv == 4 && nqf == 3) return launch_t<Cube, 4, 3, false>(a, s);
    if (nqv == 4 && nqf == 2) return launch_t<Cube, 4, 2, false>(a, s);
  }
  *supported = false;
  return hipSuccess;
}

}  // namespace dev
}  // namespace hdd
