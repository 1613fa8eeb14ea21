// dune-hdd_amd/csrc/kernels/swipdg_vol.hip -- element-local products (l2, h1_semi, elliptic, boundary_l2) of
// P1 / Q1 meshes with piecewise-constant data on the persistent tile driver (VolProductPolicy).
#include "swipdg_device.hh"

namespace hdd {
namespace dev {

template <class E, int KIND, int VX>
static hipError_t launch_vol_product_vx(const AssembleArgs& a, hipStream_t s)
{
  if constexpr (KIND != HDD_PRODUCT_ELLIPTIC) {
    return launch_persistent<VolProductPolicy<E, KIND, HDD_TENSOR_CONST, HDD_FN_CONST, VX>>(a, s);
  } else {
    const bool pe = a.kappa[0].kind == HDD_FN_PER_ELEM;
    if (a.tkind == HDD_TENSOR_CONST)
      return pe ? launch_persistent<VolProductPolicy<E, KIND, HDD_TENSOR_CONST, HDD_FN_PER_ELEM, VX>>(a, s)
                : launch_persistent<VolProductPolicy<E, KIND, HDD_TENSOR_CONST, HDD_FN_CONST, VX>>(a, s);
    if (a.tkind == HDD_TENSOR_ISO_PER_ELEM)
      return pe ? launch_persistent<VolProductPolicy<E, KIND, HDD_TENSOR_ISO_PER_ELEM, HDD_FN_PER_ELEM, VX>>(a, s)
                : launch_persistent<VolProductPolicy<E, KIND, HDD_TENSOR_ISO_PER_ELEM, HDD_FN_CONST, VX>>(a, s);
    return pe ? launch_persistent<VolProductPolicy<E, KIND, HDD_TENSOR_SYM_PER_ELEM, HDD_FN_PER_ELEM, VX>>(a, s)
              : launch_persistent<VolProductPolicy<E, KIND, HDD_TENSOR_SYM_PER_ELEM, HDD_FN_CONST, VX>>(a, s);
  }
}

template <class E, int KIND>
static hipError_t launch_vol_product(const AssembleArgs& a, hipStream_t s)
{
  if constexpr (std::is_same_v<E, Simplex>)
    if (a.ev) return launch_vol_product_vx<E, KIND, 1>(a, s);
  return launch_vol_product_vx<E, KIND, 0>(a, s);
}


hipError_t launch_vol_products(const AssembleArgs& a, int product, hipStream_t s)
{
  const bool tri = a.elem_type == HDD_SIMPLEX;
  switch (product) {
    case HDD_PRODUCT_L2:
      return tri ? launch_vol_product<Simplex, HDD_PRODUCT_L2>(a, s) : launch_vol_product<Cube, HDD_PRODUCT_L2>(a, s);
    case HDD_PRODUCT_H1_SEMI:
      return tri ? launch_vol_product<Simplex, HDD_PRODUCT_H1_SEMI>(a, s)
                 : launch_vol_product<Cube, HDD_PRODUCT_H1_SEMI>(a, s);
    case HDD_PRODUCT_ELLIPTIC:
      return tri ? launch_vol_product<Simplex, HDD_PRODUCT_ELLIPTIC>(a, s)
                 : launch_vol_product<Cube, HDD_PRODUCT_ELLIPTIC>(a, s);
    default:
      return tri ? launch_vol_product<Simplex, HDD_PRODUCT_BOUNDARY_L2>(a, s)
                 : launch_vol_product<Cube, HDD_PRODUCT_BOUNDARY_L2>(a, s);
  }
}

}  // namespace dev
}  // namespace hdd
