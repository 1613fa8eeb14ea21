// dune-hdd_amd/csrc/kernels/swipdg_kernels.hh -- kernel argument blocks shared by the ABI and the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hdd.h"

namespace hdd {
namespace dev {

struct KappaArg {
  int32_t kind, order;
  double c, b, kx, ky;
  const double* per_elem;
};

struct AssembleArgs {
  int32_t elem_type, n_comp;
  int64_t n_local, own_begin, own_end;
  const double* coords;
  const int32_t* nbrs;
  const uint32_t* finfo;
  const int64_t* elem_ptr;
  int32_t tkind, pad;
  double tc0, tc1, tc2;
  const double* tper;
  double sigma_inner, sigma_boundary, beta;
  int32_t debug_flags, pad2;   // ablation switches (HDD_DEBUG_FLAGS), 0 in production
  const int32_t* tile_list;    // optional: 64-element tiles to assemble (relative to own_begin)
  int64_t n_tile_list;         // entries of tile_list (tile_list == nullptr: all tiles)
  KappaArg kappa[HDD_MAX_COMP];
  double* vals[HDD_MAX_COMP];
};

int volume_points(int elem_type, int order);
int face_points(int order);
hipError_t launch_assemble(const AssembleArgs& a, int nqv, int nqf, hipStream_t s, bool* supported);

}  // namespace dev
}  // namespace hdd
