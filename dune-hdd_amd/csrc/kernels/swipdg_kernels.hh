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
  const double* table;   // HDD_FN_FLATTOP boxes [n_table][HDD_FLATTOP_REC] (flattop.hh)
  int32_t n_table, pad;
};
// smooth (evaluated at quadrature points) diffusion-factor kinds
__host__ __device__ constexpr bool smooth_kind(int k) { return k == HDD_FN_SINUSOID || k == HDD_FN_FLATTOP; }

struct AssembleArgs {
  int32_t elem_type, n_comp;
  int64_t n_local, own_begin, own_end;
  const double* coords;
  const int32_t* nbrs;
  const uint32_t* finfo;
  const int64_t* elem_ptr;
  int32_t tkind, n_cu;         // n_cu: compute units of the device (cached in hdd_ctx)
  double tc0, tc1, tc2;
  const double* tper;
  double sigma_inner, sigma_boundary, beta;
  int32_t debug_flags, wgcu;   // ablation switches (HDD_ABLATION builds only); wgcu: tiles per CU override (0: policy default)
  uint32_t variant;            // HDD_VARIANT_* verification variants (hdd_ctx_set_variant; 0: the default kernels)
  int32_t pad_v;
  const int32_t* tile_list;    // optional: 64-element tiles to assemble (relative to own_begin)
  int64_t n_tile_list;         // entries of tile_list (tile_list == nullptr: all tiles)
  int32_t list_elements;       // 1: tile_list holds single owned elements (relative to own_begin), not tiles;
                               // 2: the same, row blocks into side buffers vals[c] of fix_rb doubles per element;
                               // 3: the same, in place without LDS (beside a skip_ghost assembly)
  int32_t fix_rb;
  int64_t fix_ld;              // list_elements == 4: leading dimension of the value-major side buffers
  int32_t skip_ghost;          // 1: tiles do not store the row blocks of elements with a ghost face neighbour
  int32_t reserve_wg;          // skip_ghost launches: workgroup slots left free for the concurrent element pass
  const int32_t* ev;           // optional vertex-indexed geometry: element -> local vertex ids [nvpe][n_local]
  const double* vxy;           //   and the vertex coordinates [n_vertices][2] (hdd_mesh elem_vertices / vertex_coords)
  KappaArg kappa[HDD_MAX_COMP];
  double* vals[HDD_MAX_COMP];
};

// ---------------------------------------------------------------------------------------------
// Q_p on affine hexahedra (HDD_HEX): 1D reference tables of the tensor-product basis / quadrature
// (host-computed, passed by value), one launch per affine component.
// ---------------------------------------------------------------------------------------------
struct HexTables {
  double sv[8], wv[8];          // volume Gauss-Legendre points / weights on [0,1]
  double sf[8], wf[8];          // face rule
  double Lv[4][8], Dv[4][8];    // L_k(sv_q), L_k'(sv_q): equidistant Lagrange polynomials of degree p
  double Lf[4][8], Df[4][8];    // at the face points
  double Le[4][2], De[4][2];    // at 0 and 1 (face planes)
};

struct HexArgs {
  int64_t n_local, own_begin, own_end;
  const double* coords;         // [24][n_local]
  const int32_t* nbrs;          // [6][n_local]
  const int64_t* elem_ptr;      // [n_own+1]
  int32_t tkind, kkind;
  double tc[6];
  const double* tper;           // ISO [n_local] / SYM [6][n_local]
  double kc, kb, kx, ky;
  const double* kper;
  double* vals;
  double sigma_inner, sigma_boundary, beta;
  double* ws;                   // p=3 register kernel: per-element coefficient records [n_own][HEX_REC]
  int32_t debug_flags;          // ablations (HDD_ABLATION builds only)
  uint32_t variant;             // HDD_VARIANT_HEX_Q3_REGISTER: the register-fragment MFMA q3 kernel
  HexTables tab;
  // p=3 reference-matrix GEMM path (hex_q3g_kernel): per 16-element group the coefficient vectors
  // [n_groups][Q3G_K][16], per element {value offset, packed row-block layout} [n_own][2], and the
  // element-independent reference matrices [Q3G_K][4096] (Q3G_K = 32 self-block + 6 x 8 face-block terms)
  double* q3g_coef;
  int64_t* q3g_meta;
  const double* q3g_tab;
  int32_t q3g_reps, pad3;
};

constexpr int HEX_REC = 72;     // doubles per element record (see hex_qp.hip)
constexpr int Q3G_K = 80;       // coefficient / reference-matrix terms of the p=3 GEMM path
bool hex_uses_records(const HexArgs& a, int degree, int nq1v, int nq1f);
// doubles of workspace the p=3 path needs for n_own elements (records + GEMM coefficients + layout)
size_t hex_q3_workspace_doubles(int64_t n_own);
// the reference matrices of the p=3 GEMM path from the 1D tables (host): out [Q3G_K][4096]
void hex_q3g_reference_tables(const HexTables& t, double* out);

// degree p in 1..3; (nq1v, nq1f) Gauss points per direction; *supported = false if no kernel matches
hipError_t launch_hex(const HexArgs& a, int degree, int nq1v, int nq1f, hipStream_t s, bool* supported);

// device pattern (any element type): blocks per element = 1 + interior faces
hipError_t launch_pattern_counts(const int32_t* nbrs, int32_t nf, int64_t n_local, int64_t own_begin, int64_t own_end,
                                 int64_t nb2, int64_t* d_counts, hipStream_t s);
// elem_ptr [n_own + 1] (exclusive prefix of the row-block sizes) in two launches (three with scan_launch or
// beyond 64 K blocks); d_scratch holds pattern_elem_ptr_scratch(n_own) int64; host_nnz (optional): a device
// pointer to mapped pinned host memory receiving elem_ptr[n_own]
int64_t pattern_elem_ptr_scratch(int64_t n_own);
hipError_t launch_pattern_elem_ptr(const int32_t* nbrs, int32_t nf, int64_t n_local, int64_t own_begin,
                                   int64_t own_end, int64_t nb2, int64_t* d_elem_ptr, int64_t* d_scratch, hipStream_t s,
                                   int64_t* host_nnz = nullptr, bool scan_launch = false);
hipError_t launch_pattern_fill(const int32_t* nbrs, int32_t nf, int32_t nb, int64_t n_local, int64_t own_begin,
                               int64_t own_end, const int64_t* gid, const int64_t* elem_ptr, int64_t* row_ptr,
                               int32_t* col, int n_cu, hipStream_t s);

// right-hand side functionals (rhs.hip)
struct RhsArgs {
  int32_t elem_type, degree, nb, tkind;
  int64_t n_local, own_begin, own_end;
  const double* coords;
  const int32_t* nbrs;
  double tc[6];
  const double* tper;
  KappaArg force, kappa, dirichlet, neumann;
  int32_t has_force, has_dirichlet, has_neumann;
  int32_t skip_face;   // 1: error injection (HDD_DEBUG_FLAGS bit 524288): the split path's face launch "fails"
  double sigma_boundary, beta;
  int32_t nqv, nqd, nqn, n_cu;
  int32_t generic;   // 1: the run-time-rule kernel only (HDD_VARIANT_RHS_GENERIC)
  int32_t no_tiny;   // 1: no TINY_PHASE tier for the force's cos products (HDD_VARIANT_RHS_NO_TINY)
  double qv[64][4];    // volume rule: reference point (3) + weight
  double qd[16][3];    // Dirichlet face rule: face parameters (2) + weight
  double qn[16][3];    // Neumann face rule
  double* out;         // [nb * n_own]
  const int32_t* ev;   // optional vertex-indexed geometry (2d): element -> vertex ids [nvpe][n_local]
  const double* vxy;   //   and vertex coordinates [n_vertices][2]
  // 2d: boundary-element list of the split path (volume kernel + face kernel); null: one fused kernel.
  // [0] count, [1] finished face workgroups (both zero between calls: reset by the face kernel's last
  // workgroup, or by launch_rhs when the face launch fails), entries from RHS_LIST_OFS (16-byte aligned, room
  // for n_own of them; the volume kernel drops entries beyond it, the face kernel clamps the count to it):
  // {own index k, the element's three vertex ids (vertex-indexed geometry)}
  uint32_t* bnd_list;
};
constexpr int RHS_LIST_OFS = 64;
inline size_t rhs_list_bytes(int64_t n_own) { return size_t(RHS_LIST_OFS) * sizeof(uint32_t) + size_t(n_own) * 16; }
hipError_t launch_rhs(const RhsArgs& a, hipStream_t s);

// products (rhs.hip): l2, h1_semi, elliptic, boundary_l2 (element-local blocks) and the SWIPDG penalty
struct ProductArgs {
  int32_t elem_type, degree, nb, kind;
  int64_t n_local, own_begin, own_end;
  const double* coords;
  const int32_t* nbrs;
  const int64_t* elem_ptr;
  int32_t tkind, nqv;            // nqv: explicit simplex volume points, else 1D Gauss points (tensor)
  double tc[6];
  const double* tper;
  KappaArg kappa;
  double sigma_inner, sigma_boundary, beta;
  int32_t nq1f, pad;             // 1D Gauss points of the face rule (tensor product in 3d)
  double qv[64][4];              // simplex: point (2) + pad + weight; tensor: qv[k][0] = point, qv[k][3] = weight
  double qf[16][2];              // 1D face rule: point, weight
  double* vals;
};
hipError_t launch_product(const ProductArgs& a, hipStream_t s);

int volume_points(int elem_type, int order);
int face_points(int order);
hipError_t launch_assemble(const AssembleArgs& a, int nqv, int nqf, hipStream_t s, bool* supported);
// products of P1 / Q1 meshes with piecewise-constant kappa on the persistent tile driver (closed forms);
// *supported = false: use launch_product
hipError_t launch_product_fast(const AssembleArgs& a, int product, hipStream_t s, bool* supported);
// the sharded Q1 step's value-major side buffers (list_elements == 4) into place (swipdg_q1.hip): a.tile_list /
// n_tile_list = the listed elements, a.elem_ptr / nbrs / finfo / n_local / own_begin / n_cu
hipError_t launch_q1_scatter_soa(const AssembleArgs& a, const double* buf, int64_t ld, double* vals, hipStream_t s);

}  // namespace dev
}  // namespace hdd
