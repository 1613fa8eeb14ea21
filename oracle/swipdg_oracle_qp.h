/*
 * oracle/swipdg_oracle_qp.h -- TEST INFRASTRUCTURE ONLY.
 * CPU restatement of the SWIPDG stiffness assembly for DG Q_p on structured 2D/3D cube grids (see the .c
 * header).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 */
#ifndef HDD_SWIPDG_ORACLE_QP_H
#define HDD_SWIPDG_ORACLE_QP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_QP_FN_CONST = 0, OR_QP_FN_PER_ELEM = 1, OR_QP_FN_SINUSOID = 2, OR_QP_FN_COS_PRODUCT = 3 };
enum { OR_QP_TENSOR_CONST = 0, OR_QP_TENSOR_ISO_PER_ELEM = 1, OR_QP_TENSOR_SYM_PER_ELEM = 2 };
enum { OR_QP_BOUNDARY_DIRICHLET = 0, OR_QP_BOUNDARY_NEUMANN = 1 };

typedef struct {
  int32_t dim;                /* 2 or 3 */
  int32_t degree;             /* p = 1..4 */
  int64_t n[3];               /* elements per direction; element id = i + n0 (j + n1 k) */
  double lower[3], upper[3];
} or_qp_grid_t;

typedef struct {
  int32_t kind, order;
  double c, b, kx, ky;        /* sinusoid: c + b sin(kx x + ky y); cos product: c cos(kx x) cos(ky y) [cos(b z) if b != 0] */
  const double* per_elem;
} or_qp_scalar_t;

typedef struct {
  int32_t kind, pad;
  double c[6];                /* constant symmetric tensor: 2D xx xy yy, 3D xx xy xz yy yz zz */
  const double* per_elem;     /* ISO: [ne]; SYM: [ne][3 | 6] */
} or_qp_tensor_t;

typedef struct {
  double sigma_inner, sigma_boundary, beta;
  int32_t boundary_kind, vol_order_override, face_order_override, pad;
} or_qp_params_t;

int64_t or_qp_num_elements(const or_qp_grid_t* g);
int64_t or_qp_pattern_nnz(const or_qp_grid_t* g);
int or_qp_pattern(const or_qp_grid_t* g, const int64_t* elem_index, int64_t* row_ptr, int32_t* col);
int or_qp_assemble(const or_qp_grid_t* g, const or_qp_scalar_t* kappa, const or_qp_tensor_t* A,
                   const or_qp_params_t* p, const int64_t* elem_index, const int64_t* row_ptr, const int32_t* col,
                   double* val);
int or_qp_rhs_swipdg(const or_qp_grid_t* g, const or_qp_scalar_t* force, const or_qp_scalar_t* kappa,
                     const or_qp_tensor_t* A, const or_qp_scalar_t* dirichlet, const or_qp_scalar_t* neumann,
                     const or_qp_params_t* p, const int64_t* elem_index, double* b);
/* products (see or_product in swipdg_oracle.h; kinds OR_PRODUCT_*) */
int or_qp_product(const or_qp_grid_t* g, int kind, const or_qp_scalar_t* kappa, const or_qp_tensor_t* A,
                  const or_qp_params_t* p, const int64_t* elem_index, const int64_t* row_ptr, const int32_t* col,
                  double* val);
int or_qp_rhs_esv2007(const or_qp_grid_t* g, int force_order, const int64_t* elem_index, double* b);
int or_qp_error_esv2007(const or_qp_grid_t* g, const double* u, const int64_t* elem_index, int order, double* l2,
                        double* h1);

#ifdef __cplusplus
}
#endif
#endif
