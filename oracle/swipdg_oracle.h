/*
 * oracle/swipdg_oracle.h -- TEST INFRASTRUCTURE ONLY.
 * CPU restatement of the dune-hdd SWIPDG / BlockSWIPDG stiffness assembly (see swipdg_oracle.c header).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 */
#ifndef HDD_SWIPDG_ORACLE_H
#define HDD_SWIPDG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_SIMPLEX = 0, OR_CUBE = 1 };
enum { OR_FN_CONST = 0, OR_FN_PER_ELEM = 1, OR_FN_SINUSOID = 2, OR_FN_COS_PRODUCT = 3, OR_FN_FLATTOP = 4 };
enum { OR_TENSOR_CONST = 0, OR_TENSOR_ISO_PER_ELEM = 1, OR_TENSOR_SYM_PER_ELEM = 2 };
enum { OR_BOUNDARY_DIRICHLET = 0, OR_BOUNDARY_NEUMANN = 1 };

typedef struct {
  int32_t elem_type;          /* OR_SIMPLEX (P1) or OR_CUBE (Q1, parallelograms) */
  int32_t pad;
  int64_t n_vertices;
  const double* coords;       /* [n_vertices][2] */
  int64_t n_elements;
  const int32_t* elem_vert;   /* [n_elements][3|4], Dune reference vertex order */
} or_mesh_t;

typedef struct {
  int32_t kind;               /* OR_FN_* */
  int32_t order;              /* integration order attributed to the function (expression functions) */
  double c;                   /* constant value / sinusoid offset a */
  double b, kx, ky;           /* sinusoid: a + b*sin(kx*x + ky*y); cos product: a*cos(kx*x)*cos(ky*y)[*cos(b*z)] */
  const double* per_elem;     /* OR_FN_PER_ELEM: [n_elements] */
  const double* table;        /* OR_FN_FLATTOP: [n_table][7] = lx, ly, ux, uy, layer_x, layer_y, value */
  int32_t n_table;
  int32_t pad;
} or_scalar_t;

/* dune-stuff FlatTop of one box (restated, see swipdg_oracle.c) at x: exposed for the CPU tests */
double or_flattop(const double* box, double x, double y);

typedef struct {
  int32_t kind;               /* OR_TENSOR_* */
  int32_t pad;
  double c[3];                /* constant symmetric tensor a11 a12 a22 */
  const double* per_elem;     /* ISO: [ne]; SYM: [ne][3] */
} or_tensor_t;

typedef struct {
  double sigma_inner;         /* dune-gdt inner_sigma(p) */
  double sigma_boundary;      /* dune-gdt boundary_sigma(p) */
  double beta;                /* dune-gdt default_beta(d) = 1/(d-1) */
  int32_t boundary_kind;      /* OR_BOUNDARY_* for every domain-boundary face */
  int32_t vol_order_override; /* -1: reference integrand order */
  int32_t face_order_override;
  int32_t pad;
} or_params_t;

void* or_grid_create(const or_mesh_t* m);
void or_grid_destroy(void* g);
int64_t or_grid_neighbor(void* g, int64_t e, int f);
int or_grid_neighbor_face(void* g, int64_t e, int f);
int or_quadrature(int elem_type, int order, double* x, double* w);

int64_t or_pattern_nnz(void* g);
int or_pattern(void* g, const int64_t* elem_index, int64_t* row_ptr, int32_t* col);
int or_assemble_swipdg(void* g, const or_scalar_t* kappa, const or_tensor_t* A, const or_params_t* p,
                       const int64_t* elem_index, const int64_t* row_ptr, const int32_t* col, double* val);
int or_assemble_swipdg_owner(void* g, const or_scalar_t* kappa, const or_tensor_t* A, const or_params_t* p,
                             const int64_t* elem_index, const int64_t* row_ptr, const int32_t* col, double* val,
                             int n_threads);
int or_block_numbering(void* g, const int32_t* subdomain, int32_t n_sub, int64_t* elem_index);
int or_assemble_block_swipdg(void* g, const int32_t* subdomain, int32_t n_sub, const or_scalar_t* kappa,
                             const or_tensor_t* A, const or_params_t* p, const int64_t* elem_index,
                             const int64_t* row_ptr, const int32_t* col, double* val);
int or_rhs_l2(void* g, int force_kind, int force_order, const int64_t* elem_index, double* b);
/* SWIPDG right-hand side (swipdg.hh:251-347): L2Volume(force) + DirichletBoundarySWIPDG(kappa, A, g_D) on
 * Dirichlet faces + L2Face(g_N) on Neumann faces; any of force / dirichlet / neumann may be NULL */
int or_rhs_swipdg(void* g, const or_scalar_t* force, const or_scalar_t* kappa, const or_tensor_t* A,
                  const or_scalar_t* dirichlet, const or_scalar_t* neumann, const or_params_t* p,
                  const int64_t* elem_index, double* b);
/* products of SWIPDG::init() (swipdg.hh:358-508), over_integrate = 2:
 *   L2 / H1_SEMI / ELLIPTIC (kappa, A) / BOUNDARY_L2: element-local blocks (volume pattern)
 *   PENALTY (kappa, A): the SWIPDG penalty terms on inner (4 blocks) and Dirichlet faces (face pattern) */
enum { OR_PRODUCT_L2 = 0, OR_PRODUCT_H1_SEMI = 1, OR_PRODUCT_ELLIPTIC = 2, OR_PRODUCT_BOUNDARY_L2 = 3,
       OR_PRODUCT_PENALTY = 4 };
int or_product(void* g, int kind, const or_scalar_t* kappa, const or_tensor_t* A, const or_params_t* p,
               const int64_t* elem_index, const int64_t* row_ptr, const int32_t* col, double* val);
int or_error_norms_esv2007(void* g, const double* u, const int64_t* elem_index, int order, double* l2, double* h1);

#ifdef __cplusplus
}
#endif
#endif
