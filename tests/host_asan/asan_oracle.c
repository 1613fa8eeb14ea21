/* Sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer) for the CPU oracle -- TEST INFRASTRUCTURE
 * ONLY, like the oracle itself: every oracle entry point the parity tests use (grid, pattern, monolithic /
 * owner-computes / block SWIPDG assembly, right-hand sides, products, error norms, the Q_p restatement in 2d and
 * 3d) over small meshes, every coefficient and tensor kind and both boundary kinds.  A memory error in the
 * checker would silently corrupt every parity claim.  Built and run by tests/test_host_sanitizers.py. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "swipdg_oracle.h"
#include "swipdg_oracle_qp.h"

static int failures = 0;
#define CHECK(cond)                                                                    \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond);          \
      ++failures;                                                                      \
    }                                                                                  \
  } while (0)

static int finite_all(const double* v, int64_t n)
{
  for (int64_t i = 0; i < n; ++i)
    if (!isfinite(v[i])) return 0;
  return 1;
}

/* nx x ny squares on [0,1]^2: Kuhn triangles (0: (v00, v10, v11), (v00, v11, v01)) or Dune-ordered quads */
static void structured(int et, int nx, int ny, double** coords, int32_t** ev, int64_t* nv, int64_t* ne)
{
  *nv = (int64_t)(nx + 1) * (ny + 1);
  *ne = (int64_t)nx * ny * (et == OR_SIMPLEX ? 2 : 1);
  *coords = malloc(sizeof(double) * 2 * *nv);
  *ev = malloc(sizeof(int32_t) * (et == OR_SIMPLEX ? 3 : 4) * *ne);
  for (int j = 0; j <= ny; ++j)
    for (int i = 0; i <= nx; ++i) {
      (*coords)[2 * (j * (nx + 1) + i)] = i / (double)nx;
      (*coords)[2 * (j * (nx + 1) + i) + 1] = j / (double)ny;
    }
  int64_t k = 0;
  for (int j = 0; j < ny; ++j)
    for (int i = 0; i < nx; ++i) {
      const int v00 = j * (nx + 1) + i, v10 = v00 + 1, v01 = v00 + nx + 1, v11 = v01 + 1;
      if (et == OR_SIMPLEX) {
        const int t[6] = {v00, v10, v11, v00, v11, v01};
        for (int q = 0; q < 6; ++q) (*ev)[k++] = t[q];
      } else {
        const int t[4] = {v00, v10, v01, v11};
        for (int q = 0; q < 4; ++q) (*ev)[k++] = t[q];
      }
    }
}

static void exercise_2d(int et, int nx, int ny, int px)
{
  double* coords;
  int32_t* ev;
  int64_t nv, ne;
  structured(et, nx, ny, &coords, &ev, &nv, &ne);
  const int nb = et == OR_SIMPLEX ? 3 : 4;
  or_mesh_t m = {et, 0, nv, coords, ne, ev};
  void* g = or_grid_create(&m);
  CHECK(g != NULL);
  for (int64_t e = 0; e < ne; ++e)
    for (int f = 0; f < nb; ++f) {
      const int64_t n = or_grid_neighbor(g, e, f);
      CHECK(n >= -2 && n < ne);
      if (n >= 0) CHECK(or_grid_neighbor(g, n, or_grid_neighbor_face(g, e, f)) == e);
    }
  const int64_t nnz = or_pattern_nnz(g);
  int64_t* rp = malloc(sizeof(int64_t) * (ne * nb + 1));
  int32_t* col = malloc(sizeof(int32_t) * nnz);
  double* val = malloc(sizeof(double) * nnz);
  double* val2 = malloc(sizeof(double) * nnz);
  CHECK(or_pattern(g, NULL, rp, col) == 0);
  CHECK(rp[ne * nb] == nnz);

  double* pe = malloc(sizeof(double) * ne);
  double* sym = malloc(sizeof(double) * 3 * ne);
  for (int64_t e = 0; e < ne; ++e) {
    pe[e] = 0.5 + (double)(e % 7);
    sym[3 * e] = 2.0; sym[3 * e + 1] = 0.1 * (e % 3); sym[3 * e + 2] = 1.5;
  }
  const double box[2][7] = {{0.2, 0.2, 0.6, 0.7, 0.05, 0.05, 3.0}, {0.5, 0.0, 0.9, 0.4, 0.0, 0.0, 2.0}};
  or_scalar_t kap[5] = {
      {OR_FN_CONST, 0, 1.0, 0, 0, 0, NULL, NULL, 0, 0},
      {OR_FN_PER_ELEM, 0, 0, 0, 0, 0, pe, NULL, 0, 0},
      {OR_FN_SINUSOID, 3, 1.0, 0.75, 12.566370614359172, 6.283185307179586, NULL, NULL, 0, 0},
      {OR_FN_COS_PRODUCT, 3, 1.0, 0.0, 3.0, 2.0, NULL, NULL, 0, 0},
      {OR_FN_FLATTOP, 3, 1.0, 1.0, 0, 0, NULL, &box[0][0], 2, 0}};
  or_tensor_t ten[3] = {{OR_TENSOR_CONST, 0, {1.0, 0.0, 1.0}, NULL},
                        {OR_TENSOR_ISO_PER_ELEM, 0, {0, 0, 0}, pe},
                        {OR_TENSOR_SYM_PER_ELEM, 0, {0, 0, 0}, sym}};
  for (int bk = 0; bk < 2; ++bk) {
    or_params_t prm = {8.0, 14.0, 1.0, bk, -1, -1, 0};
    for (int k = 0; k < 5; ++k)
      for (int t = 0; t < 3; ++t) {
        CHECK(or_assemble_swipdg(g, &kap[k], &ten[t], &prm, NULL, rp, col, val) == 0);
        CHECK(finite_all(val, nnz));
      }
    CHECK(or_assemble_swipdg_owner(g, &kap[1], &ten[2], &prm, NULL, rp, col, val2, 2) == 0);
    CHECK(or_assemble_swipdg(g, &kap[1], &ten[2], &prm, NULL, rp, col, val) == 0);
    for (int64_t q = 0; q < nnz; ++q) CHECK(fabs(val[q] - val2[q]) <= 1e-12 * (1.0 + fabs(val[q])));
    /* right-hand side with Dirichlet / Neumann data, products, error norms */
    double* b = malloc(sizeof(double) * ne * nb);
    CHECK(or_rhs_l2(g, 0, 3, NULL, b) == 0 && finite_all(b, ne * nb));
    CHECK(or_rhs_swipdg(g, &kap[3], &kap[0], &ten[1], &kap[2], &kap[2], &prm, NULL, b) == 0 && finite_all(b, ne * nb));
    double l2 = -1, h1 = -1;
    CHECK(or_error_norms_esv2007(g, b, NULL, 4, &l2, &h1) == 0 && l2 >= 0 && h1 >= 0);
    free(b);
    for (int kind = OR_PRODUCT_L2; kind <= OR_PRODUCT_PENALTY; ++kind) {
      /* volume products live on the element-local pattern: row r of element e holds the nb columns of e */
      if (kind == OR_PRODUCT_PENALTY) {
        CHECK(or_product(g, kind, &kap[1], &ten[1], &prm, NULL, rp, col, val) == 0 && finite_all(val, nnz));
      } else {
        int64_t* vrp = malloc(sizeof(int64_t) * (ne * nb + 1));
        int32_t* vcol = malloc(sizeof(int32_t) * ne * nb * nb);
        double* vval = malloc(sizeof(double) * ne * nb * nb);
        for (int64_t r = 0; r <= ne * nb; ++r) vrp[r] = r * nb;
        for (int64_t r = 0; r < ne * nb; ++r)
          for (int c = 0; c < nb; ++c) vcol[r * nb + c] = (int32_t)((r / nb) * nb + c);
        CHECK(or_product(g, kind, &kap[2], &ten[2], &prm, NULL, vrp, vcol, vval) == 0 && finite_all(vval, ne * nb * nb));
        free(vrp); free(vcol); free(vval);
      }
    }
  }
  /* block numbering and BlockSWIPDG in it: px column strips of subdomains */
  int32_t* sd = malloc(sizeof(int32_t) * ne);
  for (int64_t e = 0; e < ne; ++e) {
    const int64_t sq = et == OR_SIMPLEX ? e / 2 : e;
    sd[e] = (int32_t)((sq % nx) * px / nx);
  }
  int64_t* ei = malloc(sizeof(int64_t) * ne);
  CHECK(or_block_numbering(g, sd, px, ei) == 0);
  CHECK(or_pattern(g, ei, rp, col) == 0);
  or_params_t prm = {8.0, 14.0, 1.0, 0, -1, -1, 0};
  CHECK(or_assemble_block_swipdg(g, sd, px, &kap[0], &ten[1], &prm, ei, rp, col, val) == 0 && finite_all(val, nnz));
  CHECK(or_assemble_swipdg(g, &kap[0], &ten[1], &prm, ei, rp, col, val2) == 0);
  for (int64_t q = 0; q < nnz; ++q) CHECK(fabs(val[q] - val2[q]) <= 1e-12 * (1.0 + fabs(val2[q])));
  free(sd); free(ei); free(pe); free(sym);
  free(rp); free(col); free(val); free(val2);
  or_grid_destroy(g);
  free(coords); free(ev);
}

static void exercise_qp(int dim, int p, int nx, int ny, int nz)
{
  or_qp_grid_t g = {dim, p, {nx, ny, dim == 3 ? nz : 1}, {0, 0, 0}, {1, 1, 1}};
  const int64_t ne = or_qp_num_elements(&g);
  int nb = 1;
  for (int d = 0; d < dim; ++d) nb *= p + 1;
  const int64_t nnz = or_qp_pattern_nnz(&g);
  int64_t* rp = malloc(sizeof(int64_t) * (ne * nb + 1));
  int32_t* col = malloc(sizeof(int32_t) * nnz);
  double* val = malloc(sizeof(double) * nnz);
  CHECK(or_qp_pattern(&g, NULL, rp, col) == 0 && rp[ne * nb] == nnz);
  double* pe = malloc(sizeof(double) * ne * 6);
  for (int64_t i = 0; i < ne * 6; ++i) pe[i] = (i % 6 == 0 || i % 6 == 3 || i % 6 == 5) ? 1.0 + 0.1 * (i % 5) : 0.05;
  or_qp_scalar_t kap[3] = {{OR_QP_FN_CONST, 0, 1.0, 0, 0, 0, NULL},
                           {OR_QP_FN_PER_ELEM, 0, 0, 0, 0, 0, pe},
                           {OR_QP_FN_SINUSOID, 3, 1.0, 0.5, 3.0, 2.0, NULL}};
  or_qp_tensor_t ten[3] = {{OR_QP_TENSOR_CONST, 0, {1, 0, 0, 1, 0, 1}, NULL},   /* 3d xx xy xz yy yz zz; 2d below */
                           {OR_QP_TENSOR_ISO_PER_ELEM, 0, {0}, pe},
                           {OR_QP_TENSOR_SYM_PER_ELEM, 0, {0}, pe}};
  if (dim == 2) ten[0].c[1] = 0.0, ten[0].c[2] = 1.0;   /* 2d xx xy yy */
  for (int bk = 0; bk < 2; ++bk) {
    or_qp_params_t prm = {20.0, 38.0, dim == 3 ? 0.5 : 1.0, bk, -1, -1, 0};
    for (int k = 0; k < 3; ++k)
      for (int t = 0; t < 3; ++t) {
        CHECK(or_qp_assemble(&g, &kap[k], &ten[t], &prm, NULL, rp, col, val) == 0);
        CHECK(finite_all(val, nnz));
      }
    double* b = malloc(sizeof(double) * ne * nb);
    or_qp_scalar_t force = {OR_QP_FN_COS_PRODUCT, 3, 1.0, dim == 3 ? 1.0 : 0.0, 3.0, 2.0, NULL};
    CHECK(or_qp_rhs_swipdg(&g, &force, &kap[0], &ten[0], &kap[2], &kap[2], &prm, NULL, b) == 0 && finite_all(b, ne * nb));
    CHECK(or_qp_rhs_esv2007(&g, 3, NULL, b) == 0 && finite_all(b, ne * nb));
    double l2 = -1, h1 = -1;
    CHECK(or_qp_error_esv2007(&g, b, NULL, 4, &l2, &h1) == 0 && l2 >= 0 && h1 >= 0);
    CHECK(or_qp_product(&g, OR_PRODUCT_PENALTY, &kap[1], &ten[1], &prm, NULL, rp, col, val) == 0 && finite_all(val, nnz));
    free(b);
  }
  free(pe); free(rp); free(col); free(val);
}

int main(void)
{
  double x[512], w[256];
  for (int et = 0; et < 2; ++et)
    for (int o = 0; o <= 10; ++o) {
      const int n = or_quadrature(et, o, x, w);
      CHECK(n > 0 && n <= 256);
    }
  const int sizes[][3] = {{1, 1, 1}, {3, 1, 1}, {1, 4, 1}, {6, 5, 2}, {9, 4, 3}};
  for (int et = 0; et < 2; ++et)
    for (int s = 0; s < 5; ++s) exercise_2d(et, sizes[s][0], sizes[s][1], sizes[s][2]);
  for (int p = 1; p <= 3; ++p) {
    exercise_qp(2, p, 4, 3, 1);
    exercise_qp(3, p, 3, 2, 2);
  }
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("oracle sanitizer run: all checks passed\n");
  return 0;
}
