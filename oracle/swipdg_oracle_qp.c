/*
 * oracle/swipdg_oracle_qp.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * CPU restatement of the dune-hdd SWIPDG stiffness assembly for discontinuous Q_p Lagrange spaces
 * (p = 1..4) on structured tensor-product grids of cubes in 2D and 3D -- the C5 configuration
 * ("ESV2007 3D structured, SWIPDG p=3", BASELINE.json configs[4]).  Same walk as swipdg_oracle.c:
 *   - Discretizations::SWIPDG::init(): one SystemAssembler walk, volume Elliptic + SWIPDG::Inner on inner
 *     intersections visited primally (entity index < neighbour index) + BoundaryLHS on Dirichlet faces
 *     (dune/hdd/linearelliptic/discretizations/swipdg.hh:218-249, 485);
 *   - local matrices by quadrature with the basis evaluated at points mapped through the element geometries
 *     (geometryInInside / geometryInOutside: the neighbour's local coordinates come from inverting its
 *     geometry), scatter by a binary search in the sorted CSR row (Stuff::LA add_to_entry);
 *   - integrand orders of dune-gdt's LocalEvaluation: volume ord(kappa)+ord(A)+2*max(p-1,0), faces
 *     ord(kappa)+ord(A)+2p; Gauss-Legendre tensor rules with ceil((order+1)/2) points per direction;
 *   - penalty sigma * kappa^- kappa^+ gamma / |F|^beta with |F| the face volume (area in 3D), beta=1/(d-1).
 * The DG space is dune-gdt's DiscontinuousLagrange (swipdg.hh:94): Q_p Lagrange shape functions with
 * equidistant nodes, DoFs numbered lexicographically (x fastest) inside the element, element-blocked.
 *
 * Pinning: at d=2, p=1 this restatement must reproduce swipdg_oracle.c (pinned to the reference's ESV2007
 * expectation tables) entry for entry -- tests/test_oracle_qp.py.  For p>1 and d=3 there is no reference
 * fixture (the reference's ESV2007 testcase is 2D-only, testcases/ESV2007.hh:32): parity for those is
 * against this restatement, checked by the p+1 L2 convergence of the ESV2007 exact solution.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "swipdg_oracle_qp.h"

#define QP_MAXD 3
#define QP_MAXP 4
#define QP_MAXN1 12

static double linspace_node(double a, double b, int64_t n, int64_t i)
{
  if (i == n) return b;
  return (double)i * ((b - a) / (double)n) + a;
}

/* Gauss-Legendre on [0,1], n points (Newton on P_n) */
static void gauss01(int n, double* s, double* w)
{
  for (int i = 0; i < n; ++i) {
    double x = cos(M_PI * (i + 0.75) / (n + 0.5)), p0 = 1.0, p1 = x, dp = 1.0;
    for (int it = 0; it < 100; ++it) {
      p0 = 1.0; p1 = x;
      for (int k = 2; k <= n; ++k) { const double p2 = ((2.0 * k - 1) * x * p1 - (k - 1.0) * p0) / k; p0 = p1; p1 = p2; }
      if (n == 1) { p1 = x; p0 = 1.0; }
      dp = n * (x * p1 - p0) / (x * x - 1.0);
      const double dx = p1 / dp;
      x -= dx;
      if (fabs(dx) < 1e-16) break;
    }
    p0 = 1.0; p1 = x;
    for (int k = 2; k <= n; ++k) { const double p2 = ((2.0 * k - 1) * x * p1 - (k - 1.0) * p0) / k; p0 = p1; p1 = p2; }
    if (n == 1) { p1 = x; p0 = 1.0; }
    dp = n * (x * p1 - p0) / (x * x - 1.0);
    s[n - 1 - i] = 0.5 * (x + 1.0);
    w[n - 1 - i] = 1.0 / ((1.0 - x * x) * dp * dp);
  }
}

static int points_for_order(int order)
{
  int n = (order + 2) / 2;
  if (n < 1) n = 1;
  if (n > QP_MAXN1) n = QP_MAXN1;
  return n;
}

/* 1D Lagrange polynomial k of degree p on equidistant nodes j/p, and its derivative */
static void lagrange1(int p, int k, double x, double* v, double* d)
{
  double val = 1.0, der = 0.0;
  for (int m = 0; m <= p; ++m) {
    if (m == k) continue;
    const double den = (double)(k - m) / p;
    const double f = (x - (double)m / p) / den;
    der = der * f + val / den;
    val *= f;
  }
  *v = val;
  *d = der;
}

typedef struct {
  int dim, p, nb, nf;
  int64_t n[3], ne;
  double lower[3], upper[3];
} qgrid_t;

static int init_grid(const or_qp_grid_t* in, qgrid_t* g)
{
  if (in->dim < 2 || in->dim > 3 || in->degree < 1 || in->degree > QP_MAXP) return -1;
  g->dim = in->dim;
  g->p = in->degree;
  g->nb = 1;
  g->ne = 1;
  for (int a = 0; a < 3; ++a) {
    g->n[a] = a < g->dim ? in->n[a] : 1;
    g->lower[a] = in->lower[a];
    g->upper[a] = in->upper[a];
    if (a < g->dim) {
      if (g->n[a] < 1) return -1;
      g->nb *= g->p + 1;
      g->ne *= g->n[a];
    }
  }
  g->nf = 2 * g->dim;
  return 0;
}

static void elem_ijk(const qgrid_t* g, int64_t e, int64_t* ijk)
{
  ijk[0] = e % g->n[0];
  ijk[1] = (e / g->n[0]) % g->n[1];
  ijk[2] = e / (g->n[0] * g->n[1]);
}

/* neighbour across local face f (2a: x_a = 0 side, 2a+1: x_a = 1 side), or -1 on the domain boundary */
static int64_t neighbour(const qgrid_t* g, int64_t e, int f)
{
  int64_t ijk[3];
  elem_ijk(g, e, ijk);
  const int a = f / 2, side = f % 2;
  const int64_t c = ijk[a] + (side ? 1 : -1);
  if (c < 0 || c >= g->n[a]) return -1;
  int64_t stride = 1;
  for (int b = 0; b < a; ++b) stride *= g->n[b];
  return e + (side ? stride : -stride);
}

/* affine geometry x = v0 + J xh, J columns = edges from vertex 0 to vertices 1, 2, 4 (Dune cube order) */
typedef struct { int d; double v0[3]; double J[3][3]; double Jinv[3][3]; double det; } geo_t;

static void geometry(const qgrid_t* g, int64_t e, geo_t* G)
{
  int64_t ijk[3];
  elem_ijk(g, e, ijk);
  const int d = g->dim;
  G->d = d;
  memset(G->J, 0, sizeof(G->J));
  memset(G->Jinv, 0, sizeof(G->Jinv));
  for (int a = 0; a < d; ++a) {
    const double x0 = linspace_node(g->lower[a], g->upper[a], g->n[a], ijk[a]);
    const double x1 = linspace_node(g->lower[a], g->upper[a], g->n[a], ijk[a] + 1);
    G->v0[a] = x0;
    G->J[a][a] = x1 - x0;
  }
  /* general inverse (the grid is axis-aligned, the integrand code does not rely on it) */
  if (d == 2) {
    G->det = G->J[0][0] * G->J[1][1] - G->J[0][1] * G->J[1][0];
    G->Jinv[0][0] = G->J[1][1] / G->det; G->Jinv[0][1] = -G->J[0][1] / G->det;
    G->Jinv[1][0] = -G->J[1][0] / G->det; G->Jinv[1][1] = G->J[0][0] / G->det;
  } else {
    double (*J)[3] = G->J;
    const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
    const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
    const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
    G->det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
    const double id = 1.0 / G->det;
    G->Jinv[0][0] = c00 * id;
    G->Jinv[1][0] = c01 * id;
    G->Jinv[2][0] = c02 * id;
    G->Jinv[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * id;
    G->Jinv[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * id;
    G->Jinv[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * id;
    G->Jinv[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * id;
    G->Jinv[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * id;
    G->Jinv[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * id;
  }
}

static void global_pt(const geo_t* G, const double* xh, double* x)
{
  for (int a = 0; a < G->d; ++a) {
    x[a] = G->v0[a];
    for (int b = 0; b < G->d; ++b) x[a] += G->J[a][b] * xh[b];
  }
}

static void local_pt(const geo_t* G, const double* x, double* xh)
{
  for (int a = 0; a < G->d; ++a) {
    xh[a] = 0.0;
    for (int b = 0; b < G->d; ++b) xh[a] += G->Jinv[a][b] * (x[b] - G->v0[b]);
  }
}

/* physical gradient = J^{-T} reference gradient */
static void map_grad(const geo_t* G, const double* gh, double* gp)
{
  for (int a = 0; a < G->d; ++a) {
    gp[a] = 0.0;
    for (int b = 0; b < G->d; ++b) gp[a] += G->Jinv[b][a] * gh[b];
  }
}

/* Q_p shape functions at a reference point: phi[nb], grad[nb][d] */
static void shape(const qgrid_t* g, const double* xh, double* phi, double (*grad)[3])
{
  double v[3][QP_MAXP + 1], dv[3][QP_MAXP + 1];
  for (int a = 0; a < g->dim; ++a)
    for (int k = 0; k <= g->p; ++k) lagrange1(g->p, k, xh[a], &v[a][k], &dv[a][k]);
  for (int i = 0; i < g->nb; ++i) {
    int idx[3], r = i;
    for (int a = 0; a < g->dim; ++a) { idx[a] = r % (g->p + 1); r /= g->p + 1; }
    double val = 1.0;
    for (int a = 0; a < g->dim; ++a) val *= v[a][idx[a]];
    phi[i] = val;
    for (int b = 0; b < g->dim; ++b) {
      double gb = 1.0;
      for (int a = 0; a < g->dim; ++a) gb *= a == b ? dv[a][idx[a]] : v[a][idx[a]];
      grad[i][b] = gb;
    }
  }
}

static double eval_scalar(const or_qp_scalar_t* s, int64_t e, const double* x)
{
  switch (s->kind) {
    case OR_QP_FN_CONST: return s->c;
    case OR_QP_FN_PER_ELEM: return s->per_elem[e];
    case OR_QP_FN_SINUSOID: return s->c + s->b * sin(s->kx * x[0] + s->ky * x[1]);
    case OR_QP_FN_COS_PRODUCT:   /* z factor only for b != 0 (3d data); 2d callers leave b = 0 */
      return s->c * cos(s->kx * x[0]) * cos(s->ky * x[1]) * (s->b != 0.0 ? cos(s->b * x[2]) : 1.0);
    default: return 0.0;
  }
}

/* symmetric tensor: 2D (xx, xy, yy), 3D (xx, xy, xz, yy, yz, zz) */
static void eval_tensor(const qgrid_t* g, const or_qp_tensor_t* t, int64_t e, double A[3][3])
{
  const int d = g->dim, ns = d == 2 ? 3 : 6;
  double c[6];
  memset(A, 0, sizeof(double) * 9);
  if (t->kind == OR_QP_TENSOR_ISO_PER_ELEM) {
    for (int a = 0; a < d; ++a) A[a][a] = t->per_elem[e];
    return;
  }
  for (int k = 0; k < ns; ++k) c[k] = t->kind == OR_QP_TENSOR_SYM_PER_ELEM ? t->per_elem[e * ns + k] : t->c[k];
  if (d == 2) {
    A[0][0] = c[0]; A[0][1] = A[1][0] = c[1]; A[1][1] = c[2];
  } else {
    A[0][0] = c[0]; A[0][1] = A[1][0] = c[1]; A[0][2] = A[2][0] = c[2];
    A[1][1] = c[3]; A[1][2] = A[2][1] = c[4]; A[2][2] = c[5];
  }
}

static int scalar_order(const or_qp_scalar_t* s)
{
  return (s->kind == OR_QP_FN_SINUSOID || s->kind == OR_QP_FN_COS_PRODUCT) ? s->order : 0;
}

static inline int64_t gid_of(const int64_t* elem_index, int64_t e) { return elem_index ? elem_index[e] : e; }

int64_t or_qp_num_elements(const or_qp_grid_t* in)
{
  qgrid_t g;
  return init_grid(in, &g) ? -1 : g.ne;
}

int64_t or_qp_pattern_nnz(const or_qp_grid_t* in)
{
  qgrid_t g;
  if (init_grid(in, &g)) return -1;
  int64_t nnz = 0;
  for (int64_t e = 0; e < g.ne; ++e) {
    int blocks = 1;
    for (int f = 0; f < g.nf; ++f) blocks += neighbour(&g, e, f) >= 0;
    nnz += (int64_t)g.nb * g.nb * blocks;
  }
  return nnz;
}

static int cmp_i64(const void* a, const void* b)
{
  const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return x < y ? -1 : (x > y);
}

/* rows = DoFs gid*nb + i (rows of the elements in gid order); row: all DoFs of the element and its face
 * neighbours, sorted ascending (EllipticSWIPDG pattern, swipdg.hh:169) */
int or_qp_pattern(const or_qp_grid_t* in, const int64_t* elem_index, int64_t* row_ptr, int32_t* col)
{
  qgrid_t g;
  if (init_grid(in, &g)) return -1;
  int64_t* inv = (int64_t*)malloc(sizeof(int64_t) * (size_t)g.ne);
  int64_t* len = (int64_t*)malloc(sizeof(int64_t) * (size_t)g.ne);
  for (int64_t e = 0; e < g.ne; ++e) inv[gid_of(elem_index, e)] = e;
  for (int64_t e = 0; e < g.ne; ++e) {
    int blocks = 1;
    for (int f = 0; f < g.nf; ++f) blocks += neighbour(&g, e, f) >= 0;
    len[gid_of(elem_index, e)] = (int64_t)g.nb * blocks;
  }
  row_ptr[0] = 0;
  for (int64_t k = 0; k < g.ne; ++k)
    for (int i = 0; i < g.nb; ++i) row_ptr[k * g.nb + i + 1] = row_ptr[k * g.nb + i] + len[k];
  for (int64_t k = 0; k < g.ne; ++k) {
    const int64_t e = inv[k];
    int64_t blk[7];
    int nblk = 0;
    blk[nblk++] = k;
    for (int f = 0; f < g.nf; ++f) {
      const int64_t n = neighbour(&g, e, f);
      if (n >= 0) blk[nblk++] = gid_of(elem_index, n);
    }
    qsort(blk, (size_t)nblk, sizeof(int64_t), cmp_i64);
    for (int i = 0; i < g.nb; ++i) {
      int64_t o = row_ptr[k * g.nb + i];
      for (int b = 0; b < nblk; ++b)
        for (int j = 0; j < g.nb; ++j) col[o++] = (int32_t)(blk[b] * g.nb + j);
    }
  }
  free(inv);
  free(len);
  return 0;
}

static inline void add_to_entry(const int64_t* row_ptr, const int32_t* col, double* val, int64_t r, int64_t c,
                                double v)
{
  int64_t lo = row_ptr[r], hi = row_ptr[r + 1] - 1;
  while (lo <= hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (col[mid] == c) { val[mid] += v; return; }
    if (col[mid] < c) lo = mid + 1; else hi = mid - 1;
  }
  val[row_ptr[r]] = NAN;   /* not in the pattern: the reference throws; make tests fail loudly */
}

typedef struct {
  const qgrid_t* g;
  const or_qp_scalar_t* kappa;
  const or_qp_tensor_t* A;
  const or_qp_params_t* prm;
  const int64_t* elem_index;
  const int64_t* row_ptr;
  const int32_t* col;
  double* val;
} qctx_t;

static void scatter(const qctx_t* c, int64_t te, int64_t ae, const double* L)
{
  const int nb = c->g->nb;
  const int64_t tg = gid_of(c->elem_index, te), ag = gid_of(c->elem_index, ae);
  for (int i = 0; i < nb; ++i)
    for (int j = 0; j < nb; ++j)
      add_to_entry(c->row_ptr, c->col, c->val, tg * nb + i, ag * nb + j, L[i * nb + j]);
}

/* tensor Gauss rule of dimension k on [0,1]^k */
typedef struct { int n; double x[QP_MAXN1 * QP_MAXN1 * QP_MAXN1][3]; double w[QP_MAXN1 * QP_MAXN1 * QP_MAXN1]; } qrule_t;

static void tensor_rule(int k, int order, qrule_t* q)
{
  double s[QP_MAXN1], w[QP_MAXN1];
  const int n = points_for_order(order);
  gauss01(n, s, w);
  int tot = 1;
  for (int a = 0; a < k; ++a) tot *= n;
  q->n = tot;
  for (int m = 0; m < tot; ++m) {
    int r = m;
    q->w[m] = 1.0;
    for (int a = 0; a < 3; ++a) q->x[m][a] = 0.0;
    for (int a = 0; a < k; ++a) {
      const int ia = r % n;
      r /= n;
      q->x[m][a] = s[ia];
      q->w[m] *= w[ia];
    }
  }
}

static double dot(int d, const double* a, const double* b)
{
  double s = 0.0;
  for (int k = 0; k < d; ++k) s += a[k] * b[k];
  return s;
}

static void matvec(int d, double A[3][3], const double* x, double* y)
{
  for (int a = 0; a < d; ++a) {
    y[a] = 0.0;
    for (int b = 0; b < d; ++b) y[a] += A[a][b] * x[b];
  }
}

/* LocalEvaluation::Elliptic */
static void local_volume(const qctx_t* c, qrule_t* q, int64_t e, double* L)
{
  const qgrid_t* g = c->g;
  const int nb = g->nb, d = g->dim;
  geo_t G;
  geometry(g, e, &G);
  double A[3][3];
  eval_tensor(g, c->A, e, A);
  int order = scalar_order(c->kappa) + 0 + 2 * (g->p - 1);
  if (c->prm->vol_order_override >= 0) order = c->prm->vol_order_override;
  tensor_rule(d, order, q);
  memset(L, 0, sizeof(double) * (size_t)(nb * nb));
  double phi[125], gh[125][3], gp[125][3], Ag[125][3];
  for (int k = 0; k < q->n; ++k) {
    double x[3];
    shape(g, q->x[k], phi, gh);
    global_pt(&G, q->x[k], x);
    for (int i = 0; i < nb; ++i) { map_grad(&G, gh[i], gp[i]); matvec(d, A, gp[i], Ag[i]); }
    const double fac = q->w[k] * fabs(G.det) * eval_scalar(c->kappa, e, x);
    for (int i = 0; i < nb; ++i)
      for (int j = 0; j < nb; ++j) L[i * nb + j] += fac * dot(d, Ag[j], gp[i]);
  }
}

/* reference face f of [0,1]^d: point for face-rule coordinates s (free axes in increasing order) */
static void face_ref_point(int d, int f, const double* s, double* xh)
{
  const int a = f / 2;
  int k = 0;
  for (int b = 0; b < d; ++b) xh[b] = b == a ? (double)(f % 2) : s[k++];
}

/* unit outer normal (J^{-T} n_ref normalised) and face volume |det J| |J^{-T} n_ref| (Nanson) */
static void face_normal(const geo_t* G, int f, double* n, double* vol)
{
  double nr[3] = {0.0, 0.0, 0.0};
  nr[f / 2] = f % 2 ? 1.0 : -1.0;
  map_grad(G, nr, n);
  double nn = sqrt(dot(G->d, n, n));
  for (int a = 0; a < G->d; ++a) n[a] /= nn;
  *vol = fabs(G->det) * nn;
}

/* SWIPDG::Inner: EE, EN, NE, NN blocks of the face f of e with neighbour ne */
static void local_inner(const qctx_t* c, qrule_t* q, int64_t e, int f, int64_t ne, double* EE, double* EN,
                        double* NE, double* NN)
{
  const qgrid_t* g = c->g;
  const int nb = g->nb, d = g->dim;
  geo_t Gi, Go;
  geometry(g, e, &Gi);
  geometry(g, ne, &Go);
  double n[3], fvol;
  face_normal(&Gi, f, n, &fvol);
  double Ai[3][3], Ao[3][3];
  eval_tensor(g, c->A, e, Ai);
  eval_tensor(g, c->A, ne, Ao);
  int order = scalar_order(c->kappa) + 0 + 2 * g->p;
  if (c->prm->face_order_override >= 0) order = c->prm->face_order_override;
  tensor_rule(d - 1, order, q);
  const size_t sz = sizeof(double) * (size_t)(nb * nb);
  memset(EE, 0, sz); memset(EN, 0, sz); memset(NE, 0, sz); memset(NN, 0, sz);
  double An_i[3], An_o[3];
  matvec(d, Ai, n, An_i);
  matvec(d, Ao, n, An_o);
  const double delta_minus = dot(d, n, An_i), delta_plus = dot(d, n, An_o);
  const double gamma = delta_plus * delta_minus / (delta_plus + delta_minus);
  const double wp = delta_minus / (delta_plus + delta_minus);
  const double wm = delta_plus / (delta_plus + delta_minus);
  const double hpow = pow(fvol, c->prm->beta);
  double pe[125], ghe[125][3], ge[125][3], pn[125], ghn[125][3], gn[125][3], Ae[125], An[125];
  for (int k = 0; k < q->n; ++k) {
    double xin[3], x[3], xout[3];
    face_ref_point(d, f, q->x[k], xin);
    global_pt(&Gi, xin, x);
    local_pt(&Go, x, xout);
    shape(g, xin, pe, ghe);
    shape(g, xout, pn, ghn);
    for (int i = 0; i < nb; ++i) {
      map_grad(&Gi, ghe[i], ge[i]);
      map_grad(&Go, ghn[i], gn[i]);
      Ae[i] = dot(d, An_i, ge[i]);   /* (A grad phi) . n  (A symmetric) */
      An[i] = dot(d, An_o, gn[i]);
    }
    const double ke = eval_scalar(c->kappa, e, x), kn = eval_scalar(c->kappa, ne, x);
    const double pen = ke * kn * c->prm->sigma_inner * gamma / hpow;
    const double fac = q->w[k] * fvol;
    for (int i = 0; i < nb; ++i)
      for (int j = 0; j < nb; ++j) {
        EE[i * nb + j] += fac * (-wm * ke * Ae[j] * pe[i] - wm * ke * pe[j] * Ae[i] + pen * pe[j] * pe[i]);
        EN[i * nb + j] += fac * (-wp * kn * An[j] * pe[i] + wm * ke * pn[j] * Ae[i] - pen * pn[j] * pe[i]);
        NE[i * nb + j] += fac * (wm * ke * Ae[j] * pn[i] - wp * kn * pe[j] * An[i] - pen * pe[j] * pn[i]);
        NN[i * nb + j] += fac * (wp * kn * An[j] * pn[i] + wp * kn * pn[j] * An[i] + pen * pn[j] * pn[i]);
      }
  }
}

/* SWIPDG::BoundaryLHS */
static void local_boundary(const qctx_t* c, qrule_t* q, int64_t e, int f, double* L)
{
  const qgrid_t* g = c->g;
  const int nb = g->nb, d = g->dim;
  geo_t G;
  geometry(g, e, &G);
  double n[3], fvol;
  face_normal(&G, f, n, &fvol);
  double A[3][3], An_[3];
  eval_tensor(g, c->A, e, A);
  matvec(d, A, n, An_);
  int order = scalar_order(c->kappa) + 0 + 2 * g->p;
  if (c->prm->face_order_override >= 0) order = c->prm->face_order_override;
  tensor_rule(d - 1, order, q);
  memset(L, 0, sizeof(double) * (size_t)(nb * nb));
  const double gamma = dot(d, n, An_);
  const double hpow = pow(fvol, c->prm->beta);
  double ph[125], gh[125][3], gp[125][3], Ag[125];
  for (int k = 0; k < q->n; ++k) {
    double xin[3], x[3];
    face_ref_point(d, f, q->x[k], xin);
    global_pt(&G, xin, x);
    shape(g, xin, ph, gh);
    for (int i = 0; i < nb; ++i) { map_grad(&G, gh[i], gp[i]); Ag[i] = dot(d, An_, gp[i]); }
    const double kap = eval_scalar(c->kappa, e, x);
    const double pen = c->prm->sigma_boundary * kap * gamma / hpow;
    const double fac = q->w[k] * fvol;
    for (int i = 0; i < nb; ++i)
      for (int j = 0; j < nb; ++j)
        L[i * nb + j] += fac * (-kap * Ag[j] * ph[i] - kap * ph[j] * Ag[i] + pen * ph[j] * ph[i]);
  }
}

int or_qp_assemble(const or_qp_grid_t* in, const or_qp_scalar_t* kappa, const or_qp_tensor_t* A,
                   const or_qp_params_t* prm, const int64_t* elem_index, const int64_t* row_ptr, const int32_t* col,
                   double* val)
{
  qgrid_t g;
  if (init_grid(in, &g)) return -1;
  qctx_t c = {&g, kappa, A, prm, elem_index, row_ptr, col, val};
  const int nb = g.nb;
  memset(val, 0, sizeof(double) * (size_t)row_ptr[g.ne * nb]);
  double* buf = (double*)malloc(sizeof(double) * (size_t)(4 * nb * nb));
  qrule_t* q = (qrule_t*)malloc(sizeof(qrule_t));
  double *L = buf, *EN = buf + nb * nb, *NE = buf + 2 * nb * nb, *NN = buf + 3 * nb * nb;
  for (int64_t e = 0; e < g.ne; ++e) {
    local_volume(&c, q, e, L);
    scatter(&c, e, e, L);
    for (int f = 0; f < g.nf; ++f) {
      const int64_t ne = neighbour(&g, e, f);
      if (ne >= 0) {
        if (e < ne) {   /* ApplyOn::InnerIntersectionsPrimally */
          local_inner(&c, q, e, f, ne, L, EN, NE, NN);
          scatter(&c, e, e, L); scatter(&c, e, ne, EN); scatter(&c, ne, e, NE); scatter(&c, ne, ne, NN);
        }
      } else if (prm->boundary_kind == OR_QP_BOUNDARY_DIRICHLET) {
        local_boundary(&c, q, e, f, L);
        scatter(&c, e, e, L);
      }
    }
  }
  free(buf);
  free(q);
  return 0;
}

/* products, over_integrate = 2 (kinds as OR_PRODUCT_* of swipdg_oracle.h: 0 L2, 1 H1 semi, 2 elliptic,
 * 3 boundary L2, 4 SWIPDG penalty) */
int or_qp_product(const or_qp_grid_t* in, int kind, const or_qp_scalar_t* kappa, const or_qp_tensor_t* A,
                  const or_qp_params_t* prm, const int64_t* elem_index, const int64_t* row_ptr, const int32_t* col,
                  double* val)
{
  qgrid_t g;
  if (init_grid(in, &g)) return -1;
  qctx_t c = {&g, kappa, A, prm, elem_index, row_ptr, col, val};
  const int nb = g.nb, d = g.dim, over = 2;
  memset(val, 0, sizeof(double) * (size_t)row_ptr[g.ne * nb]);
  double* buf = (double*)malloc(sizeof(double) * (size_t)(4 * nb * nb));
  double *L = buf, *EN = buf + nb * nb, *NE = buf + 2 * nb * nb, *NN = buf + 3 * nb * nb;
  qrule_t* q = (qrule_t*)malloc(sizeof(qrule_t));
  double phi[125], gh[125][3], gp[125][3], pn[125], ghn[125][3];
  for (int64_t e = 0; e < g.ne; ++e) {
    geo_t G;
    geometry(&g, e, &G);
    if (kind <= 2) {
      int order = kind == 0 ? 2 * g.p + over : 2 * (g.p - 1) + over;
      if (kind == 2) order += scalar_order(kappa);
      double Am[3][3];
      if (kind == 2) eval_tensor(&g, A, e, Am);
      tensor_rule(d, order, q);
      memset(L, 0, sizeof(double) * (size_t)(nb * nb));
      for (int k = 0; k < q->n; ++k) {
        double x[3], Ag[3];
        shape(&g, q->x[k], phi, gh);
        global_pt(&G, q->x[k], x);
        for (int i = 0; i < nb; ++i) map_grad(&G, gh[i], gp[i]);
        const double w = q->w[k] * fabs(G.det) * (kind == 2 ? eval_scalar(kappa, e, x) : 1.0);
        for (int i = 0; i < nb; ++i)
          for (int j = 0; j < nb; ++j) {
            double v;
            if (kind == 0) v = phi[i] * phi[j];
            else if (kind == 1) v = dot(d, gp[i], gp[j]);
            else { matvec(d, Am, gp[j], Ag); v = dot(d, Ag, gp[i]); }
            L[i * nb + j] += w * v;
          }
      }
      scatter(&c, e, e, L);
      continue;
    }
    for (int f = 0; f < g.nf; ++f) {
      const int64_t ne = neighbour(&g, e, f);
      double n[3], fvol;
      face_normal(&G, f, n, &fvol);
      if (kind == 3) {
        if (ne >= 0) continue;
        tensor_rule(d - 1, 2 * g.p + over, q);
        memset(L, 0, sizeof(double) * (size_t)(nb * nb));
        for (int k = 0; k < q->n; ++k) {
          double xin[3];
          face_ref_point(d, f, q->x[k], xin);
          shape(&g, xin, phi, gh);
          for (int i = 0; i < nb; ++i)
            for (int j = 0; j < nb; ++j) L[i * nb + j] += q->w[k] * fvol * phi[i] * phi[j];
        }
        scatter(&c, e, e, L);
        continue;
      }
      if (ne < 0 && prm->boundary_kind != OR_QP_BOUNDARY_DIRICHLET) continue;
      if (ne >= 0 && !(e < ne)) continue;
      double Ai[3][3], An_i[3];
      eval_tensor(&g, A, e, Ai);
      matvec(d, Ai, n, An_i);
      const double dm = dot(d, n, An_i);
      double gamma = dm, sigma = prm->sigma_boundary;
      geo_t Go;
      if (ne >= 0) {
        double Ao[3][3], An_o[3];
        eval_tensor(&g, A, ne, Ao);
        matvec(d, Ao, n, An_o);
        geometry(&g, ne, &Go);
        const double dp = dot(d, n, An_o);
        gamma = dp * dm / (dp + dm);
        sigma = prm->sigma_inner;
      }
      const double hpow = pow(fvol, prm->beta);
      tensor_rule(d - 1, scalar_order(kappa) + 2 * g.p + over, q);
      const size_t sz = sizeof(double) * (size_t)(nb * nb);
      memset(L, 0, sz); memset(EN, 0, sz); memset(NE, 0, sz); memset(NN, 0, sz);
      for (int k = 0; k < q->n; ++k) {
        double xin[3], x[3], xout[3];
        face_ref_point(d, f, q->x[k], xin);
        global_pt(&G, xin, x);
        shape(&g, xin, phi, gh);
        const double ke = eval_scalar(kappa, e, x);
        double pen;
        if (ne >= 0) {
          local_pt(&Go, x, xout);
          shape(&g, xout, pn, ghn);
          pen = ke * eval_scalar(kappa, ne, x) * sigma * gamma / hpow;
        } else {
          for (int i = 0; i < nb; ++i) pn[i] = 0.0;
          pen = ke * sigma * gamma / hpow;
        }
        const double fac = q->w[k] * fvol * pen;
        for (int i = 0; i < nb; ++i)
          for (int j = 0; j < nb; ++j) {
            L[i * nb + j] += fac * phi[j] * phi[i];
            EN[i * nb + j] -= fac * pn[j] * phi[i];
            NE[i * nb + j] -= fac * phi[j] * pn[i];
            NN[i * nb + j] += fac * pn[j] * pn[i];
          }
      }
      scatter(&c, e, e, L);
      if (ne >= 0) { scatter(&c, e, ne, EN); scatter(&c, ne, e, NE); scatter(&c, ne, ne, NN); }
    }
  }
  free(buf);
  free(q);
  return 0;
}

/* SWIPDG right-hand side (see or_rhs_swipdg in swipdg_oracle.c for the functionals and orders) */
int or_qp_rhs_swipdg(const or_qp_grid_t* in, const or_qp_scalar_t* force, const or_qp_scalar_t* kappa,
                     const or_qp_tensor_t* A, const or_qp_scalar_t* dirichlet, const or_qp_scalar_t* neumann,
                     const or_qp_params_t* prm, const int64_t* elem_index, double* b)
{
  qgrid_t g;
  if (init_grid(in, &g)) return -1;
  const int nb = g.nb, d = g.dim;
  qrule_t* q = (qrule_t*)malloc(sizeof(qrule_t));
  memset(b, 0, sizeof(double) * (size_t)(g.ne * nb));
  double phi[125], gh[125][3], gp[3];
  for (int64_t e = 0; e < g.ne; ++e) {
    geo_t G;
    geometry(&g, e, &G);
    double* be = b + gid_of(elem_index, e) * nb;
    if (force) {
      tensor_rule(d, scalar_order(force) + g.p, q);
      for (int k = 0; k < q->n; ++k) {
        double x[3];
        shape(&g, q->x[k], phi, gh);
        global_pt(&G, q->x[k], x);
        const double fv = eval_scalar(force, e, x) * q->w[k] * fabs(G.det);
        for (int i = 0; i < nb; ++i) be[i] += fv * phi[i];
      }
    }
    for (int f = 0; f < g.nf; ++f) {
      if (neighbour(&g, e, f) >= 0) continue;
      const int dir = prm->boundary_kind == OR_QP_BOUNDARY_DIRICHLET;
      const or_qp_scalar_t* data = dir ? dirichlet : neumann;
      if (!data) continue;
      double n[3], fvol, Am[3][3], An[3];
      face_normal(&G, f, n, &fvol);
      eval_tensor(&g, A, e, Am);
      matvec(d, Am, n, An);
      const double gamma = dot(d, n, An), hpow = pow(fvol, prm->beta);
      int order = scalar_order(data) + g.p;
      if (dir) {
        const int o2 = scalar_order(kappa) + 0 + (g.p - 1) + scalar_order(data);
        if (o2 > order) order = o2;
      }
      tensor_rule(d - 1, order, q);
      for (int k = 0; k < q->n; ++k) {
        double xin[3], x[3];
        face_ref_point(d, f, q->x[k], xin);
        global_pt(&G, xin, x);
        shape(&g, xin, phi, gh);
        const double gv = eval_scalar(data, e, x) * q->w[k] * fvol;
        if (dir) {
          const double kap = eval_scalar(kappa, e, x);
          const double pen = prm->sigma_boundary * kap * gamma / hpow;
          for (int i = 0; i < nb; ++i) {
            map_grad(&G, gh[i], gp);
            be[i] += gv * (-kap * dot(d, An, gp) + pen * phi[i]);
          }
        } else {
          for (int i = 0; i < nb; ++i) be[i] += gv * phi[i];
        }
      }
    }
  }
  free(q);
  return 0;
}

/* ESV2007 testcase extended to d dimensions: u = prod cos(pi x_a / 2), f = d pi^2/4 u (kappa = 1, A = I) */
static double esv_u(int d, const double* x)
{
  double u = 1.0;
  for (int a = 0; a < d; ++a) u *= cos(0.5 * M_PI * x[a]);
  return u;
}

int or_qp_rhs_esv2007(const or_qp_grid_t* in, int force_order, const int64_t* elem_index, double* b)
{
  qgrid_t g;
  if (init_grid(in, &g)) return -1;
  qrule_t* q = (qrule_t*)malloc(sizeof(qrule_t));
  tensor_rule(g.dim, force_order + g.p, q);
  memset(b, 0, sizeof(double) * (size_t)(g.ne * g.nb));
  double phi[125], gh[125][3];
  for (int64_t e = 0; e < g.ne; ++e) {
    geo_t G;
    geometry(&g, e, &G);
    const int64_t gid = gid_of(elem_index, e);
    for (int k = 0; k < q->n; ++k) {
      double x[3];
      shape(&g, q->x[k], phi, gh);
      global_pt(&G, q->x[k], x);
      const double fv = 0.25 * g.dim * M_PI * M_PI * esv_u(g.dim, x) * q->w[k] * fabs(G.det);
      for (int i = 0; i < g.nb; ++i) b[gid * g.nb + i] += fv * phi[i];
    }
  }
  free(q);
  return 0;
}

int or_qp_error_esv2007(const or_qp_grid_t* in, const double* u, const int64_t* elem_index, int order, double* l2,
                        double* h1)
{
  qgrid_t g;
  if (init_grid(in, &g)) return -1;
  qrule_t* q = (qrule_t*)malloc(sizeof(qrule_t));
  tensor_rule(g.dim, order, q);
  double sl2 = 0.0, sh1 = 0.0;
  double phi[125], gh[125][3], gp[3];
  for (int64_t e = 0; e < g.ne; ++e) {
    geo_t G;
    geometry(&g, e, &G);
    const double* ue = u + gid_of(elem_index, e) * g.nb;
    for (int k = 0; k < q->n; ++k) {
      double x[3], uh = 0.0, guh[3] = {0.0, 0.0, 0.0}, gu[3];
      shape(&g, q->x[k], phi, gh);
      global_pt(&G, q->x[k], x);
      for (int i = 0; i < g.nb; ++i) {
        map_grad(&G, gh[i], gp);
        uh += ue[i] * phi[i];
        for (int a = 0; a < g.dim; ++a) guh[a] += ue[i] * gp[a];
      }
      for (int a = 0; a < g.dim; ++a) {
        gu[a] = -0.5 * M_PI * sin(0.5 * M_PI * x[a]);
        for (int b = 0; b < g.dim; ++b)
          if (b != a) gu[a] *= cos(0.5 * M_PI * x[b]);
      }
      const double w = q->w[k] * fabs(G.det), dd = esv_u(g.dim, x) - uh;
      sl2 += w * dd * dd;
      for (int a = 0; a < g.dim; ++a) sh1 += w * (gu[a] - guh[a]) * (gu[a] - guh[a]);
    }
  }
  free(q);
  *l2 = sqrt(sl2);
  *h1 = sqrt(sh1);
  return 0;
}
