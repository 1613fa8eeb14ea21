// dune-hdd_amd/csrc/kernels/abi_device.hip
//
// Device half of the C ABI: context, SWIPDG assembly dispatch, the theta-lincomb of affine components
// (AffinelyDecomposedContainer::freeze_parameter, base.hh:338-341) and the SoA halo gather/scatter used
// around the RCCL face-halo exchange of a sharded BlockSWIPDG.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "hdd.h"
#include "../host/hdd_internal.hh"
#include "swipdg_kernels.hh"

struct hdd_ctx {
  int device = 0;
  void* ws = nullptr;       // device workspace (per-element coefficient records of the p=3 hex kernel)
  size_t ws_bytes = 0;
  // read once at hdd_ctx_create, never per launch
  int n_cu = 256;           // hipDeviceAttributeMultiprocessorCount
  int debug_flags = 0;      // HDD_DEBUG_FLAGS: error injection of the tests; ablation bits (HDD_ABLATION builds only)
  uint32_t variant = 0;     // hdd_ctx_set_variant (ablation build: also HDD_VARIANT): verification variants (0: default)
  int wgcu = 0;             // ablation build, HDD_P1_WGCU: tiles-per-CU sweep override (0: the policy's measured value)
  int q3g_reps = 0;         // ablation build, HDD_Q3G_REPS: workgroups per (XCD, row quad) of the p=3 GEMM kernel
  double* q3g_tab = nullptr;   // p=3 reference matrices [Q3G_K][4096], uploaded on first use
  void* scan_ws = nullptr;     // device-pattern row-length scan scratch (kept: no allocation per build)
  size_t scan_ws_bytes = 0;
  void* ops_d = nullptr;       // batched block operators: device descriptor table,
  void* ops_h = nullptr;       //   its pinned host staging copy (reused once the last upload has completed)
  size_t ops_bytes = 0;
  hipEvent_t ops_evt = nullptr;
  int64_t* nnz_h = nullptr;    // mapped pinned host word: the device pattern's nnz, written by the elem_ptr kernel
  int64_t* nnz_hd = nullptr;   //   (its device address)
  void* rhs_ws = nullptr;      // 2d RHS boundary-element list (counters zero between calls)
  size_t rhs_ws_bytes = 0;
  hipStream_t rhs_stream = nullptr;   // stream of the last split RHS call, and an event behind its face kernel:
  hipEvent_t rhs_evt = nullptr;       //   a call on another stream waits for it (the list is shared state)
  bool rhs_used = false;
};

int hdd::ctx_device(const hdd_ctx* ctx) { return ctx ? ctx->device : 0; }

// grows the context workspace; allocation happens only on the first call of a size class, so warm the
// context up once before capturing hdd_swipdg_assemble into a hipGraph
static hipError_t ctx_workspace(hdd_ctx* ctx, size_t bytes, void** out)
{
  if (bytes > ctx->ws_bytes) {
    if (ctx->ws) (void)hipFree(ctx->ws);
    ctx->ws = nullptr;
    ctx->ws_bytes = 0;
    const size_t grow = bytes + bytes / 4;
    hipError_t e = hipMalloc(&ctx->ws, grow);
    if (e != hipSuccess) return e;
    ctx->ws_bytes = grow;
  }
  *out = ctx->ws;
  return hipSuccess;
}

using hdd::set_error;

// vertex-indexed geometry is read with 32-bit byte offsets (swipdg_device.hh rsrc32): every [rows][n_local] int32 /
// f64 row offset and every vertex row (at most 3 n_local vertices of 16 B) must stay below 2^32
static bool vx_offsets_fit(int64_t n_local) { return n_local >= 0 && n_local * 48 < (int64_t(1) << 32); }

static int hip_fail(hipError_t e, const char* where)
{
  return set_error(HDD_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

extern "C" int hdd_ctx_create(int hip_device, hdd_ctx** out)
{
  if (!out) return set_error(HDD_ERR_INVALID, "hdd_ctx_create: null out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return hip_fail(e, "hdd_ctx_create: hipGetDeviceCount");
  if (hip_device < 0 || hip_device >= n) return set_error(HDD_ERR_RANGE, "hdd_ctx_create: no such HIP device");
  e = hipSetDevice(hip_device);
  if (e != hipSuccess) return hip_fail(e, "hdd_ctx_create: hipSetDevice");
  auto* c = new hdd_ctx;
  c->device = hip_device;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, hip_device) == hipSuccess && cus > 0)
    c->n_cu = cus;
  if (const char* df = getenv("HDD_DEBUG_FLAGS")) c->debug_flags = atoi(df);
#ifdef HDD_ABLATION
  // study knobs: only the ablation build reads them from the environment, so an inherited variable cannot change
  // which kernel a release build times; the tests select variants with hdd_ctx_set_variant
  if (const char* v = getenv("HDD_VARIANT")) c->variant = uint32_t(strtoul(v, nullptr, 0));
  if (const char* w = getenv("HDD_P1_WGCU")) c->wgcu = std::max(0, atoi(w));
  if (const char* r = getenv("HDD_Q3G_REPS")) c->q3g_reps = std::max(0, atoi(r));
#endif
  *out = c;
  return HDD_OK;
}

extern "C" int hdd_ctx_set_debug_flags(hdd_ctx* ctx, int32_t flags)
{
  if (!ctx) return set_error(HDD_ERR_INVALID, "hdd_ctx_set_debug_flags: null context");
  ctx->debug_flags = flags;
  return HDD_OK;
}

extern "C" int hdd_ctx_set_variant(hdd_ctx* ctx, uint32_t variant)
{
  if (!ctx) return set_error(HDD_ERR_INVALID, "hdd_ctx_set_variant: null context");
  ctx->variant = variant;
  return HDD_OK;
}

extern "C" void hdd_ctx_destroy(hdd_ctx* ctx)
{
  if (ctx && ctx->ws) (void)hipFree(ctx->ws);
  if (ctx && ctx->q3g_tab) (void)hipFree(ctx->q3g_tab);
  if (ctx && ctx->scan_ws) (void)hipFree(ctx->scan_ws);
  if (ctx && ctx->rhs_ws) (void)hipFree(ctx->rhs_ws);
  if (ctx && ctx->rhs_evt) (void)hipEventDestroy(ctx->rhs_evt);
  if (ctx && ctx->nnz_h) (void)hipHostFree(ctx->nnz_h);
  if (ctx && ctx->ops_d) (void)hipFree(ctx->ops_d);
  if (ctx && ctx->ops_h) (void)hipHostFree(ctx->ops_h);
  if (ctx && ctx->ops_evt) (void)hipEventDestroy(ctx->ops_evt);
  delete ctx;
}

static int fn_order(const hdd_scalar_fn& f)
{
  return (f.kind == HDD_FN_SINUSOID || f.kind == HDD_FN_COS_PRODUCT || f.kind == HDD_FN_FLATTOP) ? f.order : 0;
}

// ---------------------------------------------------------------------------------------------------
// HDD_HEX: Q_p on affine hexahedra (hex_qp.hip)
// ---------------------------------------------------------------------------------------------------
static void gauss_legendre01(int n, double* x, double* w)   // Newton on P_n, mapped to [0,1]
{
  for (int i = 0; i < n; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5)), dp = 1.0;
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = z;
      for (int k = 2; k <= n; ++k) {
        const double p2 = ((2.0 * k - 1.0) * z * p1 - (k - 1.0) * p0) / k;
        p0 = p1;
        p1 = p2;
      }
      if (n == 1) { p0 = 1.0; p1 = z; }
      dp = n * (z * p1 - p0) / (z * z - 1.0);
      const double dz = p1 / dp;
      z -= dz;
      if (std::fabs(dz) < 1e-16) {
        double q0 = 1.0, q1 = z;
        for (int k = 2; k <= n; ++k) {
          const double q2 = ((2.0 * k - 1.0) * z * q1 - (k - 1.0) * q0) / k;
          q0 = q1;
          q1 = q2;
        }
        if (n == 1) { q0 = 1.0; q1 = z; }
        dp = n * (z * q1 - q0) / (z * z - 1.0);
        break;
      }
    }
    x[n - 1 - i] = 0.5 * (z + 1.0);
    w[n - 1 - i] = 1.0 / ((1.0 - z * z) * dp * dp);
  }
}

// equidistant Lagrange polynomial k of degree p and its derivative at x
static void lagrange_1d(int p, int k, double x, double* v, double* d)
{
  double val = 1.0, der = 0.0;
  for (int m = 0; m <= p; ++m) {
    if (m == k) continue;
    const double den = double(k - m) / p, f = (x - double(m) / p) / den;
    der = der * f + val / den;
    val *= f;
  }
  *v = val;
  *d = der;
}

static int assemble_hex(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                        const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                        double* const* d_vals, void* stream)
{
  using namespace hdd::dev;
  const int deg = m->degree < 1 ? 1 : m->degree;
  if (deg > 3) return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: HDD_HEX supports p = 1..3");
  const int nb = (deg + 1) * (deg + 1) * (deg + 1);
  if (pattern->n_rows != int64_t(nb) * (m->own_end - m->own_begin))
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: pattern rows != nb * owned elements");
  if (tensor->kind != HDD_TENSOR_CONST && tensor->kind != HDD_TENSOR_ISO_PER_ELEM &&
      tensor->kind != HDD_TENSOR_SYM_PER_ELEM)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: unknown tensor kind");
  if (tensor->kind != HDD_TENSOR_CONST && !tensor->per_elem)
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: tensor per_elem missing");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_swipdg_assemble: hipSetDevice");
  for (int c = 0; c < n_comp; ++c) {
    const hdd_scalar_fn& k = kappa[c];
    if (k.kind != HDD_FN_CONST && k.kind != HDD_FN_PER_ELEM && k.kind != HDD_FN_SINUSOID)
      return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: unknown diffusion factor kind");
    if (k.kind == HDD_FN_PER_ELEM && !k.per_elem)
      return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: diffusion factor per_elem missing");
    if (!d_vals[c]) return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: null value array");
    // integrand orders (dune-gdt): volume ord(kappa) + ord(A) + 2 (p-1), faces ord(kappa) + ord(A) + 2p
    const int ko = fn_order(k);
    const int vol_order = p->vol_order >= 0 ? p->vol_order : ko + 2 * (deg - 1);
    const int face_order = p->face_order >= 0 ? p->face_order : ko + 2 * deg;
    const int nq1v = std::max(1, (vol_order + 2) / 2), nq1f = std::max(1, (face_order + 2) / 2);
    if (nq1v > 8 || nq1f > 8)
      return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: quadrature order too high for HDD_HEX");
    HexArgs a{};
    a.n_local = m->n_local;
    a.own_begin = m->own_begin;
    a.own_end = m->own_end;
    a.coords = m->coords;
    a.nbrs = m->neighbors;
    a.elem_ptr = pattern->elem_ptr;
    a.tkind = tensor->kind;
    for (int r = 0; r < 6; ++r) a.tc[r] = tensor->c[r];
    a.tper = tensor->per_elem;
    a.kkind = k.kind;
    a.kc = k.c;
    a.kb = k.b;
    a.kx = k.kx;
    a.ky = k.ky;
    a.kper = k.per_elem;
    a.vals = d_vals[c];
    a.sigma_inner = p->sigma_inner;
    a.sigma_boundary = p->sigma_boundary;
    a.beta = p->beta;
    a.debug_flags = ctx->debug_flags;   // profiling ablations (HDD_ABLATION builds only)
    a.variant = ctx->variant;
    gauss_legendre01(nq1v, a.tab.sv, a.tab.wv);
    gauss_legendre01(nq1f, a.tab.sf, a.tab.wf);
    for (int r = 0; r <= deg; ++r) {
      for (int q = 0; q < nq1v; ++q) lagrange_1d(deg, r, a.tab.sv[q], &a.tab.Lv[r][q], &a.tab.Dv[r][q]);
      for (int q = 0; q < nq1f; ++q) lagrange_1d(deg, r, a.tab.sf[q], &a.tab.Lf[r][q], &a.tab.Df[r][q]);
      for (int q = 0; q < 2; ++q) lagrange_1d(deg, r, double(q), &a.tab.Le[r][q], &a.tab.De[r][q]);
    }
    if (hex_uses_records(a, deg, nq1v, nq1f)) {
      const int64_t n_own = std::max<int64_t>(1, m->own_end - m->own_begin);
      void* ws = nullptr;
      e = ctx_workspace(ctx, hex_q3_workspace_doubles(n_own) * sizeof(double), &ws);
      if (e != hipSuccess) return hip_fail(e, "hdd_swipdg_assemble: workspace");
      a.ws = static_cast<double*>(ws);
      a.q3g_coef = a.ws + n_own * HEX_REC;
      a.q3g_meta = reinterpret_cast<int64_t*>(a.q3g_coef + (n_own + 15) / 16 * 16 * Q3G_K);
      if (!ctx->q3g_tab) {   // element-independent: the 1D tables are fixed for (p, nq1v, nq1f) = (3, 3, 4)
        std::vector<double> tab(size_t(Q3G_K) * 4096);
        hex_q3g_reference_tables(a.tab, tab.data());
        e = hipMalloc(&ctx->q3g_tab, tab.size() * sizeof(double));
        if (e != hipSuccess) return hip_fail(e, "hdd_swipdg_assemble: reference matrices");
        e = hipMemcpy(ctx->q3g_tab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_fail(e, "hdd_swipdg_assemble: reference matrices");
      }
      a.q3g_tab = ctx->q3g_tab;
      // 4 row waves per workgroup, 128 workgroups per replica: 2 replicas per 128 CUs (8 waves per CU)
      a.q3g_reps = ctx->q3g_reps > 0 ? ctx->q3g_reps : std::max(1, ctx->n_cu / 64);
    }
    bool supported = false;
    e = launch_hex(a, deg, nq1v, nq1f, static_cast<hipStream_t>(stream), &supported);
    if (!supported)
      return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: no HDD_HEX kernel for p=" + std::to_string(deg) +
                                                ", volume order " + std::to_string(vol_order) + ", face order " +
                                                std::to_string(face_order));
    if (e != hipSuccess) return hip_fail(e, "hdd_swipdg_assemble: launch");
  }
  return HDD_OK;
}

static int assemble_impl(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                         const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                         double* const* d_vals, const int32_t* d_tiles, int64_t n_tiles, void* stream,
                         int list_elements = 0, bool skip_ghost = false, int32_t reserve_wg = 0,
                         int64_t fix_ld = 0)
{
  using namespace hdd::dev;
  if (!ctx || !m || !kappa || !tensor || !p || !pattern || !d_vals)
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: null argument");
  if (n_comp < 1 || n_comp > HDD_MAX_COMP)
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: need 1 <= n_comp <= HDD_MAX_COMP");
  if (m->elem_type != HDD_SIMPLEX && m->elem_type != HDD_CUBE && m->elem_type != HDD_HEX)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: unknown element type");
  if (!m->coords || !m->neighbors || !m->face_info || !pattern->elem_ptr)
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: mesh / pattern arrays missing");
  if (m->own_begin < 0 || m->own_end > m->n_local || m->own_begin > m->own_end)
    return set_error(HDD_ERR_RANGE, "hdd_swipdg_assemble: 0 <= own_begin <= own_end <= n_local violated");
  if (m->n_local >= int64_t(INT32_MAX))
    return set_error(HDD_ERR_RANGE, "hdd_swipdg_assemble: n_local must fit int32 neighbour ids");
  // hdd_last_tile_kernel names the kernel THIS call launches (every launch path sets it); an element-list pass (the
  // sharded step's side pass beside its tile launch) leaves the tile launch's name in place
  if (!list_elements) hdd::last_tile_kernel_slot() = "";
  // The sharded step (shard.hip) runs this function on two streams at once with one context: the element-list
  // pass on the transfer stream beside the SKIP launch on the caller's stream.  That is safe only because the
  // 2d paths below (tiles, element lists, skip_ghost) use no context workspace (ws / scan_ws / rhs_ws); the
  // one path that does (HDD_HEX, p = 3) takes no lists, and the sharded step runs it exchange-then-assemble.
  if (m->elem_type == HDD_HEX) {
    if (d_tiles || skip_ghost)
      return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble_tiles: no tile / element lists for HDD_HEX");
    return assemble_hex(ctx, m, kappa, n_comp, tensor, p, pattern, d_vals, stream);
  }
  if (m->degree > 1)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: 2d meshes carry P1 / Q1 only (degree <= 1)");
  const int nb = m->elem_type == HDD_SIMPLEX ? 3 : 4;
  if (pattern->n_rows != int64_t(nb) * (m->own_end - m->own_begin))
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: pattern rows != nb * owned elements");
  // The reference requires a non-parametric, non-empty tensor (swipdg.hh:173-176); here the tensor is a
  // plain function, so only its kind is checked.
  if (tensor->kind != HDD_TENSOR_CONST && tensor->kind != HDD_TENSOR_ISO_PER_ELEM &&
      tensor->kind != HDD_TENSOR_SYM_PER_ELEM)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: unknown tensor kind");
  if (tensor->kind != HDD_TENSOR_CONST && !tensor->per_elem)
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: tensor per_elem missing");
  AssembleArgs a{};
  a.elem_type = m->elem_type;
  a.n_comp = n_comp;
  a.n_local = m->n_local;
  a.own_begin = m->own_begin;
  a.own_end = m->own_end;
  a.coords = m->coords;
  a.nbrs = m->neighbors;
  a.finfo = m->face_info;
  a.elem_ptr = pattern->elem_ptr;
  a.tkind = tensor->kind;
  a.tc0 = tensor->c[0];
  a.tc1 = tensor->c[1];
  a.tc2 = tensor->c[2];
  a.tper = tensor->per_elem;
  a.sigma_inner = p->sigma_inner;
  a.sigma_boundary = p->sigma_boundary;
  a.beta = p->beta;
  a.tile_list = d_tiles;
  a.n_tile_list = n_tiles;
  a.list_elements = list_elements;
  a.skip_ghost = skip_ghost ? 1 : 0;
  a.reserve_wg = list_elements ? 0 : reserve_wg;
  a.fix_ld = fix_ld;
  a.fix_rb = (m->elem_type == HDD_SIMPLEX ? 3 * 3 * 4 : 4 * 4 * 5);
  if (!m->elem_vertices != !m->vertex_coords)
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: mesh elem_vertices / vertex_coords: both or neither");
  // vertex-indexed geometry (HDD_VARIANT_ELEMENT_MAJOR: the element-major coords, cross-check)
  // (the P1 vertex-indexed loads use 32-bit byte offsets: meshes beyond n_local * 48 >= 2^32 take the element-major
  // coords, vx_offsets_fit)
  if (m->elem_vertices && !(ctx->variant & HDD_VARIANT_ELEMENT_MAJOR) && vx_offsets_fit(m->n_local)) {
    a.ev = m->elem_vertices;
    a.vxy = m->vertex_coords;
  }
  a.n_cu = ctx->n_cu;
  a.debug_flags = ctx->debug_flags;   // profiling ablations only
  a.variant = ctx->variant;
  a.wgcu = ctx->wgcu;
  // integrand orders of LocalEvaluation::Elliptic / SWIPDG::Inner / BoundaryLHS at p = 1 (piecewise
  // constant tensors): volume ord(kappa); faces ord(kappa) + 2.  One kernel serves components of equal
  // order -- the caller splits mixed-order component sets.
  const int ko = fn_order(kappa[0]);
  for (int c = 0; c < n_comp; ++c) {
    const hdd_scalar_fn& k = kappa[c];
    if (k.kind != HDD_FN_CONST && k.kind != HDD_FN_PER_ELEM && k.kind != HDD_FN_SINUSOID && k.kind != HDD_FN_FLATTOP)
      return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: unknown diffusion factor kind");
    if (k.kind == HDD_FN_PER_ELEM && !k.per_elem)
      return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: diffusion factor per_elem missing");
    if (fn_order(k) != ko)
      return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: components of different integration order");
    if (!d_vals[c]) return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: null value array");
    if (k.kind == HDD_FN_FLATTOP && (k.n_table < 0 || (k.n_table > 0 && !k.table)))
      return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble: FLATTOP box table missing");
    a.kappa[c] = KappaArg{k.kind, k.order, k.c, k.b, k.kx, k.ky, k.per_elem, k.table, k.n_table, 0};
    a.vals[c] = d_vals[c];
  }
  const int vol_order = p->vol_order >= 0 ? p->vol_order : ko;
  const int face_order = p->face_order >= 0 ? p->face_order : ko + 2;
  const int nqv = volume_points(m->elem_type, vol_order);
  const int nqf = face_points(face_order);
  bool supported = false;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_swipdg_assemble: hipSetDevice");
  e = launch_assemble(a, nqv, nqf, static_cast<hipStream_t>(stream), &supported);
  if (!supported)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_assemble: no kernel for volume order " + std::to_string(vol_order) +
                                              " / face order " + std::to_string(face_order));
  if (e != hipSuccess) return hip_fail(e, "hdd_swipdg_assemble: launch");
  return HDD_OK;
}

extern "C" int hdd_swipdg_assemble(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                                   const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                                   double* const* d_vals, void* stream)
{
  return assemble_impl(ctx, m, kappa, n_comp, tensor, p, pattern, d_vals, nullptr, 0, stream);
}

extern "C" int hdd_swipdg_assemble_tiles(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                                         const hdd_tensor_fn* tensor, const hdd_swipdg_params* p,
                                         const hdd_csr* pattern, double* const* d_vals, const int32_t* d_tiles,
                                         int64_t n_tiles, void* stream)
{
  if (!d_tiles && n_tiles) return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble_tiles: null tile list");
  if (n_tiles == 0) return HDD_OK;
  return assemble_impl(ctx, m, kappa, n_comp, tensor, p, pattern, d_vals, d_tiles, n_tiles, stream);
}

extern "C" int hdd_swipdg_assemble_elements(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa,
                                            int32_t n_comp, const hdd_tensor_fn* tensor, const hdd_swipdg_params* p,
                                            const hdd_csr* pattern, double* const* d_vals, const int32_t* d_elems,
                                            int64_t n_elems, void* stream)
{
  if (!d_elems && n_elems) return set_error(HDD_ERR_INVALID, "hdd_swipdg_assemble_elements: null element list");
  if (n_elems == 0) return HDD_OK;
  return assemble_impl(ctx, m, kappa, n_comp, tensor, p, pattern, d_vals, d_elems, n_elems, stream, 1);
}

// ------------------------------------------------------------------------------------------------
// Sharded-step fixup off the assembly stream (shard.hip): the element-list pass writes each listed element's row
// block into a side buffer (slot fix_rb(m) doubles, one buffer of n + 1 slots per component) on the transfer
// stream while the full-range assembly runs; after the join, fix_scatter_kernel copies the blocks into place.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) fix_scatter_kernel(const double* __restrict__ buf, int32_t rb,
                                                         const int32_t* __restrict__ list, int64_t n,
                                                         const int64_t* __restrict__ elem_ptr, double* vals)
{
  for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const int64_t el = list[i];
    const int64_t b = elem_ptr[el], len = elem_ptr[el + 1] - b;
    for (int64_t k = threadIdx.x; k < len; k += 64) vals[b + k] = buf[i * rb + k];
  }
}

int hdd_fix_rb(int32_t elem_type) { return elem_type == HDD_SIMPLEX ? 3 * 3 * 4 : 4 * 4 * 5; }

int hdd_assemble_elements_buf(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                              const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                              double* const* d_bufs, const int32_t* d_elems, int64_t n_elems, void* stream)
{
  if (n_elems == 0) return HDD_OK;
  return assemble_impl(ctx, m, kappa, n_comp, tensor, p, pattern, d_bufs, d_elems, n_elems, stream, 2);
}

int hdd_assemble_elements_inplace(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                                  const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                                  double* const* d_vals, const int32_t* d_elems, int64_t n_elems, void* stream)
{
  if (n_elems == 0) return HDD_OK;
  return assemble_impl(ctx, m, kappa, n_comp, tensor, p, pattern, d_vals, d_elems, n_elems, stream, 3);
}

int hdd_assemble_elements_soa(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                              const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                              double* const* d_bufs, int64_t ld, const int32_t* d_elems, int64_t n_elems, void* stream)
{
  if (n_elems == 0) return HDD_OK;
  if (m->elem_type != HDD_CUBE) return set_error(HDD_ERR_UNSUPPORTED, "hdd_assemble_elements_soa: Q1 only");
  return assemble_impl(ctx, m, kappa, n_comp, tensor, p, pattern, d_bufs, d_elems, n_elems, stream, 4, false, 0, ld);
}

int hdd_assemble_reserve(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                         const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                         double* const* d_vals, void* stream, int32_t reserve_wg)
{
  return assemble_impl(ctx, m, kappa, n_comp, tensor, p, pattern, d_vals, nullptr, 0, stream, 0, false, reserve_wg);
}

int hdd_scatter_fix_q1_soa(hdd_ctx* ctx, const hdd_mesh* m, const hdd_csr* pattern, double* const* d_bufs, int64_t ld,
                           int32_t n_comp, const int32_t* d_elems, int64_t n_elems, double* const* d_vals, void* stream)
{
  if (n_elems == 0) return HDD_OK;
  hdd::dev::AssembleArgs a{};
  a.n_local = m->n_local;
  a.own_begin = m->own_begin;
  a.own_end = m->own_end;
  a.nbrs = m->neighbors;
  a.finfo = m->face_info;
  a.elem_ptr = pattern->elem_ptr;
  a.tile_list = d_elems;
  a.n_tile_list = n_elems;
  a.n_cu = ctx->n_cu;
  for (int32_t c = 0; c < n_comp; ++c) {
    const hipError_t e = hdd::dev::launch_q1_scatter_soa(a, d_bufs[c], ld, d_vals[c], static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "hdd_scatter_fix_q1_soa");
  }
  return HDD_OK;
}

int hdd_assemble_skip_ghost(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                            const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                            double* const* d_vals, void* stream, int32_t reserve_wg)
{
  return assemble_impl(ctx, m, kappa, n_comp, tensor, p, pattern, d_vals, nullptr, 0, stream, 0, true, reserve_wg);
}

int hdd_scatter_fix(hdd_ctx* ctx, const hdd_csr* pattern, int32_t rb, double* const* d_bufs, int32_t n_comp,
                    const int32_t* d_elems, int64_t n_elems, double* const* d_vals, void* stream)
{
  if (n_elems == 0) return HDD_OK;
  const unsigned grid = unsigned(std::min<int64_t>(n_elems, int64_t(ctx->n_cu) * 8));
  for (int32_t c = 0; c < n_comp; ++c) {
    hipLaunchKernelGGL(fix_scatter_kernel, dim3(grid), dim3(64), 0, static_cast<hipStream_t>(stream), d_bufs[c], rb,
                       d_elems, n_elems, pattern->elem_ptr, d_vals[c]);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "hdd_scatter_fix");
  }
  return HDD_OK;
}

// ------------------------------------------------------------------------------------------------
// theta-lincomb: out[s][k] = sum_q theta[s][q] v_q[k]; up to LC_T / n_comp samples per launch (128 for the
// affine + 1 component case: the components are read once for all of them), 2 values per lane written as one
// 16-byte non-temporal store per sample.  All samples in one launch: 12.5-12.7 ms for 128 C3 samples against
// 15.2 ms in launches of 32 (scripts/microbench/lincomb_mb.hip, profiles/r02/s3/lincomb_mb.log).
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int LC_T = 256;   // theta values per launch (samples x components): 2 KB of kernel arguments
typedef double lc_dvec2 __attribute__((ext_vector_type(2)));
struct LincombArgs {
  const double* v[HDD_MAX_COMP];
  double theta[LC_T];         // [n_s][n_comp]
  double* out;
  int64_t nnz, stride;
  int32_t n_comp, n_s;
};

__global__ void __launch_bounds__(256) lincomb_kernel(const LincombArgs a)
{
  __shared__ double th[LC_T];
  for (int i = threadIdx.x; i < a.n_s * a.n_comp; i += 256) th[i] = a.theta[i];
  __syncthreads();
  const int64_t n2 = a.nnz >> 1;
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n2; k += int64_t(gridDim.x) * blockDim.x) {
    double2 v[HDD_MAX_COMP];
#pragma unroll
    for (int c = 0; c < HDD_MAX_COMP; ++c)
      v[c] = c < a.n_comp ? reinterpret_cast<const double2*>(a.v[c])[k] : make_double2(0.0, 0.0);
    for (int s = 0; s < a.n_s; ++s) {
      lc_dvec2 r = {0.0, 0.0};
      const double* ts = th + s * a.n_comp;
#pragma unroll
      for (int c = 0; c < HDD_MAX_COMP; ++c) {
        if (c < a.n_comp) {
          r.x += ts[c] * v[c].x;
          r.y += ts[c] * v[c].y;
        }
      }
      __builtin_nontemporal_store(r, reinterpret_cast<lc_dvec2*>(a.out + s * a.stride) + k);
    }
  }
  if ((a.nnz & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t k = a.nnz - 1;
    for (int s = 0; s < a.n_s; ++s) {
      double r = 0.0;
      for (int c = 0; c < a.n_comp; ++c) r += th[s * a.n_comp + c] * a.v[c][k];
      a.out[s * a.stride + k] = r;
    }
  }
}
}  // namespace

extern "C" int hdd_affine_lincomb(hdd_ctx* ctx, int64_t nnz, const double* const* d_vals, int32_t n_comp,
                                  const double* theta, int32_t n_samples, double* d_out, int64_t out_stride,
                                  void* stream)
{
  if (!ctx || !d_vals || !theta || !d_out) return set_error(HDD_ERR_INVALID, "hdd_affine_lincomb: null argument");
  if (n_comp < 1 || n_comp > HDD_MAX_COMP || n_samples < 0 || nnz < 0 || out_stride < nnz)
    return set_error(HDD_ERR_INVALID, "hdd_affine_lincomb: invalid sizes");
  bool aligned = true;
  for (int c = 0; c < n_comp; ++c) aligned &= d_vals[c] && (reinterpret_cast<uintptr_t>(d_vals[c]) % 16 == 0);
  aligned &= reinterpret_cast<uintptr_t>(d_out) % 16 == 0 && (out_stride % 2 == 0);
  if (!aligned) return set_error(HDD_ERR_INVALID, "hdd_affine_lincomb: arrays must be 16-byte aligned, stride even");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_affine_lincomb: hipSetDevice");
  const int64_t n2 = (nnz + 1) / 2;
  const unsigned grid = unsigned(std::min<int64_t>(std::max<int64_t>((n2 + 255) / 256, 1), 256 * 32));
  const int per_launch = LC_T / n_comp;
  for (int s0 = 0; s0 < n_samples; s0 += per_launch) {
    LincombArgs a{};
    for (int c = 0; c < n_comp; ++c) a.v[c] = d_vals[c];
    a.n_comp = n_comp;
    a.n_s = std::min(per_launch, n_samples - s0);
    for (int s = 0; s < a.n_s; ++s)
      for (int c = 0; c < n_comp; ++c) a.theta[s * n_comp + c] = theta[(s0 + s) * n_comp + c];
    a.out = d_out + int64_t(s0) * out_stride;
    a.nnz = nnz;
    a.stride = out_stride;
    hipLaunchKernelGGL(lincomb_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), a);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "hdd_affine_lincomb: launch");
  }
  return HDD_OK;
}

// ------------------------------------------------------------------------------------------------
// SoA gather / scatter of element columns (halo records)
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int SOA_MAX = 16;
struct SoaArgs {
  const double* src[SOA_MAX];
  double* dst[SOA_MAX];
  int32_t rows[SOA_MAX];
  int32_t row_first[SOA_MAX + 1];
  int32_t n_arrays;
  int64_t ld, n, offset;
  const int32_t* idx;
  const double* buf_in;
  double* buf_out;
};

__global__ void __launch_bounds__(256) soa_gather_kernel(const SoaArgs a)
{
  const int64_t total = int64_t(a.row_first[a.n_arrays]) * a.n;
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = t / a.n, i = t - r * a.n;
    int arr = 0;
    while (arr + 1 < a.n_arrays && a.row_first[arr + 1] <= r) ++arr;
    const int64_t rr = r - a.row_first[arr];
    a.buf_out[t] = a.src[arr][rr * a.ld + a.idx[i]];
  }
}

__global__ void __launch_bounds__(256) soa_scatter_kernel(const SoaArgs a)
{
  const int64_t total = int64_t(a.row_first[a.n_arrays]) * a.n;
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = t / a.n, i = t - r * a.n;
    int arr = 0;
    while (arr + 1 < a.n_arrays && a.row_first[arr + 1] <= r) ++arr;
    const int64_t rr = r - a.row_first[arr];
    a.dst[arr][rr * a.ld + a.offset + i] = a.buf_in[t];
  }
}

int soa_args(SoaArgs& a, const int32_t* rows, int32_t n_arrays, int64_t ld, int64_t n)
{
  if (n_arrays < 1 || n_arrays > SOA_MAX || !rows || ld < 0 || n < 0)
    return set_error(HDD_ERR_INVALID, "hdd_soa_*: invalid sizes (1 <= n_arrays <= 16)");
  a.n_arrays = n_arrays;
  a.row_first[0] = 0;
  for (int k = 0; k < n_arrays; ++k) {
    if (rows[k] < 1) return set_error(HDD_ERR_INVALID, "hdd_soa_*: rows must be >= 1");
    a.rows[k] = rows[k];
    a.row_first[k + 1] = a.row_first[k] + rows[k];
  }
  a.ld = ld;
  a.n = n;
  return HDD_OK;
}
}  // namespace

extern "C" int hdd_soa_gather(hdd_ctx* ctx, const double* const* arrays, const int32_t* rows, int32_t n_arrays,
                              int64_t ld, const int32_t* d_idx, int64_t n, double* d_buf, void* stream)
{
  if (!ctx || !arrays || !d_idx || !d_buf) return set_error(HDD_ERR_INVALID, "hdd_soa_gather: null argument");
  SoaArgs a{};
  int rc = soa_args(a, rows, n_arrays, ld, n);
  if (rc) return rc;
  for (int k = 0; k < n_arrays; ++k) a.src[k] = arrays[k];
  a.idx = d_idx;
  a.buf_out = d_buf;
  if (n == 0) return HDD_OK;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_soa_gather: hipSetDevice");
  const int64_t total = int64_t(a.row_first[n_arrays]) * n;
  const unsigned grid = unsigned(std::min<int64_t>((total + 255) / 256, 4096));
  hipLaunchKernelGGL(soa_gather_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  e = hipGetLastError();
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_soa_gather: launch");
}

extern "C" int hdd_soa_scatter(hdd_ctx* ctx, double* const* arrays, const int32_t* rows, int32_t n_arrays, int64_t ld,
                               int64_t dst_offset, int64_t n, const double* d_buf, void* stream)
{
  if (!ctx || !arrays || !d_buf) return set_error(HDD_ERR_INVALID, "hdd_soa_scatter: null argument");
  SoaArgs a{};
  int rc = soa_args(a, rows, n_arrays, ld, n);
  if (rc) return rc;
  for (int k = 0; k < n_arrays; ++k) a.dst[k] = arrays[k];
  a.offset = dst_offset;
  a.buf_in = d_buf;
  if (n == 0) return HDD_OK;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_soa_scatter: hipSetDevice");
  const int64_t total = int64_t(a.row_first[n_arrays]) * n;
  const unsigned grid = unsigned(std::min<int64_t>((total + 255) / 256, 4096));
  hipLaunchKernelGGL(soa_scatter_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  e = hipGetLastError();
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_soa_scatter: launch");
}

// ------------------------------------------------------------------------------------------------
// value gather (block operator extraction)
// ------------------------------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(256) gather_values_kernel(const double* v, const int64_t* src, int64_t n, double* out)
{
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n; k += int64_t(gridDim.x) * blockDim.x)
    __builtin_nontemporal_store(v[src[k]], out + k);
}
}  // namespace

extern "C" int hdd_gather_values(hdd_ctx* ctx, const double* d_vals, const int64_t* d_src, int64_t n, double* d_out,
                                 void* stream)
{
  if (!ctx || !d_vals || !d_src || !d_out || n < 0) return set_error(HDD_ERR_INVALID, "hdd_gather_values: invalid argument");
  if (n == 0) return HDD_OK;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_gather_values: hipSetDevice");
  const unsigned grid = unsigned(std::min<int64_t>((n + 255) / 256, 256 * 16));
  hipLaunchKernelGGL(gather_values_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), d_vals, d_src, n,
                     d_out);
  e = hipGetLastError();
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_gather_values: launch");
}

// ------------------------------------------------------------------------------------------------
// device pattern build (EllipticSWIPDG::pattern, swipdg.hh:169)
// ------------------------------------------------------------------------------------------------
static int mesh_faces(const hdd_mesh* m)
{
  return m->elem_type == HDD_SIMPLEX ? 3 : (m->elem_type == HDD_CUBE ? 4 : (m->elem_type == HDD_HEX ? 6 : 0));
}

extern "C" int hdd_pattern_elem_ptr_device(hdd_ctx* ctx, const hdd_mesh* m, int32_t nb, int64_t* d_elem_ptr,
                                           int64_t* nnz, void* stream)
{
  if (!ctx || !m || !d_elem_ptr || !nnz || nb < 1 || !m->neighbors)
    return set_error(HDD_ERR_INVALID, "hdd_pattern_elem_ptr_device: invalid argument");
  const int nf = mesh_faces(m);
  if (!nf) return set_error(HDD_ERR_UNSUPPORTED, "hdd_pattern_elem_ptr_device: unknown element type");
  if (m->own_begin < 0 || m->own_end > m->n_local || m->own_begin > m->own_end)
    return set_error(HDD_ERR_RANGE, "hdd_pattern_elem_ptr_device: 0 <= own_begin <= own_end <= n_local violated");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_pattern_elem_ptr_device: hipSetDevice");
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n_own = m->own_end - m->own_begin;
  const size_t tmp_bytes = size_t(hdd::dev::pattern_elem_ptr_scratch(n_own) + 1) * sizeof(int64_t);
  if (tmp_bytes > ctx->scan_ws_bytes) {   // the context keeps the scratch (one stream at a time per context)
    (void)hipStreamSynchronize(s);
    if (ctx->scan_ws) (void)hipFree(ctx->scan_ws);
    ctx->scan_ws = nullptr;
    ctx->scan_ws_bytes = 0;
    e = hipMalloc(&ctx->scan_ws, tmp_bytes);
    if (e != hipSuccess) return hip_fail(e, "hdd_pattern_elem_ptr_device: scan scratch");
    ctx->scan_ws_bytes = tmp_bytes;
  }
  // nnz reaches the host through a mapped pinned word the elem_ptr kernel writes (no copy launch);
  // HDD_VARIANT_PATTERN_SCAN_COPY: the round-3 scheme (scan launch + device-to-host copy), cross-check
  const bool legacy = (ctx->variant & HDD_VARIANT_PATTERN_SCAN_COPY) != 0;
  if (!legacy && !ctx->nnz_h && n_own > 0) {
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&ctx->nnz_h), sizeof(int64_t), hipHostMallocMapped)) != hipSuccess)
      return hip_fail(e, "hdd_pattern_elem_ptr_device: pinned nnz");
    if ((e = hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->nnz_hd), ctx->nnz_h, 0)) != hipSuccess) {
      (void)hipHostFree(ctx->nnz_h);
      ctx->nnz_h = nullptr;
      return hip_fail(e, "hdd_pattern_elem_ptr_device: pinned nnz device address");
    }
  }
  const bool mapped = !legacy && n_own > 0;
  e = hdd::dev::launch_pattern_elem_ptr(m->neighbors, nf, m->n_local, m->own_begin, m->own_end, int64_t(nb) * nb,
                                        d_elem_ptr, static_cast<int64_t*>(ctx->scan_ws), s,
                                        mapped ? ctx->nnz_hd : nullptr, legacy);
  if (e != hipSuccess) return hip_fail(e, "hdd_pattern_elem_ptr_device: elem_ptr");
  if (!mapped) e = hipMemcpyAsync(nnz, d_elem_ptr + n_own, sizeof(int64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "hdd_pattern_elem_ptr_device: read nnz");
  if (mapped) *nnz = *static_cast<volatile int64_t*>(ctx->nnz_h);
  return HDD_OK;
}

extern "C" int hdd_pattern_fill_device(hdd_ctx* ctx, const hdd_mesh* m, int32_t nb, const int64_t* d_global_id,
                                       const int64_t* d_elem_ptr, int64_t* d_row_ptr, int32_t* d_col, void* stream)
{
  if (!ctx || !m || !d_elem_ptr || !d_row_ptr || !d_col || nb < 1 || !m->neighbors)
    return set_error(HDD_ERR_INVALID, "hdd_pattern_fill_device: invalid argument");
  const int nf = mesh_faces(m);
  if (!nf) return set_error(HDD_ERR_UNSUPPORTED, "hdd_pattern_fill_device: unknown element type");
  if (m->own_begin < 0 || m->own_end > m->n_local || m->own_begin > m->own_end)
    return set_error(HDD_ERR_RANGE, "hdd_pattern_fill_device: 0 <= own_begin <= own_end <= n_local violated");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_pattern_fill_device: hipSetDevice");
  e = hdd::dev::launch_pattern_fill(m->neighbors, nf, nb, m->n_local, m->own_begin, m->own_end, d_global_id,
                                    d_elem_ptr, d_row_ptr, d_col, ctx->n_cu, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_pattern_fill_device: launch");
}

// ------------------------------------------------------------------------------------------------
// right-hand side (rhs.hip): host-side quadrature rules
// ------------------------------------------------------------------------------------------------
namespace {
// simplex rules on the reference triangle (area 1/2): centroid (order <= 1), 3-point interior (2),
// Dunavant 6-point (3..4), collapsed Gauss-Legendre (Duffy) beyond
int simplex_rule(int order, double (*q)[4], int cap)
{
  if (order <= 1) {
    q[0][0] = q[0][1] = 1.0 / 3.0; q[0][2] = 0.0; q[0][3] = 0.5;
    return 1;
  }
  if (order == 2) {
    const double a = 1.0 / 6.0, b = 2.0 / 3.0;
    const double P[3][2] = {{a, a}, {b, a}, {a, b}};
    for (int k = 0; k < 3; ++k) { q[k][0] = P[k][0]; q[k][1] = P[k][1]; q[k][2] = 0.0; q[k][3] = 1.0 / 6.0; }
    return 3;
  }
  if (order <= 4) {
    const double a = 0.44594849091596488632, wa = 0.22338158967801146570;
    const double b = 0.091576213509770743460, wb = 0.10995174365532186764;
    const double P[6][3] = {{a, a, wa}, {1 - 2 * a, a, wa}, {a, 1 - 2 * a, wa},
                            {b, b, wb}, {1 - 2 * b, b, wb}, {b, 1 - 2 * b, wb}};
    for (int k = 0; k < 6; ++k) { q[k][0] = P[k][0]; q[k][1] = P[k][1]; q[k][2] = 0.0; q[k][3] = 0.5 * P[k][2]; }
    return 6;
  }
  const int n = (order + 3) / 2;
  if (n * n > cap) return -1;
  double s[16], w[16];
  gauss_legendre01(n, s, w);
  int k = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j, ++k) {
      q[k][0] = s[i]; q[k][1] = s[j] * (1.0 - s[i]); q[k][2] = 0.0; q[k][3] = w[i] * w[j] * (1.0 - s[i]);
    }
  return n * n;
}

int tensor_rule(int dim, int order, double (*q)[4], int cap)
{
  const int n = std::max(1, (order + 2) / 2);
  int tot = 1;
  for (int a = 0; a < dim; ++a) tot *= n;
  if (tot > cap || n > 16) return -1;
  double s[16], w[16];
  gauss_legendre01(n, s, w);
  for (int m = 0; m < tot; ++m) {
    int r = m;
    q[m][0] = q[m][1] = q[m][2] = 0.0;
    q[m][3] = 1.0;
    for (int a = 0; a < dim; ++a) {
      q[m][a] = s[r % n];
      q[m][3] *= w[r % n];
      r /= n;
    }
  }
  return tot;
}

int face_rule(int fdim, int order, double (*q)[3], int cap)
{
  double t[64][4];
  const int nq = tensor_rule(fdim, order, t, std::min(cap, 64));
  for (int k = 0; k < nq; ++k) { q[k][0] = t[k][0]; q[k][1] = t[k][1]; q[k][2] = t[k][3]; }
  return nq;
}

hdd::dev::KappaArg kap_arg(const hdd_scalar_fn* f)
{
  if (!f) return hdd::dev::KappaArg{HDD_FN_CONST, 0, 0.0, 0.0, 0.0, 0.0, nullptr, nullptr, 0, 0};
  return hdd::dev::KappaArg{f->kind, f->order, f->c, f->b, f->kx, f->ky, f->per_elem, f->table, f->n_table, 0};
}
}  // namespace

extern "C" int hdd_swipdg_rhs(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* force, const hdd_scalar_fn* kappa,
                              const hdd_tensor_fn* tensor, const hdd_scalar_fn* dirichlet,
                              const hdd_scalar_fn* neumann, const hdd_swipdg_params* p, double* d_rhs, void* stream)
{
  using namespace hdd::dev;
  if (!ctx || !m || !p || !d_rhs) return set_error(HDD_ERR_INVALID, "hdd_swipdg_rhs: null argument");
  if (m->elem_type != HDD_SIMPLEX && m->elem_type != HDD_CUBE && m->elem_type != HDD_HEX)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_rhs: unknown element type");
  if (!m->coords || !m->neighbors) return set_error(HDD_ERR_INVALID, "hdd_swipdg_rhs: mesh arrays missing");
  if (m->own_begin < 0 || m->own_end > m->n_local || m->own_begin > m->own_end)
    return set_error(HDD_ERR_RANGE, "hdd_swipdg_rhs: 0 <= own_begin <= own_end <= n_local violated");
  if (dirichlet && (!kappa || !tensor))
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_rhs: the Dirichlet functional needs kappa and the tensor");
  for (const hdd_scalar_fn* f : {force, kappa, dirichlet, neumann}) {
    if (f && f->kind == HDD_FN_PER_ELEM && !f->per_elem)
      return set_error(HDD_ERR_INVALID, "hdd_swipdg_rhs: per_elem function without values");
    if (f && f->kind == HDD_FN_FLATTOP && (m->elem_type == HDD_HEX || f->n_table < 0 || (f->n_table > 0 && !f->table)))
      return set_error(f->n_table < 0 || !f->table ? HDD_ERR_INVALID : HDD_ERR_UNSUPPORTED,
                       "hdd_swipdg_rhs: FLATTOP needs a box table and a 2d mesh");
  }
  if (tensor && tensor->kind != HDD_TENSOR_CONST && !tensor->per_elem)
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_rhs: tensor per_elem missing");
  const int deg = m->elem_type == HDD_HEX ? std::max(1, int(m->degree)) : 1;
  if (m->elem_type != HDD_HEX && m->degree > 1)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_rhs: 2d meshes carry P1 / Q1 only");
  if (deg > 3) return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_rhs: HDD_HEX supports p = 1..3");
  const int dim = m->elem_type == HDD_HEX ? 3 : 2;
  RhsArgs a{};
  a.elem_type = m->elem_type;
  a.degree = deg;
  a.nb = m->elem_type == HDD_SIMPLEX ? 3 : (m->elem_type == HDD_CUBE ? 4 : (deg + 1) * (deg + 1) * (deg + 1));
  a.n_local = m->n_local;
  a.own_begin = m->own_begin;
  a.own_end = m->own_end;
  a.coords = m->coords;
  if (!m->elem_vertices != !m->vertex_coords)
    return set_error(HDD_ERR_INVALID, "hdd_swipdg_rhs: mesh elem_vertices / vertex_coords: both or neither");
  if (m->elem_vertices && m->elem_type != HDD_HEX && !(ctx->variant & HDD_VARIANT_ELEMENT_MAJOR)) {
    a.ev = m->elem_vertices;   // vertex-indexed geometry
    a.vxy = m->vertex_coords;
  }
  a.nbrs = m->neighbors;
  a.tkind = tensor ? tensor->kind : HDD_TENSOR_CONST;
  for (int r = 0; r < 6; ++r) a.tc[r] = tensor ? tensor->c[r] : 0.0;
  a.tper = tensor ? tensor->per_elem : nullptr;
  a.force = kap_arg(force);
  a.kappa = kap_arg(kappa);
  a.dirichlet = kap_arg(dirichlet);
  a.neumann = kap_arg(neumann);
  a.has_force = force != nullptr;
  a.has_dirichlet = dirichlet != nullptr;
  a.has_neumann = neumann != nullptr;
  a.sigma_boundary = p->sigma_boundary;
  a.beta = p->beta;
  a.out = d_rhs;
  a.n_cu = ctx->n_cu;
  a.generic = (ctx->variant & HDD_VARIANT_RHS_GENERIC) ? 1 : 0;
  a.no_tiny = (ctx->variant & HDD_VARIANT_RHS_NO_TINY) ? 1 : 0;
  if (force) {
    const int order = fn_order(*force) + deg;
    a.nqv = m->elem_type == HDD_SIMPLEX ? simplex_rule(order, a.qv, 64) : tensor_rule(dim, order, a.qv, 64);
    if (a.nqv < 0) return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_rhs: force integration order too high");
  }
  if (dirichlet) {
    const int order = std::max(fn_order(*dirichlet) + deg, fn_order(*kappa) + 0 + (deg - 1) + fn_order(*dirichlet));
    a.nqd = face_rule(dim - 1, order, a.qd, 16);
    if (a.nqd < 0) return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_rhs: Dirichlet integration order too high");
  }
  if (neumann) {
    a.nqn = face_rule(dim - 1, fn_order(*neumann) + deg, a.qn, 16);
    if (a.nqn < 0) return set_error(HDD_ERR_UNSUPPORTED, "hdd_swipdg_rhs: Neumann integration order too high");
  }
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_swipdg_rhs: hipSetDevice");
  const int64_t n_own = m->own_end - m->own_begin;
  // split path (HDD_VARIANT_RHS_FUSED: the fused kernel, cross-check): the list is kept in the context, allocated
  // (and its counters zeroed) on the first call of a size class -- warm up before hipGraph capture
  if (m->elem_type != HDD_HEX && (dirichlet || neumann) && n_own > 0 && n_own < (int64_t(1) << 31) &&
      !(ctx->variant & HDD_VARIANT_RHS_FUSED)) {
    const size_t bytes = hdd::dev::rhs_list_bytes(n_own);
    if (bytes > ctx->rhs_ws_bytes) {
      if (ctx->rhs_ws) {
        if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "hdd_swipdg_rhs: list sync");
        (void)hipFree(ctx->rhs_ws);
      }
      ctx->rhs_ws = nullptr;
      ctx->rhs_ws_bytes = 0;
      if ((e = hipMalloc(&ctx->rhs_ws, bytes + bytes / 4)) != hipSuccess) return hip_fail(e, "hdd_swipdg_rhs: list");
      if ((e = hipMemset(ctx->rhs_ws, 0, hdd::dev::RHS_LIST_OFS * sizeof(uint32_t))) != hipSuccess)
        return hip_fail(e, "hdd_swipdg_rhs: list counters");
      ctx->rhs_ws_bytes = bytes + bytes / 4;
    }
    a.bnd_list = static_cast<uint32_t*>(ctx->rhs_ws);
  }
  a.skip_face = (ctx->debug_flags & 524288) ? 1 : 0;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  // The boundary-element list is context state: calls on different streams are ordered behind each other (the
  // previous call's face kernel has re-armed the counters before this call's volume kernel appends).  Not under
  // hipGraph capture, where the captured stream alone orders the replays.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool ordered = a.bnd_list && hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone;
  if (ordered) {
    if (!ctx->rhs_evt && (e = hipEventCreateWithFlags(&ctx->rhs_evt, hipEventDisableTiming)) != hipSuccess)
      return hip_fail(e, "hdd_swipdg_rhs: list event");
    if (ctx->rhs_used && ctx->rhs_stream != s && (e = hipStreamWaitEvent(s, ctx->rhs_evt, 0)) != hipSuccess)
      return hip_fail(e, "hdd_swipdg_rhs: order behind the previous call's stream");
  }
  e = launch_rhs(a, s);
  if (ordered) {
    const hipError_t er = hipEventRecord(ctx->rhs_evt, s);
    if (er != hipSuccess && e == hipSuccess) e = er;
    ctx->rhs_stream = s;
    ctx->rhs_used = true;
  }
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_swipdg_rhs: launch");
}

extern "C" int hdd_product_assemble(hdd_ctx* ctx, const hdd_mesh* m, int32_t product, const hdd_scalar_fn* kappa,
                                    const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                                    double* d_vals, void* stream)
{
  using namespace hdd::dev;
  if (!ctx || !m || !p || !pattern || !d_vals || !pattern->elem_ptr)
    return set_error(HDD_ERR_INVALID, "hdd_product_assemble: null argument");
  if (product < HDD_PRODUCT_L2 || product > HDD_PRODUCT_PENALTY)
    return set_error(HDD_ERR_INVALID, "hdd_product_assemble: unknown product");
  if (m->elem_type != HDD_SIMPLEX && m->elem_type != HDD_CUBE && m->elem_type != HDD_HEX)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_product_assemble: unknown element type");
  if (m->own_begin < 0 || m->own_end > m->n_local || m->own_begin > m->own_end)
    return set_error(HDD_ERR_RANGE, "hdd_product_assemble: 0 <= own_begin <= own_end <= n_local violated");
  const bool needs_coeff = product == HDD_PRODUCT_ELLIPTIC || product == HDD_PRODUCT_PENALTY;
  if (needs_coeff && (!kappa || !tensor))
    return set_error(HDD_ERR_INVALID, "hdd_product_assemble: elliptic / penalty products need kappa and the tensor");
  if (needs_coeff && kappa->kind == HDD_FN_PER_ELEM && !kappa->per_elem)
    return set_error(HDD_ERR_INVALID, "hdd_product_assemble: kappa per_elem missing");
  if (needs_coeff && kappa->kind == HDD_FN_FLATTOP &&
      (m->elem_type == HDD_HEX || kappa->n_table < 0 || (kappa->n_table > 0 && !kappa->table)))
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_product_assemble: FLATTOP needs a box table and a 2d mesh");
  if (needs_coeff && tensor->kind != HDD_TENSOR_CONST && !tensor->per_elem)
    return set_error(HDD_ERR_INVALID, "hdd_product_assemble: tensor per_elem missing");
  const int deg = m->elem_type == HDD_HEX ? std::max(1, int(m->degree)) : 1;
  if (m->elem_type != HDD_HEX && m->degree > 1)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_product_assemble: 2d meshes carry P1 / Q1 only");
  if (deg > 3) return set_error(HDD_ERR_UNSUPPORTED, "hdd_product_assemble: HDD_HEX supports p = 1..3");
  const int nb = m->elem_type == HDD_SIMPLEX ? 3 : (m->elem_type == HDD_CUBE ? 4 : (deg + 1) * (deg + 1) * (deg + 1));
  if (pattern->n_rows != int64_t(nb) * (m->own_end - m->own_begin))
    return set_error(HDD_ERR_INVALID, "hdd_product_assemble: pattern rows != nb * owned elements");
  ProductArgs a{};
  a.elem_type = m->elem_type;
  a.degree = deg;
  a.nb = nb;
  a.kind = product;
  a.n_local = m->n_local;
  a.own_begin = m->own_begin;
  a.own_end = m->own_end;
  a.coords = m->coords;
  a.nbrs = m->neighbors;
  a.elem_ptr = pattern->elem_ptr;
  a.tkind = tensor ? tensor->kind : HDD_TENSOR_CONST;
  for (int r = 0; r < 6; ++r) a.tc[r] = tensor ? tensor->c[r] : 0.0;
  a.tper = tensor ? tensor->per_elem : nullptr;
  a.kappa = kap_arg(kappa);
  a.sigma_inner = p->sigma_inner;
  a.sigma_boundary = p->sigma_boundary;
  a.beta = p->beta;
  a.vals = d_vals;
  // integrand orders + over_integrate (= 2): test + ansatz order [+ kappa + A]; gradients count p - 1
  const int over = 2, ko = kappa ? fn_order(*kappa) : 0;
  if (product <= HDD_PRODUCT_ELLIPTIC) {
    int order = product == HDD_PRODUCT_L2 ? 2 * deg + over : 2 * (deg - 1) + over;
    if (product == HDD_PRODUCT_ELLIPTIC) order += ko;
    if (m->elem_type == HDD_SIMPLEX) {
      a.nqv = simplex_rule(order, a.qv, 64);
      if (a.nqv < 0) return set_error(HDD_ERR_UNSUPPORTED, "hdd_product_assemble: integration order too high");
    } else {
      const int n1 = std::max(1, (order + 2) / 2);
      if (n1 > 16) return set_error(HDD_ERR_UNSUPPORTED, "hdd_product_assemble: integration order too high");
      double s[16], w[16];
      gauss_legendre01(n1, s, w);
      for (int q = 0; q < n1; ++q) { a.qv[q][0] = s[q]; a.qv[q][3] = w[q]; }
      a.nqv = n1;
    }
  } else {
    const int order = product == HDD_PRODUCT_BOUNDARY_L2 ? 2 * deg + over : ko + 2 * deg + over;
    const int n1 = std::max(1, (order + 2) / 2);
    if (n1 > 16) return set_error(HDD_ERR_UNSUPPORTED, "hdd_product_assemble: integration order too high");
    double s[16], w[16];
    gauss_legendre01(n1, s, w);
    for (int q = 0; q < n1; ++q) { a.qf[q][0] = s[q]; a.qf[q][1] = w[q]; }
    a.nq1f = n1;
  }
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_product_assemble: hipSetDevice");
  if (m->elem_type != HDD_HEX && m->face_info) {
    // P1 / Q1 with piecewise-constant data: closed forms on the persistent tile driver
    AssembleArgs f{};
    f.elem_type = m->elem_type;
    f.n_comp = 1;
    f.n_local = m->n_local;
    f.own_begin = m->own_begin;
    f.own_end = m->own_end;
    f.coords = m->coords;
    f.nbrs = m->neighbors;
    f.finfo = m->face_info;
    f.elem_ptr = pattern->elem_ptr;
    f.tkind = a.tkind;
    f.tc0 = a.tc[0];
    f.tc1 = a.tc[1];
    f.tc2 = a.tc[2];
    f.tper = a.tper;
    f.sigma_inner = p->sigma_inner;
    f.sigma_boundary = p->sigma_boundary;
    f.beta = p->beta;
    f.kappa[0] = a.kappa;
    f.vals[0] = d_vals;
    f.n_cu = ctx->n_cu;
    f.debug_flags = ctx->debug_flags;
    f.variant = ctx->variant;
    f.wgcu = ctx->wgcu;
    if (!m->elem_vertices != !m->vertex_coords)
      return set_error(HDD_ERR_INVALID, "hdd_product_assemble: mesh elem_vertices / vertex_coords: both or neither");
    if (m->elem_vertices && m->elem_type == HDD_SIMPLEX && !(ctx->variant & HDD_VARIANT_ELEMENT_MAJOR) &&
        vx_offsets_fit(m->n_local)) {
      f.ev = m->elem_vertices;   // vertex-indexed geometry, as hdd_swipdg_assemble
      f.vxy = m->vertex_coords;
    }
    bool fast = false;
    e = launch_product_fast(f, product, static_cast<hipStream_t>(stream), &fast);
    if (fast) return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_product_assemble: launch");
  }
  e = launch_product(a, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_product_assemble: launch");
}

// ------------------------------------------------------------------------------------------------
// block operators on the device (BlockSWIPDG::get_local_operator / get_coupling_operator,
// block-swipdg.hh:625-676, 1328-1379): rows [r0, r1) of a sorted CSR pattern restricted to the columns
// [c0, c1).  In the subdomain-major numbering the columns of one subdomain are ONE contiguous sub-range of
// every sorted row, found by two binary searches: count -> scan -> fill, thread per row (rows hold <= 5 (2d)
// or 7 (3d) blocks).  The values need no index map: a second pass copies each row's sub-range.
// ------------------------------------------------------------------------------------------------
namespace {
__device__ __forceinline__ int64_t lower_bound_col(const int32_t* col, int64_t lo, int64_t hi, int64_t v)
{
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (int64_t(col[m]) < v) lo = m + 1;
    else hi = m;
  }
  return lo;
}

__global__ void __launch_bounds__(256) subcsr_count_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                           int64_t r0, int64_t n, int64_t c0, int64_t c1,
                                                           int64_t* __restrict__ out_rp)
{
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t a = rp[r0 + i], b = rp[r0 + i + 1];
    const int64_t lo = lower_bound_col(col, a, b, c0);
    out_rp[i + 1] = lower_bound_col(col, lo, b, c1) - lo;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out_rp[0] = 0;
}

__global__ void __launch_bounds__(256) subcsr_fill_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                          int64_t r0, int64_t n, int64_t c0,
                                                          const int64_t* __restrict__ out_rp, int32_t* __restrict__ out_col,
                                                          int64_t* __restrict__ out_src)
{
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t lo = lower_bound_col(col, rp[r0 + i], rp[r0 + i + 1], c0);
    const int64_t k0 = out_rp[i], len = out_rp[i + 1] - k0;
    for (int64_t j = 0; j < len; ++j) {
      out_col[k0 + j] = int32_t(int64_t(col[lo + j]) - c0);
      if (out_src) out_src[k0 + j] = lo + j;
    }
  }
}

struct ValPtrs {
  const double* in[HDD_MAX_COMP];
  double* out[HDD_MAX_COMP];
};

__global__ void __launch_bounds__(256) subcsr_values_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                            int64_t r0, int64_t n, int64_t c0,
                                                            const int64_t* __restrict__ out_rp, ValPtrs v, int nc)
{
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t lo = lower_bound_col(col, rp[r0 + i], rp[r0 + i + 1], c0);
    const int64_t k0 = out_rp[i], len = out_rp[i + 1] - k0;
    for (int c = 0; c < nc; ++c)
      for (int64_t j = 0; j < len; ++j) v.out[c][k0 + j] = v.in[c][lo + j];
  }
}

int subcsr_check(const hdd_csr* p, int64_t r0, int64_t r1, int64_t c0, int64_t c1, const char* who)
{
  if (!p || !p->row_ptr || !p->col) return set_error(HDD_ERR_INVALID, std::string(who) + ": pattern arrays missing");
  if (r0 < 0 || r1 < r0 || r1 > p->n_rows || c0 < 0 || c1 < c0)
    return set_error(HDD_ERR_RANGE, std::string(who) + ": 0 <= row_begin <= row_end <= n_rows, col_begin <= col_end violated");
  if (c1 - c0 > int64_t(INT32_MAX)) return set_error(HDD_ERR_RANGE, std::string(who) + ": column range exceeds int32");
  return HDD_OK;
}

unsigned rows_grid(int64_t n, int n_cu) { return unsigned(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, int64_t(n_cu) * 16))); }

// ---- batched: n_ops sub-blocks of one pattern in four launches.  The concatenated row-pointer array holds
// a leading slot per operator (count 0) before its row counts, so ONE inclusive scan over all operators leaves
// at operator k's leading slot the number of entries of the operators before it (base) and at its slot j the
// global start of its row j.  Operator k's entries start at noff = the prefix of the EVEN-rounded counts
// (16-byte aligned value arrays: hdd_affine_lincomb takes every operator as it is).
struct OpDesc {
  int64_t r0, c0, c1;   // rows [r0, r0 + rows), columns [c0, c1) of the pattern
  int64_t roff, rows;   // slots [roff, roff + rows + 1) of the concatenated row-pointer array
  int64_t base;         // entries of the operators before k (the scan's value at the leading slot)
  int64_t noff;         // where operator k's entries start in the concatenated outputs (even)
};

__device__ __forceinline__ int op_of_slot(const OpDesc* d, int n_ops, int64_t x)
{
  int lo = 0, hi = n_ops - 1;   // last k with roff_k <= x
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (d[m].roff <= x) lo = m;
    else hi = m - 1;
  }
  return lo;
}

// the sub-range [lo, lo + len) of sorted row [a, b) with columns in [c0, c1): most rows of a coupling operator
// lie wholly outside (first / last column decide, two independent loads), only the rest binary-search
__device__ __forceinline__ void row_range(const int32_t* __restrict__ col, int64_t a, int64_t b, int64_t c0,
                                          int64_t c1, int64_t& lo, int64_t& len)
{
  lo = a;
  len = 0;
  if (a == b) return;
  const int64_t first = col[a], last = col[b - 1];
  if (last < c0 || first >= c1) return;
  if (first >= c0 && last < c1) {
    len = b - a;
    return;
  }
  lo = lower_bound_col(col, a, b, c0);
  len = lower_bound_col(col, lo, b, c1) - lo;
}

__global__ void __launch_bounds__(256) ops_count_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                        const OpDesc* __restrict__ d, int n_ops, int64_t n_slots,
                                                        int64_t* __restrict__ out)
{
  for (int64_t x = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; x < n_slots; x += int64_t(gridDim.x) * blockDim.x) {
    const OpDesc o = d[op_of_slot(d, n_ops, x)];
    const int64_t j = x - o.roff;
    int64_t lo = 0, c = 0;
    if (j > 0) row_range(col, rp[o.r0 + j - 1], rp[o.r0 + j], o.c0, o.c1, lo, c);
    out[x] = c;
  }
}

// one wave: bases and even-rounded offsets of 64 operators per step (loads in parallel, a wave prefix sum)
__global__ void __launch_bounds__(64) ops_base_kernel(const int64_t* __restrict__ scanned, OpDesc* d, int n_ops,
                                                      int64_t* __restrict__ totals)
{
  const int lane = threadIdx.x;
  int64_t carry = 0;
  for (int k0 = 0; k0 < n_ops; k0 += 64) {
    const int k = k0 + lane;
    int64_t b = 0, n = 0;
    if (k < n_ops) {
      b = scanned[d[k].roff];
      n = scanned[d[k].roff + d[k].rows] - b;
    }
    int64_t incl = n + (n & 1);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t v = __shfl_up(incl, off, 64);
      if (lane >= off) incl += v;
    }
    const int64_t noff = carry + incl - (n + (n & 1));
    if (k < n_ops) {
      d[k].base = b;
      d[k].noff = noff;
      if (totals) totals[k] = noff;
    }
    carry += __shfl(incl, 63, 64);
  }
  if (totals && lane == 0) totals[n_ops] = carry;
}

// Wave-cooperative copy of the 64 row segments a wave holds (lane l: len[l] entries): the segments' entries
// are numbered through a wave prefix sum and every lane takes entries lane, lane + 64, ...; copy(seg, off)
// handles entry off of segment seg.  Consecutive lanes then write consecutive positions of the
// (operator-contiguous) destination and read runs of the source, instead of 64 lanes each walking its own row
// (64 cache lines per instruction).  Whole waves call it (the slot loops below are wave-uniform).
template <class F>
__device__ __forceinline__ void wave_segments(int len, int* s_end, F&& copy)
{
  const int lane = threadIdx.x & 63;
  int incl = len;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off, 64);
    if (lane >= off) incl += v;
  }
  s_end[lane] = incl;
  const int total = __shfl(incl, 63, 64);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int p = lane; p < total; p += 64) {
    int lo = 0, hi = 63;   // the first segment whose inclusive end exceeds p
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (s_end[m] > p) hi = m;
      else lo = m + 1;
    }
    copy(lo, p - (lo ? s_end[lo - 1] : 0));
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct SegShared {
  int64_t src[4][64], dst[4][64], c0[4][64];
  int end[4][64];
};

// columns (local) / sources at the operators' positions, then the row pointer made operator-relative in place
// (each slot reads only itself: its count is recomputed, the base comes from the descriptor)
__global__ void __launch_bounds__(256) ops_fill_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                       const OpDesc* __restrict__ d, int n_ops, int64_t n_slots,
                                                       int64_t* __restrict__ out_rp, int32_t* __restrict__ out_col,
                                                       int64_t* __restrict__ out_src)
{
  __shared__ SegShared sh;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t xb = int64_t(blockIdx.x) * blockDim.x; xb < n_slots; xb += int64_t(gridDim.x) * blockDim.x) {
    const int64_t x = xb + threadIdx.x;
    int64_t lo = 0, len = 0, dst = 0, c0 = 0;
    if (x < n_slots) {
      const OpDesc o = d[op_of_slot(d, n_ops, x)];
      const int64_t j = x - o.roff;
      const int64_t end = out_rp[x] - o.base;   // operator-relative end of row j - 1
      if (j > 0) row_range(col, rp[o.r0 + j - 1], rp[o.r0 + j], o.c0, o.c1, lo, len);
      dst = o.noff + end - len;
      c0 = o.c0;
      out_rp[x] = end;
    }
    if (out_col || out_src) {
      sh.src[w][lane] = lo;
      sh.dst[w][lane] = dst;
      sh.c0[w][lane] = c0;   // a wave's segments may belong to two operators
      wave_segments(int(len), sh.end[w], [&](int seg, int off) {
        const int64_t si = sh.src[w][seg] + off, di = sh.dst[w][seg] + off;
        if (out_col) out_col[di] = int32_t(int64_t(col[si]) - sh.c0[w][seg]);
        if (out_src) out_src[di] = si;
      });
    }
  }
}

// values: operator k's entries at noff_k + its (relative) row pointer, copied wave-cooperatively
__global__ void __launch_bounds__(256) ops_values_kernel(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                         const OpDesc* __restrict__ d, int n_ops, int64_t n_slots,
                                                         const int64_t* __restrict__ out_rp, ValPtrs v, int nc)
{
  __shared__ SegShared sh;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t xb = int64_t(blockIdx.x) * blockDim.x; xb < n_slots; xb += int64_t(gridDim.x) * blockDim.x) {
    const int64_t x = xb + threadIdx.x;
    int64_t lo = 0, len = 0, dst = 0;
    if (x < n_slots) {
      const OpDesc o = d[op_of_slot(d, n_ops, x)];
      const int64_t j = x - o.roff;
      if (j > 0) {
        const int64_t r0 = out_rp[x - 1];
        len = out_rp[x] - r0;
        dst = o.noff + r0;
        if (len) lo = lower_bound_col(col, rp[o.r0 + j - 1], rp[o.r0 + j], o.c0);
      }
    }
    sh.src[w][lane] = lo;
    sh.dst[w][lane] = dst;
    wave_segments(int(len), sh.end[w], [&](int seg, int off) {
      const int64_t si = sh.src[w][seg] + off, di = sh.dst[w][seg] + off;
      for (int c = 0; c < nc; ++c) v.out[c][di] = v.in[c][si];
    });
  }
}
}  // namespace

// descriptor table of a batched call -> ctx->ops_d (stream-ordered upload through the pinned staging copy,
// reused only after the previous upload completed); noff from the host array when given
static int ops_upload(hdd_ctx* ctx, const hdd_csr* p, int32_t n_ops, const hdd_block_range* ops,
                      const int64_t* nnz_off, hipStream_t s, int64_t* n_slots, const char* who)
{
  if (n_ops < 1 || !ops) return set_error(HDD_ERR_INVALID, std::string(who) + ": need n_ops >= 1 ranges");
  const size_t bytes = size_t(n_ops) * sizeof(OpDesc);
  hipError_t e = hipSuccess;
  if (!ctx->ops_evt && (e = hipEventCreateWithFlags(&ctx->ops_evt, hipEventDisableTiming)) != hipSuccess)
    return hip_fail(e, who);
  if ((e = hipEventSynchronize(ctx->ops_evt)) != hipSuccess) return hip_fail(e, who);
  if (bytes > ctx->ops_bytes) {
    if (ctx->ops_d) (void)hipFree(ctx->ops_d);
    if (ctx->ops_h) (void)hipHostFree(ctx->ops_h);
    ctx->ops_d = ctx->ops_h = nullptr;
    ctx->ops_bytes = 0;
    if ((e = hipMalloc(&ctx->ops_d, bytes)) != hipSuccess) return hip_fail(e, who);
    if ((e = hipHostMalloc(&ctx->ops_h, bytes, hipHostMallocDefault)) != hipSuccess) return hip_fail(e, who);
    ctx->ops_bytes = bytes;
  }
  auto* h = static_cast<OpDesc*>(ctx->ops_h);
  int64_t slots = 0;
  for (int32_t k = 0; k < n_ops; ++k) {
    const hdd_block_range& r = ops[k];
    if (int rc = subcsr_check(p, r.row_begin, r.row_end, r.col_begin, r.col_end, who)) return rc;
    if (nnz_off && (nnz_off[k] & 1))
      return set_error(HDD_ERR_INVALID, std::string(who) + ": nnz_off must be even (16-byte aligned operators)");
    h[k] = OpDesc{r.row_begin, r.col_begin, r.col_end, slots, r.row_end - r.row_begin, 0, nnz_off ? nnz_off[k] : 0};
    slots += r.row_end - r.row_begin + 1;
  }
  if (slots >= int64_t(INT32_MAX))
    return set_error(HDD_ERR_RANGE, std::string(who) + ": sum of (rows + 1) over the operators must fit int32");
  if ((e = hipMemcpyAsync(ctx->ops_d, ctx->ops_h, bytes, hipMemcpyHostToDevice, s)) != hipSuccess) return hip_fail(e, who);
  if ((e = hipEventRecord(ctx->ops_evt, s)) != hipSuccess) return hip_fail(e, who);
  *n_slots = slots;
  return HDD_OK;
}

extern "C" int hdd_block_operators_map_device(hdd_ctx* ctx, const hdd_csr* pattern, int32_t n_ops,
                                              const hdd_block_range* ops, int64_t* d_out_row_ptr, int32_t* d_out_col,
                                              int64_t* d_out_src, int64_t* nnz_off, void* stream)
{
  static const char* who = "hdd_block_operators_map_device";
  if (!ctx || !d_out_row_ptr) return set_error(HDD_ERR_INVALID, std::string(who) + ": null argument");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, who);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  int64_t n = 0;
  if (int rc = ops_upload(ctx, pattern, n_ops, ops, nullptr, s, &n, who)) return rc;
  auto* d = static_cast<OpDesc*>(ctx->ops_d);
  const unsigned grid = rows_grid(n, ctx->n_cu);
  hipLaunchKernelGGL(ops_count_kernel, dim3(grid), dim3(256), 0, s, pattern->row_ptr, pattern->col, d, int(n_ops), n,
                     d_out_row_ptr);
  if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, who);
  size_t tmp = 0;
  if ((e = hipcub::DeviceScan::InclusiveSum(nullptr, tmp, d_out_row_ptr, d_out_row_ptr, n, s)) != hipSuccess)
    return hip_fail(e, who);
  // scan scratch + (n_ops + 1) totals, kept in the context
  const size_t need = tmp + size_t(n_ops + 1) * sizeof(int64_t) + 256;
  if (need > ctx->scan_ws_bytes) {
    (void)hipStreamSynchronize(s);
    if (ctx->scan_ws) (void)hipFree(ctx->scan_ws);
    ctx->scan_ws = nullptr;
    ctx->scan_ws_bytes = 0;
    if ((e = hipMalloc(&ctx->scan_ws, need)) != hipSuccess) return hip_fail(e, who);
    ctx->scan_ws_bytes = need;
  }
  if ((e = hipcub::DeviceScan::InclusiveSum(ctx->scan_ws, tmp, d_out_row_ptr, d_out_row_ptr, n, s)) != hipSuccess)
    return hip_fail(e, who);
  auto* totals = reinterpret_cast<int64_t*>(static_cast<char*>(ctx->scan_ws) + ((tmp + 255) & ~size_t(255)));
  hipLaunchKernelGGL(ops_base_kernel, dim3(1), dim3(64), 0, s, d_out_row_ptr, d, int(n_ops),
                     nnz_off ? totals : nullptr);
  if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, who);
  hipLaunchKernelGGL(ops_fill_kernel, dim3(grid), dim3(256), 0, s, pattern->row_ptr, pattern->col, d, int(n_ops), n,
                     d_out_row_ptr, d_out_col, d_out_src);
  if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, who);
  if (nnz_off) {
    e = hipMemcpyAsync(nnz_off, totals, size_t(n_ops + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, who);
  }
  return HDD_OK;
}

extern "C" int hdd_block_operators_values_device(hdd_ctx* ctx, const hdd_csr* pattern, int32_t n_ops,
                                                 const hdd_block_range* ops, const int64_t* nnz_off,
                                                 const int64_t* d_out_row_ptr, const double* const* d_vals,
                                                 int32_t n_comp, double* const* d_out, void* stream)
{
  static const char* who = "hdd_block_operators_values_device";
  if (!ctx || !nnz_off || !d_out_row_ptr || !d_vals || !d_out || n_comp < 0 || n_comp > HDD_MAX_COMP)
    return set_error(HDD_ERR_INVALID, std::string(who) + ": invalid argument");
  ValPtrs v{};
  for (int c = 0; c < n_comp; ++c) {
    if (!d_vals[c] || !d_out[c]) return set_error(HDD_ERR_INVALID, std::string(who) + ": null value array");
    v.in[c] = d_vals[c];
    v.out[c] = d_out[c];
  }
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, who);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  int64_t n = 0;
  if (int rc = ops_upload(ctx, pattern, n_ops, ops, nnz_off, s, &n, who)) return rc;
  if (n_comp == 0) return HDD_OK;
  hipLaunchKernelGGL(ops_values_kernel, dim3(rows_grid(n, ctx->n_cu)), dim3(256), 0, s, pattern->row_ptr, pattern->col,
                     static_cast<const OpDesc*>(ctx->ops_d), int(n_ops), n, d_out_row_ptr, v, int(n_comp));
  e = hipGetLastError();
  return e == hipSuccess ? HDD_OK : hip_fail(e, who);
}


extern "C" int hdd_block_operator_map_device(hdd_ctx* ctx, const hdd_csr* pattern, int64_t row_begin, int64_t row_end,
                                             int64_t col_begin, int64_t col_end, int64_t* d_out_row_ptr,
                                             int32_t* d_out_col, int64_t* d_out_src, int64_t* nnz, void* stream)
{
  if (!ctx || !d_out_row_ptr) return set_error(HDD_ERR_INVALID, "hdd_block_operator_map_device: null argument");
  if (int rc = subcsr_check(pattern, row_begin, row_end, col_begin, col_end, "hdd_block_operator_map_device")) return rc;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_block_operator_map_device: hipSetDevice");
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = row_end - row_begin;
  const unsigned grid = rows_grid(n, ctx->n_cu);
  hipLaunchKernelGGL(subcsr_count_kernel, dim3(grid), dim3(256), 0, s, pattern->row_ptr, pattern->col, row_begin, n,
                     col_begin, col_end, d_out_row_ptr);
  if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "hdd_block_operator_map_device: count");
  if (n > 0) {
    size_t tmp = 0;
    e = hipcub::DeviceScan::InclusiveSum(nullptr, tmp, d_out_row_ptr + 1, d_out_row_ptr + 1, n, s);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_operator_map_device: scan size");
    if (tmp > ctx->scan_ws_bytes) {   // grows once per context (one stream at a time per context)
      (void)hipStreamSynchronize(s);
      if (ctx->scan_ws) (void)hipFree(ctx->scan_ws);
      ctx->scan_ws = nullptr;
      ctx->scan_ws_bytes = 0;
      if ((e = hipMalloc(&ctx->scan_ws, tmp)) != hipSuccess) return hip_fail(e, "hdd_block_operator_map_device: scratch");
      ctx->scan_ws_bytes = tmp;
    }
    e = hipcub::DeviceScan::InclusiveSum(ctx->scan_ws, tmp, d_out_row_ptr + 1, d_out_row_ptr + 1, n, s);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_operator_map_device: scan");
  }
  if (d_out_col) {
    hipLaunchKernelGGL(subcsr_fill_kernel, dim3(grid), dim3(256), 0, s, pattern->row_ptr, pattern->col, row_begin, n,
                       col_begin, d_out_row_ptr, d_out_col, d_out_src);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "hdd_block_operator_map_device: fill");
  }
  if (nnz) {
    e = hipMemcpyAsync(nnz, d_out_row_ptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_operator_map_device: read nnz");
  }
  return HDD_OK;
}

extern "C" int hdd_block_operator_values_device(hdd_ctx* ctx, const hdd_csr* pattern, int64_t row_begin, int64_t row_end,
                                                int64_t col_begin, int64_t col_end, const int64_t* d_out_row_ptr,
                                                const double* const* d_vals, int32_t n_comp, double* const* d_out,
                                                void* stream)
{
  if (!ctx || !d_out_row_ptr || !d_vals || !d_out || n_comp < 0 || n_comp > HDD_MAX_COMP)
    return set_error(HDD_ERR_INVALID, "hdd_block_operator_values_device: invalid argument");
  if (int rc = subcsr_check(pattern, row_begin, row_end, col_begin, col_end, "hdd_block_operator_values_device")) return rc;
  ValPtrs v{};
  for (int c = 0; c < n_comp; ++c) {
    if (!d_vals[c] || !d_out[c]) return set_error(HDD_ERR_INVALID, "hdd_block_operator_values_device: null value array");
    v.in[c] = d_vals[c];
    v.out[c] = d_out[c];
  }
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_block_operator_values_device: hipSetDevice");
  const int64_t n = row_end - row_begin;
  if (n == 0 || n_comp == 0) return HDD_OK;
  hipLaunchKernelGGL(subcsr_values_kernel, dim3(rows_grid(n, ctx->n_cu)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     pattern->row_ptr, pattern->col, row_begin, n, col_begin, d_out_row_ptr, v, int(n_comp));
  e = hipGetLastError();
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_block_operator_values_device: launch");
}
