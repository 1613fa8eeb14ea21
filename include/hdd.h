/*
 * include/hdd.h -- C ABI of the MI355X SWIPDG assembly engine (libhdd_amd.so).
 *
 * Drop-in boundary for dune-hdd's linearelliptic SWIPDG / BlockSWIPDG hot path.  The reference has no
 * C ABI (its boundary is C++ templates over dune-gdt's SystemAssembler); every entry point below names
 * the reference interface it replaces.  Conventions:
 *   - plain C types and pointers only; "device" pointers are HIP device memory owned by the caller;
 *   - every function returns HDD_OK (0) or an HDD_ERR_* code, never throws; hdd_last_error(ctx) (or
 *     hdd_last_error(NULL) for functions without a context) returns the message of the last failure
 *     of the calling thread;
 *   - device work is enqueued on the hipStream_t passed as `stream` (NULL = legacy default stream) and
 *     is NOT synchronised; no synchronisation happens inside hdd_swipdg_assemble / hdd_affine_lincomb /
 *     hdd_soa_gather / hdd_soa_scatter, and no allocation either except that hdd_swipdg_assemble on
 *     HDD_HEX p=3 meshes grows a context-owned workspace the first time a context sees a larger mesh --
 *     8 * (72 n + 1280 ceil(n / 16) + 2 n) bytes for n owned elements (the 576-byte element records, the
 *     GEMM coefficient fragments of 80 doubles per element padded to groups of 16, 16 bytes of layout per
 *     element; ~1.23 KB per element) -- and allocates, on its first p=3 call, the context's 80 x 4096 table
 *     of reference matrices (2.6 MB): warm a context up once, then the calls are hipGraph-capturable;
 *   - one context per thread at a time (thread-compatible, like the reference's single-threaded init()),
 *     and one stream at a time per context: the HDD_HEX p=3 coefficient records live in a per-context
 *     workspace, so concurrent assemblies on different streams need different contexts.
 *
 * Numbering: DoF (row / column) of local basis function i of element g is g*nb + i (element-blocked,
 * as dune-fem's DG mapper); a CSR row holds the DoFs of its element and of every face neighbour, sorted
 * ascending (the EllipticSWIPDG pattern, swipdg.hh:169).  Block-SWIPDG numbering is the same rule applied
 * to a subdomain-major element order (Spaces::Block::mapToGlobal(ss, ii) = offset(ss) + ii,
 * block-swipdg.hh:1042, 1093), which all hdd_grid_* builders produce.
 */
#ifndef HDD_H
#define HDD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDD_ABI_VERSION 8   /* 3: hdd_mesh vertex-indexed geometry, hdd_local_vertices;
                               4: HDD_FN_FLATTOP (hdd_scalar_fn.table / n_table), hdd_indicator_sum;
                               5: hdd_shard_info.halo_elements, hdd_swipdg_assemble_elements;
                               6: hdd_grid_create_hex_from_connectivity;
                               7: in-process device transport (hdd_device_hub, hdd_comm_create_device);
                               8: sharded-step watchdog (hdd_block_step_mark / _query / _sync, HDD_ERR_TIMEOUT), the
                                  device transport's stall injection, verification variants (hdd_ctx_set_variant) */
#define HDD_MAX_COMP 8

typedef enum {
  HDD_OK = 0,
  HDD_ERR_INVALID = 1,      /* wrong input given (Stuff::Exceptions::wrong_input_given) */
  HDD_ERR_HIP = 2,          /* HIP runtime failure */
  HDD_ERR_UNSUPPORTED = 3,  /* NotImplemented in the reference's sense */
  HDD_ERR_NOMEM = 4,
  HDD_ERR_RANGE = 5,        /* index_out_of_range */
  HDD_ERR_TIMEOUT = 6       /* a deadline passed (hdd_block_step_sync: a sharded step that did not complete) */
} hdd_status;

enum { HDD_SIMPLEX = 0, HDD_CUBE = 1,                       /* P1 triangles / Q1 parallelograms (2d) */
       HDD_HEX = 2 };                                        /* Q_p (p = 1..3) on affine hexahedra (3d) */
enum { HDD_NBR_DIRICHLET = -1, HDD_NBR_NEUMANN = -2 };       /* neighbour codes of domain-boundary faces */
enum { HDD_FN_CONST = 0, HDD_FN_PER_ELEM = 1, HDD_FN_SINUSOID = 2, HDD_FN_COS_PRODUCT = 3, HDD_FN_FLATTOP = 4 };
#define HDD_FLATTOP_REC 7      /* doubles per HDD_FN_FLATTOP box: lx, ly, ux, uy, layer_x, layer_y, value */
enum { HDD_TENSOR_CONST = 0, HDD_TENSOR_ISO_PER_ELEM = 1, HDD_TENSOR_SYM_PER_ELEM = 2 };
enum { HDD_BOUNDARY_ALL_DIRICHLET = 0, HDD_BOUNDARY_ALL_NEUMANN = 1 };

typedef struct hdd_ctx hdd_ctx;
typedef struct hdd_grid hdd_grid;
typedef struct hdd_local hdd_local;

/* ---------------------------------------------------------------------------------------------- */
/* context                                                                                         */
/* ---------------------------------------------------------------------------------------------- */
int hdd_abi_version(void);
/* binds `hip_device`; replaces nothing in the reference (DUNE is host-only) */
int hdd_ctx_create(int hip_device, hdd_ctx** out);
void hdd_ctx_destroy(hdd_ctx* ctx);
/* error injection of the tests (the HDD_DEBUG_FLAGS value a context reads at creation; 0 in production).
 * Bit 524288: hdd_swipdg_rhs's face launch is treated as failed (the call returns HDD_ERR_HIP after its volume
 * kernel; the next call must still be correct).  Profiling ablations exist only in the separate -DHDD_ABLATION
 * build (make ablation: lib_ab/libhdd_abl.so); the product library ignores every other bit. */
int hdd_ctx_set_debug_flags(hdd_ctx* ctx, int32_t flags);
/* Verification variants (ABI 8): alternative implementations of the same values, selected per context (or by the
 * HDD_VARIANT value a context of the -DHDD_ABLATION build reads at creation; the product library takes no kernel
 * choice from the environment) so that the tests can compare them bit for bit / to rounding with the default kernels.  Default 0: the kernels the dispatch picks for performance. */
enum {
  HDD_VARIANT_Q1_WHOLE_TILE = 1,      /* Q1: the whole-tile image kernel on every mesh (the default on element-major
                                         meshes and on the sharded step's SKIP launches) instead of the half-image one */
  HDD_VARIANT_ELEMENT_MAJOR = 2,      /* ignore the mesh's vertex-indexed geometry (element-major coordinates) */
  HDD_VARIANT_C3_PER_COMPONENT = 4,   /* OS2014 sinusoid components: one launch per component, not the fused one */
  HDD_VARIANT_WAVE_PER_ROW = 8,       /* the generic wave-per-row kernels instead of the persistent tile policies */
  HDD_VARIANT_P1_SMOOTH_QUADRATURE = 16,   /* P1 smooth kappa: the quadrature policy instead of the moments */
  HDD_VARIANT_HEX_Q3_REGISTER = 32,   /* hexahedra p = 3: the register-fragment MFMA kernel, not the GEMM one */
  HDD_VARIANT_PATTERN_SCAN_COPY = 64, /* device pattern nnz by a scan launch + device-to-host copy */
  HDD_VARIANT_RHS_FUSED = 128,        /* 2d RHS: one fused kernel instead of volume kernel + boundary-element list */
  HDD_VARIANT_RHS_GENERIC = 256,      /* RHS: the run-time-rule kernel only */
  HDD_VARIANT_RHS_NO_TINY = 512       /* RHS: no small-phase polynomial tier for the force's cos products */
};
int hdd_ctx_set_variant(hdd_ctx* ctx, uint32_t variant);
/* message of the last failure on this thread (ctx may be NULL); never NULL */
const char* hdd_last_error(const hdd_ctx* ctx);
/* the instantiation name of the last persistent tile kernel this thread launched ("" if none; ABI 8): what the
 * dispatch actually picked, e.g. for a benchmark's kernel label.  Element-list passes are not recorded. */
const char* hdd_last_tile_kernel(void);

/* ---------------------------------------------------------------------------------------------- */
/* grids (host) -- replace the grid providers the reference builds its spaces on:                  */
/*   Stuff::Grid::Providers::Cube (testcases/ESV2007.hh:123-129, testcases/spe10.hh:301-307) and     */
/*   grid::Multiscale::Providers::Cube with num_partitions (testcases/base.hh:150-191)             */
/* ---------------------------------------------------------------------------------------------- */
typedef struct {
  int32_t elem_type;          /* HDD_SIMPLEX: Kuhn split of every square (createSimplexGrid); HDD_CUBE */
  int32_t nx, ny;             /* squares per direction */
  int32_t px, py;             /* subdomain partition ("num_partitions" [px py 1]); 1,1 = monolithic */
  int32_t boundary;           /* HDD_BOUNDARY_* applied to every domain-boundary face */
  int32_t pad;
  double lower[2], upper[2];
} hdd_structured_desc;

/* 3d structured grid of nx x ny x nz axis-aligned hexahedra (SGrid / YaspGrid cube provider in 3d),
 * px x py x pz subdomains (subdomain id (sx*py + sy)*pz + sz: x-slabs are contiguous element ranges);
 * inside a subdomain elements are lexicographic (x fastest).  Faces: 2a (x_a = 0 side), 2a+1. */
typedef struct {
  int32_t nx, ny, nz;
  int32_t px, py, pz;
  int32_t boundary;           /* HDD_BOUNDARY_* */
  int32_t degree;             /* polynomial degree p of the DG Q_p space carried by the grid (1..3) */
  double lower[3], upper[3];
} hdd_structured3_desc;

typedef struct {
  int32_t elem_type, nb, nfaces, nvpe;   /* nb = basis functions per element of the carried DG space */
  int64_t n_elements, n_vertices;
  int32_t n_subdomains, dim;
} hdd_grid_info;

int hdd_grid_create_structured(const hdd_structured_desc* desc, hdd_grid** out);
/* 3d (C5: ESV2007 3d structured, SWIPDG p=3) */
int hdd_grid_create_structured_3d(const hdd_structured3_desc* desc, hdd_grid** out);
/* general conforming 2d mesh from connectivity (vertex order = Dune reference element order);
 * `subdomain` (nullable) assigns elements to subdomains, elements are then renumbered subdomain-major */
int hdd_grid_create_from_connectivity(int32_t elem_type, int64_t n_vertices, const double* vertex_coords,
                                      int64_t n_elements, const int32_t* elem_vert, const int32_t* subdomain,
                                      int32_t n_subdomains, int32_t boundary, hdd_grid** out);
/* general conforming 3d mesh of axis-aligned hexahedra from connectivity (vertex_coords [n_vertices][3],
 * elem_vert [n_elements][8] in Dune cube vertex order: vertex k at lower + ((k&1), (k>>1)&1, k>>2) * h),
 * carrying the DG Q_`degree` space (1..3); shared faces must be aligned (twin face f^1, the layout every
 * subset of a structured hex grid has).  Replaces the grid part the reference hands to an oversampled local
 * discretization in 3d (MsGrid::local_oversampled grid part, block-swipdg.hh:783-817); HDD_ERR_UNSUPPORTED
 * for a non-box element or a misaligned shared face. */
int hdd_grid_create_hex_from_connectivity(int32_t degree, int64_t n_vertices, const double* vertex_coords,
                                          int64_t n_elements, const int32_t* elem_vert, const int32_t* subdomain,
                                          int32_t n_subdomains, int32_t boundary, hdd_grid** out);
void hdd_grid_destroy(hdd_grid* g);
int hdd_grid_get_info(const hdd_grid* g, hdd_grid_info* out);
/* element range [first, last) of the subdomains [s_begin, s_end) in the (subdomain-major) numbering */
int hdd_grid_subdomain_range(const hdd_grid* g, int32_t s_begin, int32_t s_end, int64_t* first, int64_t* last);
/* global element -> (vertex ids [nvpe]) and subdomain ids, for tests / visualisation (host arrays) */
int hdd_grid_connectivity(const hdd_grid* g, double* vertex_coords, int32_t* elem_vert, int32_t* subdomain);

/* Rank-local view: the elements of subdomains [s_begin, s_end) ("owned") plus the ghost elements that
 * share a face with them, laid out [ghosts with smaller global id][owned][ghosts with larger global id]
 * so that local order == global order (owner-computes rows, block-swipdg.hh:355-382). */
typedef struct {
  int64_t n_local, own_begin, own_end, n_ghost;
  int64_t global_first;       /* global id of the first owned element */
} hdd_local_info;

int hdd_local_create(const hdd_grid* g, int32_t s_begin, int32_t s_end, hdd_local** out);
void hdd_local_destroy(hdd_local* l);
int hdd_local_get_info(const hdd_local* l, hdd_local_info* out);
/* host SoA arrays, n_local columns each:
 *   coords    [dim*nvpe][n_local]: coordinate c of vertex k at (dim*k + c)*n_local + e (ghosts too)
 *   neighbors [nfaces][n_local] : local neighbour id or HDD_NBR_* (ghost columns: -3)
 *   face_info [n_local]         : 4 bits per face: twin local face (bits 0-2), reversed (bit 3)
 *   global_id [n_local]         : global element id
 *   subdomain [n_local]         : subdomain of the element
 * any pointer may be NULL */
int hdd_local_fill(const hdd_local* l, double* coords, int32_t* neighbors, uint32_t* face_info,
                   int64_t* global_id, int32_t* subdomain);
/* element barycentres [dim][n_local] (coefficient lookup, e.g. the Spe10 checkerboard) */
int hdd_local_centers(const hdd_local* l, double* centers);
/* vertex-indexed geometry of the local elements (owned + ghosts), the grid's own representation (a Dune
 * grid's vertex set + element -> vertex map): the distinct vertices of the local elements, numbered in
 * ascending global vertex id, *n_vertices of them;
 *   elem_vertices [nvpe][n_local]   : local vertex id of vertex k of element e at k*n_local + e
 *   vertex_coords [n_vertices][dim] : coordinates, interleaved
 * Call with elem_vertices == vertex_coords == NULL to query *n_vertices. */
int hdd_local_vertices(const hdd_local* l, int64_t* n_vertices, int32_t* elem_vertices, double* vertex_coords);
/* halo plan with the subdomain -> rank map `owner` [n_subdomains]:
 *   peers[n_peers] ranks this rank exchanges with (ascending); for peer p: send_count[p] owned elements
 *   whose local ids are listed by hdd_local_send_list(l, p, ...), and recv_count[p] ghost slots starting
 *   at local id recv_offset[p] (ghosts of one owner are contiguous).  Call with peers == NULL to query
 *   n_peers. */
int hdd_local_halo_plan(const hdd_local* l, const int32_t* owner, int32_t my_rank, int32_t* n_peers,
                        int32_t* peers, int64_t* send_count, int64_t* recv_offset, int64_t* recv_count);
int hdd_local_send_list(const hdd_local* l, const int32_t* owner, int32_t my_rank, int32_t peer_index,
                        int32_t* local_ids);

/* dune-stuff Checkerboard evaluated at element barycentres: value of cell (cx, cy), x fastest */
int hdd_checkerboard(int64_t n, const double* centers /*[2][n]*/, const double lower[2], const double upper[2],
                     int32_t ncx, int32_t ncy, const double* cell_values, double* out);
/* dune-stuff Indicator evaluated at element barycentres (problems/spe10.hh:144, 157: the SPE10 channel and
 * force): value of the first closed box [lx, ux] x [ly, uy] containing the barycentre, 0 if none;
 * boxes[5k .. 5k+4] = lx, ly, ux, uy, value */
int hdd_indicator(int64_t n, const double* centers /*[2][n]*/, int32_t n_boxes, const double* boxes, double* out);
/* the sum of one-box Indicators (make_sum of the channel's per-box functions, problems/spe10.hh:139-148 with
 * channel_boundary_layer == 0): sum of the values of every closed box containing the barycentre */
int hdd_indicator_sum(int64_t n, const double* centers /*[2][n]*/, int32_t n_boxes, const double* boxes, double* out);
/* The SPE10 Model1 permeability data file (problems/spe10.hh:151-156: Spe10FunctionType(filename, lower_left,
 * upper_right, model1_min_value, model1_max_value)).  dune-stuff's reader is not in the reference tree; restated
 * (parity unpinned): whitespace-separated numbers, of which the first HDD_SPE10_MODEL1_CELLS (100 x 20, x
 * fastest -- the file holds 6000) are the cells of the 100 x 20 checkerboard, mapped affinely so that
 * [HDD_SPE10_MODEL1_MIN, HDD_SPE10_MODEL1_MAX] goes onto [min_value, max_value] (the identity for the values the
 * reference passes).  cells: [HDD_SPE10_MODEL1_CELLS].  Missing / short file or max_value <= min_value:
 * HDD_ERR_INVALID. */
#define HDD_SPE10_MODEL1_NX 100
#define HDD_SPE10_MODEL1_NZ 20
#define HDD_SPE10_MODEL1_CELLS 2000
#define HDD_SPE10_MODEL1_MIN 0.001
#define HDD_SPE10_MODEL1_MAX 998.915
int hdd_spe10_model1_read(const char* filename, double min_value, double max_value, double* cells);

/* ---------------------------------------------------------------------------------------------- */
/* sparsity pattern (host) -- replaces EllipticSWIPDG::pattern(test, ansatz) (swipdg.hh:169) and the */
/* block pattern of add_local_to_global_pattern / compute_face_pattern (block-swipdg.hh:304-325,     */
/* 1036-1049).  Rows of the owned elements, global columns.                                          */
/* ---------------------------------------------------------------------------------------------- */
int hdd_pattern_count(int32_t elem_type, int64_t n_local, int64_t own_begin, int64_t own_end,
                      const int32_t* neighbors, int64_t* nnz);
/* row_ptr [nb*(own_end-own_begin)+1], col [nnz], elem_ptr [own_end-own_begin+1] (= row_ptr[k*nb]);
 * global_id may be NULL (local == global) */
int hdd_pattern_fill(int32_t elem_type, int64_t n_local, int64_t own_begin, int64_t own_end,
                     const int32_t* neighbors, const int64_t* global_id, int64_t* row_ptr, int32_t* col,
                     int64_t* elem_ptr);
/* the same for any DG space: n_faces faces and nb basis functions per element (Q_p: nb = (p+1)^dim);
 * n_faces = 0 gives the element-local (volume) pattern of the l2 / h1_semi / elliptic / boundary_l2 products */
int hdd_dg_pattern_count(int32_t n_faces, int32_t nb, int64_t n_local, int64_t own_begin, int64_t own_end,
                         const int32_t* neighbors, int64_t* nnz);
int hdd_dg_pattern_fill(int32_t n_faces, int32_t nb, int64_t n_local, int64_t own_begin, int64_t own_end,
                        const int32_t* neighbors, const int64_t* global_id, int64_t* row_ptr, int32_t* col,
                        int64_t* elem_ptr);


/* ---------------------------------------------------------------------------------------------- */
/* device assembly -- replaces the LHS part of SWIPDG::init() (swipdg.hh:222-249 + walk() at 485):   */
/* one GDT::Operators::EllipticSWIPDG per diffusion-factor component = LocalEvaluation::Elliptic +    */
/* SWIPDG::Inner + SWIPDG::BoundaryLHS, scattered into Q+1 CSR value arrays on one pattern; and the  */
/* BlockSWIPDG boundary / coupling assemblers (block-swipdg.hh:1136-1179, 1270-1326).                */
/* ---------------------------------------------------------------------------------------------- */
typedef struct hdd_mesh_s {
  int32_t elem_type;          /* HDD_SIMPLEX | HDD_CUBE | HDD_HEX */
  int32_t degree;             /* polynomial degree p of the DG space (0 or 1: P1 / Q1; HDD_HEX: 1..3) */
  int64_t n_local;            /* columns of the SoA arrays (owned + ghosts) */
  int64_t own_begin, own_end; /* elements whose rows are assembled */
  const double* coords;       /* device, layout of hdd_local_fill */
  const int32_t* neighbors;   /* device */
  const uint32_t* face_info;  /* device */
  /* optional vertex-indexed geometry (hdd_local_vertices; both or neither, device): when present, the 2d
   * P1 / Q1 stiffness kernels read each element's vertices through elem_vertices from vertex_coords and
   * the neighbour's off-face vertex through its vertex id, instead of the element-major coords (4 B per
   * element vertex instead of 16; the shared vertex rows stay cache resident).  coords stays required
   * (right-hand sides, products, 3d, halo geometry).  The two representations must describe the SAME
   * geometry: a caller that moves the mesh or fills ghost coordinates itself must update vertex_coords too,
   * or pass elem_vertices = vertex_coords = NULL (the sharded step does the latter with
   * HDD_SHARD_HALO_GEOMETRY, whose ghost coordinates arrive in coords only). */
  const int32_t* elem_vertices;  /* [nvpe][n_local] */
  const double* vertex_coords;   /* [n_vertices][dim] */
} hdd_mesh;

typedef struct {              /* one diffusion-factor component kappa_q (a Stuff::LocalizableFunction) */
  int32_t kind;               /* HDD_FN_* */
  int32_t order;              /* integration order of the function (Expression: integration_order) */
  double c;                   /* CONST value, SINUSOID offset a */
  double b, kx, ky;           /* SINUSOID: a + b*sin(kx*x + ky*y);
                                 COS_PRODUCT: a*cos(kx*x)*cos(ky*y) [*cos(b*z) in 3d when b != 0]
                                 (ESV2007 Testcase1Force, problems/ESV2007.hh:78) -- right-hand sides */
  const double* per_elem;     /* PER_ELEM: device [n_local] */
  /* FLATTOP: c + b * sum_k value_k phi(x; lx_k, ux_k, layer_x_k) phi(y; ly_k, uy_k, layer_y_k) -- the sum of
   * dune-stuff FlatTop functions the Spe10::Model1 channel is built from when channel_boundary_layer != 0
   * (problems/spe10.hh:139-148, 213-222): per coordinate 1 on [l + d, u - d], 0 outside [l - d, u + d] and
   * the C^1 cubic transitions (1 + t)^2 (1 - 2t), t = (x - (l + d)) / 2d in [-1, 0), and (1 - t)^2 (1 + 2t),
   * t = (x - (u - d)) / 2d in [0, 1) (layers d > 0).  `order` is the integration order the caller
   * assigns to the function (Stuff's order()).  2d meshes only. */
  const double* table;        /* FLATTOP: device [n_table][HDD_FLATTOP_REC] */
  int32_t n_table;            /* FLATTOP: number of boxes */
  int32_t pad1;
} hdd_scalar_fn;

typedef struct {              /* the (non-parametric) diffusion tensor A */
  int32_t kind;               /* HDD_TENSOR_* */
  int32_t pad;
  double c[6];                /* CONST: 2d a11 a12 a22; 3d a11 a12 a13 a22 a23 a33 */
  const double* per_elem;     /* ISO: device [n_local]; SYM: device [3 | 6][n_local] */
} hdd_tensor_fn;

typedef struct {
  double sigma_inner;         /* LocalEvaluation::SWIPDG::internal::inner_sigma(p)    (8 at p=1) */
  double sigma_boundary;      /* LocalEvaluation::SWIPDG::internal::boundary_sigma(p) (14 at p=1) */
  double beta;                /* LocalEvaluation::SWIPDG::internal::default_beta(d) = 1/(d-1) (swipdg.hh:168) */
  int32_t vol_order;          /* -1: the reference's integrand order (ord kappa + ord A + 2 max(p-1, 0)) */
  int32_t face_order;         /* -1: ord kappa + ord A + 2p */
} hdd_swipdg_params;

typedef struct {
  int64_t n_rows, n_cols, nnz;
  const int64_t* row_ptr;     /* device [n_rows+1] */
  const int32_t* col;         /* device [nnz] */
  const int64_t* elem_ptr;    /* device [n_owned+1]: first value of each owned element's row block */
} hdd_csr;

/* Device pattern build (the pattern of a p=3 3d mesh is ~4 bytes x 28672 per
 * element, too large to build on the host).  Step 1 writes d_elem_ptr [n_own+1] and returns the total
 * nnz in *nnz (host; synchronises `stream`; the kernel writes nnz into a mapped pinned word the context
 * allocates on its first call, so one stream at a time per context).  Step 2 writes d_row_ptr [nb*n_own+1] and d_col [nnz];
 * d_global_id [n_local] maps local to global element ids (NULL: local == global). */
int hdd_pattern_elem_ptr_device(hdd_ctx* ctx, const hdd_mesh* mesh, int32_t nb, int64_t* d_elem_ptr,
                                int64_t* nnz, void* stream);
int hdd_pattern_fill_device(hdd_ctx* ctx, const hdd_mesh* mesh, int32_t nb, const int64_t* d_global_id,
                            const int64_t* d_elem_ptr, int64_t* d_row_ptr, int32_t* d_col, void* stream);

/* Writes d_vals[q][0..nnz) for q < n_comp (each value exactly once, no atomics, no zero-fill needed).
 * Face terms are evaluated by the row owner on both sides of each face (owner-computes). */
int hdd_swipdg_assemble(hdd_ctx* ctx, const hdd_mesh* mesh, const hdd_scalar_fn* kappa, int32_t n_comp,
                        const hdd_tensor_fn* tensor, const hdd_swipdg_params* params, const hdd_csr* pattern,
                        double* const* d_vals, void* stream);

/* Same, restricted to the 64-element tiles d_tiles[0..n_tiles) (tile t = owned elements
 * [own_begin + 64t, own_begin + 64t + 64)): lets a sharded assembly run its interior tiles while the face
 * halo is in flight and the halo-dependent tiles afterwards.  Only the thread-per-element kernels
 * (P1 / Q1 with the reference integrand orders) take tile lists; others return HDD_ERR_UNSUPPORTED. */
int hdd_swipdg_assemble_tiles(hdd_ctx* ctx, const hdd_mesh* mesh, const hdd_scalar_fn* kappa, int32_t n_comp,
                              const hdd_tensor_fn* tensor, const hdd_swipdg_params* params, const hdd_csr* pattern,
                              double* const* d_vals, const int32_t* d_tiles, int64_t n_tiles, void* stream);

/* Same, restricted to the single owned elements own_begin + d_elems[0..n_elems) (one lane each, any order,
 * no duplicates): the fixup pass of a sharded step, which assembles every tile while the halo is in flight
 * (ghost rows stale) and then recomputes only the row blocks of elements with a ghost face neighbour.
 * Same kernel coverage as hdd_swipdg_assemble_tiles. */
int hdd_swipdg_assemble_elements(hdd_ctx* ctx, const hdd_mesh* mesh, const hdd_scalar_fn* kappa, int32_t n_comp,
                                 const hdd_tensor_fn* tensor, const hdd_swipdg_params* params,
                                 const hdd_csr* pattern, double* const* d_vals, const int32_t* d_elems,
                                 int64_t n_elems, void* stream);

/* SWIPDG right-hand side -- replaces the functionals of SWIPDG::init() (swipdg.hh:251-347):
 *   L2Volume(force) + DirichletBoundarySWIPDG(kappa, tensor, dirichlet) on Dirichlet faces
 *   + L2Face(neumann) on Neumann faces, each of force / dirichlet / neumann nullable (absent = zero).
 * Writes d_rhs[k*nb + i] for every owned element k (local order) and basis function i; one call per
 * affine component of the right-hand side (the caller pairs kappa / dirichlet components as swipdg.hh
 * does).  Integration orders: ord(f) + p; Neumann ord(g_N) + p; Dirichlet max(ord(g_D) + p,
 * ord(kappa) + ord(A) + p - 1 + ord(g_D)).  2d meshes with Dirichlet or Neumann data: two launches (volume
 * kernel, then a face kernel over the boundary elements the first one listed) on a list the context holds
 * (16 B per owned element, allocated on the first call of a size class: warm a context up before hipGraph
 * capture).  Eager calls of one context on different streams are ordered behind each other by the library (an
 * event on the previous call's stream).  A CAPTURED call is not: the replays of a graph that captured an
 * hdd_swipdg_rhs call of context C must not run concurrently with eager hdd_swipdg_rhs calls of C or with replays
 * of another such graph of C (they share C's list); use a separate context per concurrent graph / stream. */
int hdd_swipdg_rhs(hdd_ctx* ctx, const hdd_mesh* mesh, const hdd_scalar_fn* force, const hdd_scalar_fn* kappa,
                   const hdd_tensor_fn* tensor, const hdd_scalar_fn* dirichlet, const hdd_scalar_fn* neumann,
                   const hdd_swipdg_params* params, double* d_rhs, void* stream);

/* Products of SWIPDG::init() (swipdg.hh:358-508; over_integrate = 2) -- BlockSWIPDG's local products
 * (block-swipdg.hh:392-548) are the same on the subdomain's elements:
 *   HDD_PRODUCT_L2, _H1_SEMI, _ELLIPTIC (kappa, tensor), _BOUNDARY_L2: element-local blocks; pattern =
 *   hdd_dg_pattern_fill with n_faces = 0 (row length nb);
 *   HDD_PRODUCT_PENALTY (kappa, tensor): the SWIPDG penalty terms sigma kappa^- kappa^+ gamma / |F|^beta on
 *   inner faces and the boundary penalty on Dirichlet faces; pattern = the SWIPDG pattern.
 * Writes d_vals[0..nnz) (every entry once). */
enum { HDD_PRODUCT_L2 = 0, HDD_PRODUCT_H1_SEMI = 1, HDD_PRODUCT_ELLIPTIC = 2, HDD_PRODUCT_BOUNDARY_L2 = 3,
       HDD_PRODUCT_PENALTY = 4 };
int hdd_product_assemble(hdd_ctx* ctx, const hdd_mesh* mesh, int32_t product, const hdd_scalar_fn* kappa,
                         const hdd_tensor_fn* tensor, const hdd_swipdg_params* params, const hdd_csr* pattern,
                         double* d_vals, void* stream);

/* theta-lincomb of affine components on a shared pattern -- replaces
 * AffinelyDecomposedContainer::freeze_parameter(mu) as used by ContainerBasedDefault::uncached_solve
 * (base.hh:338-341, 357-361):  out[s][k] = sum_q theta[s*n_comp+q] * d_vals[q][k]  (theta on host) */
int hdd_affine_lincomb(hdd_ctx* ctx, int64_t nnz, const double* const* d_vals, int32_t n_comp,
                       const double* theta, int32_t n_samples, double* d_out, int64_t out_stride, void* stream);

/* ---------------------------------------------------------------------------------------------- */
/* halo records (face-coupling ghosts of a sharded BlockSWIPDG) -- SoA gather / scatter of element    */
/* columns; the transport itself is RCCL send/recv (torch.distributed) between the two calls.         */
/* ---------------------------------------------------------------------------------------------- */
/* buf[(r)*n + i] = arrays[a][row(a,r)*ld + idx[i]] for the concatenated rows of all arrays */
int hdd_soa_gather(hdd_ctx* ctx, const double* const* arrays, const int32_t* rows, int32_t n_arrays, int64_t ld,
                   const int32_t* d_idx, int64_t n, double* d_buf, void* stream);
/* arrays[a][row*ld + dst_offset + i] = buf[r*n + i] */
int hdd_soa_scatter(hdd_ctx* ctx, double* const* arrays, const int32_t* rows, int32_t n_arrays, int64_t ld,
                    int64_t dst_offset, int64_t n, const double* d_buf, void* stream);

/* ---------------------------------------------------------------------------------------------- */
/* block operators -- replaces BlockSWIPDG::get_local_operator(ss) / get_coupling_operator(ss, nn)   */
/* (block-swipdg.hh:625-676): in the subdomain-major numbering they are the diagonal / off-diagonal   */
/* blocks of the global matrix, extracted through a value map built once from the pattern.            */
/* ---------------------------------------------------------------------------------------------- */
/* rows of subdomain ss, columns of subdomain nn (ss == nn: local operator), local numbering on both
 * sides.  Call with out_col == NULL to get *nnz; out_row_ptr [rows+1], out_col / out_src [nnz]
 * (out_src = index of each extracted value in the global value array).  Host arrays. */
int hdd_block_operator_map(const hdd_grid* g, int32_t ss, int32_t nn, const int64_t* row_ptr, const int32_t* col,
                           int64_t* out_row_ptr, int32_t* out_col, int64_t* out_src, int64_t* nnz);
/* d_out[k] = d_vals[d_src[k]] for k < n (device arrays) */
int hdd_gather_values(hdd_ctx* ctx, const double* d_vals, const int64_t* d_src, int64_t n, double* d_out, void* stream);
/* The same on the device, from the device pattern: rows [row_begin, row_end) of `pattern` restricted to the
 * columns [col_begin, col_end) (operator (ss, nn): rows / columns of the element ranges of ss / nn times nb,
 * hdd_grid_subdomain_range), renumbered col - col_begin.  Writes d_out_row_ptr [rows+1] always; d_out_col /
 * d_out_src [nnz] when d_out_col != NULL (d_out_src nullable); *nnz (host) when nnz != NULL, which
 * synchronises `stream` -- call once with d_out_col == NULL and nnz to size the arrays, or pass the known
 * nnz (nb^2 x the ss/nn element-face pairs, plus nb^2 |ss| for ss == nn) and stay asynchronous. */
int hdd_block_operator_map_device(hdd_ctx* ctx, const hdd_csr* pattern, int64_t row_begin, int64_t row_end,
                                  int64_t col_begin, int64_t col_end, int64_t* d_out_row_ptr, int32_t* d_out_col,
                                  int64_t* d_out_src, int64_t* nnz, void* stream);
/* the operator's values of n_comp value arrays on `pattern` (d_out_row_ptr from the map call): no index map */
int hdd_block_operator_values_device(hdd_ctx* ctx, const hdd_csr* pattern, int64_t row_begin, int64_t row_end,
                                     int64_t col_begin, int64_t col_end, const int64_t* d_out_row_ptr,
                                     const double* const* d_vals, int32_t n_comp, double* const* d_out, void* stream);

/* Batched: n_ops operators of one pattern in four launches (count, one scan over all, bases, fill) -- e.g.
 * every get_local_operator / get_coupling_operator of a BlockSWIPDG at once.  Outputs are concatenated:
 * operator k's row pointer [rows_k + 1] (operator-relative, starting at 0) is at d_out_row_ptr + row_off_k,
 * row_off_k = sum_{j<k} (rows_j + 1); its local columns / source positions at d_out_col / d_out_src +
 * nnz_off[k] (either may be NULL), nnz_off[k+1] = nnz_off[k] + nnz_k + (nnz_k & 1): every operator starts
 * 16-byte aligned in the value arrays (one padding entry after an odd count, left unwritten).  nnz_off (host
 * [n_ops + 1], nnz_off[n_ops] = the padded total) is returned when non-NULL, which synchronises `stream`; a
 * caller that knows the counts (from the mesh: nb^2 x face pairs, + nb^2 |ss| on the diagonal) passes NULL
 * and stays asynchronous.  sum_k (rows_k + 1) < 2^31. */
typedef struct {
  int64_t row_begin, row_end, col_begin, col_end;
} hdd_block_range;
int hdd_block_operators_map_device(hdd_ctx* ctx, const hdd_csr* pattern, int32_t n_ops, const hdd_block_range* ops,
                                   int64_t* d_out_row_ptr, int32_t* d_out_col, int64_t* d_out_src, int64_t* nnz_off,
                                   void* stream);
/* the operators' values of n_comp value arrays (concatenated like the columns; nnz_off host [n_ops + 1]) */
int hdd_block_operators_values_device(hdd_ctx* ctx, const hdd_csr* pattern, int32_t n_ops, const hdd_block_range* ops,
                                      const int64_t* nnz_off, const int64_t* d_out_row_ptr, const double* const* d_vals,
                                      int32_t n_comp, double* const* d_out, void* stream);

/* ---------------------------------------------------------------------------------------------- */
/* sharded BlockSWIPDG (SURVEY.md 8(b) hdd_block_assemble_sharded, 8(e)): one process (or thread) per  */
/* GPU owns a contiguous range of subdomains and assembles their rows -- A_ss and A_ss,nn are written  */
/* by the owner of ss (block-swipdg.hh:355-382, coupling 1270-1326, boundary 1136-1179), so there is  */
/* no reduction; the only exchange is the face halo (per-element records of the ghost elements).      */
/* ---------------------------------------------------------------------------------------------- */
typedef struct hdd_comm hdd_comm;
typedef struct hdd_shard hdd_shard;

#define HDD_RCCL_ID_BYTES 128   /* sizeof(ncclUniqueId) */

/* Host transport: moves n_peers messages (host memory, doubles) and returns HDD_OK; message k goes to
 * rank peers[k] (send[k], send_count[k] doubles) and the message of that rank lands in recv[k]
 * (recv_count[k] doubles).  Called synchronously from hdd_comm_post on the caller's thread (e.g. MPI,
 * gloo or an in-process mailbox). */
typedef int (*hdd_host_exchange_fn)(void* user, int32_t n_peers, const int32_t* peers, const double* const* send,
                                    const int64_t* send_count, double* const* recv, const int64_t* recv_count);

/* RCCL (librccl, resolved at run time in the calling process: PyTorch-ROCm's copy when it is loaded)
 * -- ncclGetUniqueId on one rank, broadcast the HDD_RCCL_ID_BYTES bytes, ncclCommInitRank on every rank */
int hdd_rccl_get_unique_id(void* id);
int hdd_comm_create_rccl(const void* id, int32_t nranks, int32_t rank, int32_t hip_device, hdd_comm** out);
/* wrap an existing ncclComm_t (not destroyed by hdd_comm_destroy) */
int hdd_comm_wrap_rccl(void* nccl_comm, int32_t hip_device, hdd_comm** out);
/* host-staged transport: device -> pinned host -> fn -> device (synchronous; rehearsal / tests / MPI) */
int hdd_comm_create_host(hdd_host_exchange_fn fn, void* user, int32_t hip_device, hdd_comm** out);
/* In-process device transport (ABI 7): nranks ranks of ONE process, one thread each (any devices, one device
 * allowed), exchanging device buffers with RCCL's stream schedule -- the exchange runs on the communicator's
 * transfer stream: it waits for each source's packed event, copies its messages (hipMemcpyAsync) into the
 * receive buffers, records a "copied" event, and completes (the event hdd_comm_wait joins) once every
 * destination has copied this rank's sends; so the sharded step takes exactly the branch it takes over RCCL.
 * hdd_comm_post blocks the calling thread until every source rank has posted (a host rendezvous; 120 s
 * timeout, then every waiting rank returns HDD_ERR_INVALID).  The hub is reference counted: destroying it
 * while communicators still use it is allowed. */
typedef struct hdd_device_hub hdd_device_hub;
int hdd_device_hub_create(int32_t nranks, hdd_device_hub** out);
void hdd_device_hub_destroy(hdd_device_hub* hub);
int hdd_comm_create_device(hdd_device_hub* hub, int32_t rank, int32_t hip_device, hdd_comm** out);
void hdd_comm_destroy(hdd_comm* comm);
/* Post one exchange of device buffers: it starts after the work enqueued on `stream` so far; RCCL runs
 * it on the communicator's own transfer stream (ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd), so
 * work enqueued on `stream` afterwards overlaps it until hdd_comm_wait(comm, stream). */
int hdd_comm_post(hdd_comm* comm, int32_t n_peers, const int32_t* peers, const double* const* d_send,
                  const int64_t* send_count, double* const* d_recv, const int64_t* recv_count, void* stream);
/* The same exchange ordered on `stream` itself: RCCL runs the group send/recv on `stream` (no transfer stream, no
 * cross-stream events -- for callers that overlap nothing with it, as the serial sharded step); other transports
 * behave as hdd_comm_post.  hdd_comm_wait(comm, stream) is then a no-op on that stream. */
int hdd_comm_post_direct(hdd_comm* comm, int32_t n_peers, const int32_t* peers, const double* const* d_send,
                         const int64_t* send_count, double* const* d_recv, const int64_t* recv_count, void* stream);
/* make `stream` wait for the receives of the last hdd_comm_post (no host blocking with RCCL) */
int hdd_comm_wait(hdd_comm* comm, void* stream);

typedef struct {
  int64_t n_local, own_begin, own_end, n_ghost, global_first;   /* as hdd_local_info */
  int64_t n_rows, n_cols, nnz;      /* owned rows (nb per owned element), global columns, pattern nnz */
  int32_t rank, nranks, s_begin, s_end, n_peers, nb;
  int64_t n_tiles, n_tiles_interior, n_tiles_boundary;   /* 64-element tiles of the owned elements */
  int64_t halo_send, halo_recv;     /* elements sent / ghost elements received per exchange */
  int64_t halo_faces;               /* faces between an owned and a ghost element */
  int64_t halo_elements;            /* owned elements with a ghost face neighbour (the fixup pass) */
} hdd_shard_info;

/* Rank `rank` of `nranks` owns the subdomains s with owner[s] == rank, which must form one contiguous
 * range (owner == NULL: contiguous near-equal ranges, [n_sub r / nranks, n_sub (r+1) / nranks)).  Builds
 * the rank-local mesh (host work O(owned + ghost elements): the structured grids are implicit, nothing
 * global is materialised), uploads it with the ghost geometry, the halo plan, the device send lists and
 * the interior / halo-boundary 64-element tile lists. */
int hdd_shard_create(hdd_ctx* ctx, const hdd_grid* g, int32_t nranks, int32_t rank, const int32_t* owner,
                     hdd_shard** out);
/* ctx == NULL: a host-only shard (local mesh, halo plan, tile lists; no device arrays) -- what a rank can
 * inspect without a GPU, e.g. to check the halo protocol on CPU ranks (tests/test_distributed.py) */
void hdd_shard_destroy(hdd_shard* sh);
int hdd_shard_get_info(const hdd_shard* sh, hdd_shard_info* out);
/* the halo plan (host copies): peers [n_peers] ascending; send lists = local element indices, peer k's
 * part at [send_prefix[k], send_prefix[k+1]) of send_idx [halo_send] (send_prefix [n_peers+1]); the
 * message from peer k fills ghost columns recv_col0[k] .. recv_col0[k] + (recv_prefix[k+1] - recv_prefix[k])
 * (recv_prefix [n_peers+1], recv_col0 [n_peers]).  Any pointer may be NULL. */
int hdd_shard_halo_lists(const hdd_shard* sh, int32_t* peers, int64_t* send_prefix, int32_t* send_idx,
                         int64_t* recv_prefix, int64_t* recv_col0);
/* the 64-element tiles (relative to own_begin) without / with a ghost face neighbour:
 * interior [n_tiles_interior], boundary [n_tiles_boundary]; either may be NULL */
int hdd_shard_tile_lists(const hdd_shard* sh, int32_t* interior, int32_t* boundary);
/* the shard's device mesh (shard-owned arrays; usable with every hdd_* device call) */
int hdd_shard_mesh(const hdd_shard* sh, hdd_mesh* out);
/* host arrays [n_local]: global element ids; element barycentres [dim][n_local] (coefficient lookup) */
int hdd_shard_global_ids(const hdd_shard* sh, int64_t* global_id);
int hdd_shard_centers(const hdd_shard* sh, double* centers);
/* device pattern of the owned rows (global columns) into caller buffers d_row_ptr [n_rows+1],
 * d_col [nnz], d_elem_ptr [own_end-own_begin+1]; synchronises `stream` */
int hdd_shard_pattern_fill(hdd_ctx* ctx, const hdd_shard* sh, int64_t* d_row_ptr, int32_t* d_col,
                           int64_t* d_elem_ptr, void* stream);

enum {
  HDD_SHARD_NO_OVERLAP = 1,     /* exchange, then assemble every tile (the default on Q1 shards; P1 shards overlap
                                   the assembly with the halo) */
  HDD_SHARD_HALO_GEOMETRY = 2,  /* also send the ghost vertex coordinates (default: geometry is rank-local) */
  HDD_SHARD_NO_HALO = 4,        /* ghost columns already valid (static coefficients): no exchange at all */
  HDD_SHARD_NO_TRANSFER = 8,    /* timing studies only: pack and split tile launches as in an exchange, one
                                   loopback kernel instead of the transfer -- the unpack, reading the send buffer
                                   (a copy per peer first when send and receive counts differ) (comm may be NULL; the
                                   ghost columns receive the rank's own send buffers, i.e. wrong values) -- an
                                   upper bound of the GPU-side cost of the sharded step */
  HDD_SHARD_SPLIT_TILES = 16,   /* overlap by tiles: interior tiles during the exchange, the tiles with a
                                   ghost-adjacent element after it -- the default for P1 shards with two peers;
                                   other P1 shards default to every tile during the exchange and the ghost-adjacent
                                   ELEMENTS again, off-stream, in place (HDD_SHARD_FIX_INPLACE); Q1 shards to the
                                   serial step (HDD_SHARD_NO_OVERLAP; measured fastest) */
  HDD_SHARD_FIX_INLINE = 32,    /* study (round 3 A/B): the ghost-adjacent elements recomputed on `stream` after
                                   the wait (default: on the transfer stream right after the receives, beside the
                                   assembly) */
  HDD_SHARD_FIX_SCATTER = 64,   /* the off-stream fixup into a side buffer, copied into place by one kernel after the
                                   join (the assembly's tiles store every row block; Q1: a value-major buffer, one
                                   full-range half-image launch beside the element pass) */
  HDD_SHARD_FIX_INPLACE = 128,  /* the off-stream fixup in place, the assembly's tiles skip those row blocks (a SKIP
                                   launch; Q1: the pack on `stream` ahead of it): the default on P1 end ranks */
  HDD_SHARD_LAUNCH_LAST = 256   /* ablation builds only (round 3's order, measured and rejected): with the in-place
                                   fixup, enqueue the full-range launch after the halo work instead of before it;
                                   the product library ignores it */
};
/* One sharded assembly step -- the LHS of BlockSWIPDG::init() for the owned subdomains: pack the halo
 * records (per-element tensor / kappa rows, [+ coordinates]) of the elements the peers need -> post the
 * exchange, one message per (peer, halo row), received straight into the ghost columns (the ghosts of one
 * owner are contiguous, recv_col0) -> every tile except the row blocks that read a ghost column; those
 * elements (hdd_shard_info.halo_elements of them, one lane each) are computed on
 * the transfer stream as soon as their halo has landed, concurrently with the assembly, whose tiles leave those
 * row blocks to them -> join.  The per-element arrays
 * of `kappa` / `tensor` must span n_local columns: their owned columns are read and their GHOST COLUMNS ARE
 * WRITTEN by the receives.  comm may be NULL when the shard has no peers. */
int hdd_block_assemble_sharded(hdd_ctx* ctx, hdd_shard* sh, hdd_comm* comm, const hdd_scalar_fn* kappa,
                               int32_t n_comp, const hdd_tensor_fn* tensor, const hdd_swipdg_params* params,
                               const hdd_csr* pattern, double* const* d_vals, uint32_t flags, void* stream);

/* Watchdog of the sharded step (ABI 8).  A lost or stalled peer shows as a step that never completes on the device
 * (RCCL waits inside its kernels), so instead of blocking in a device synchronize a rank can poll the events of its
 * last step with a deadline and report where it stopped.  Stages in pipeline order: */
enum {
  HDD_STAGE_COMPLETE = 0,
  HDD_STAGE_PACK = 1,       /* the halo pack kernel (the event the transfer starts from) */
  HDD_STAGE_EXCHANGE = 2,   /* the group send / recv with the halo peers */
  HDD_STAGE_ELEMENTS = 3,   /* the ghost-adjacent element pass behind the receives */
  HDD_STAGE_ASSEMBLY = 4    /* the tile launch(es) and the join on `stream` (up to the last hdd_block_step_mark) */
};
/* record the marker event on `stream` (after the steps to watch) */
int hdd_block_step_mark(hdd_shard* sh, void* stream);
/* non-blocking: *stage = the first stage of the last step (and the marker) whose event has not completed */
int hdd_block_step_query(hdd_shard* sh, int32_t* stage);
const char* hdd_block_stage_name(int32_t stage);
/* mark, then poll until every stage has completed or timeout_s has passed: HDD_ERR_TIMEOUT with a message naming
 * the rank, the stage and the halo peers (hdd_last_error) */
int hdd_block_step_sync(hdd_shard* sh, void* stream, double timeout_s);
/* Error injection (tests of the watchdog): the next hdd_comm_post of `rank` on this hub publishes sends that complete
 * only when hdd_device_hub_release() opens a device-side gate, or after max_seconds (a one-wave kernel polling a
 * host word; it always ends) -- a peer whose sends do not arrive. */
int hdd_device_hub_stall(hdd_device_hub* hub, int32_t rank, double max_seconds);
int hdd_device_hub_release(hdd_device_hub* hub);

#ifdef __cplusplus
}
#endif
#endif /* HDD_H */
