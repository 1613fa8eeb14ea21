// Geometry-layout microbenchmark for the C2 kernel: the production element-major coordinates (6 doubles per
// triangle, the neighbour's opposite vertex gathered from them) against vertex-indexed geometry (3 int32
// vertex ids per triangle + a shared (x, y) vertex array; the neighbour's opposite vertex through its id),
// on the real 3200 x 640 Kuhn structure (element 2 (j nx + i) + t, x fastest), the production tile
// schedule, order [own t+1][compute t][gathers t+1][stores t] and an 18 KB image per 64-element tile.
// Build: hipcc -O3 --offload-arch=gfx950 vgeom.hip -o vgeom
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <cstdio>
#include <vector>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));
constexpr int RB = 36, IMG = 64 * RB, STORES = (IMG / 2 + 63) / 64;

struct Args {
  const ivec4* vf4;       // [n] (v0, v1, v2, finfo)
  const ivec4* nb4;       // [n] (nb0, nb1, nb2, 0)
  const double* tiled;    // [ntiles][7][64] doubles: X0 Y0 X1 Y1 X2 Y2 k
  const int* tiledi;      // [ntiles][4][64] ints: nb0 nb1 nb2 finfo
  const double* coords;   // [6][n] element-major
  const int* vid;         // [3][n]
  const dvec2* xy;        // [nv]
  const int* nbr;         // [3][n]
  const unsigned* finfo;  // [n]
  const double* tper;     // [n]
  double* out;
  long n, ntiles;
};

__device__ __forceinline__ void sched(long ntiles, long& t, long& t_end, long& step)
{
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  t = (ntiles * x) / 8 + w; t_end = (ntiles * (x + 1)) / 8; step = gx;
}
__device__ __forceinline__ void store_tile(const Args& a, long t, const double* lds, int lane)
{
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(a.out + t * IMG, (short)0, IMG * 8, 0x00020000);
#pragma unroll
  for (int k = 0; k < STORES; ++k) {
    const int idx = 2 * (lane + 64 * k);
    const dvec2 v = *reinterpret_cast<const dvec2*>(lds + (idx < IMG ? idx : 0));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, idx * 8, 0, 2);
  }
}
__device__ __forceinline__ int opp(unsigned fi, int f) { return 3 - 1 - int((fi >> (4 * f)) & 1u); }   // 1 or 2

// ---- element-major (production) ----
struct OwnE { double X[3], Y[3], k; int nb[3]; unsigned fi; };
struct GatE { double Ox[3], Oy[3], kn[3]; };
__device__ __forceinline__ void own_e(const Args& a, long e, OwnE& o)
{
#pragma unroll
  for (int v = 0; v < 3; ++v) { o.X[v] = a.coords[2 * v * a.n + e]; o.Y[v] = a.coords[(2 * v + 1) * a.n + e]; }
#pragma unroll
  for (int f = 0; f < 3; ++f) o.nb[f] = a.nbr[f * a.n + e];
  o.fi = a.finfo[e]; o.k = a.tper[e];
}
__device__ __forceinline__ void gat_e(const Args& a, long e, const OwnE& o, GatE& g)
{
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const long m = o.nb[f] >= 0 ? o.nb[f] : e;
    const int to = opp(o.fi, f);
    g.Ox[f] = a.coords[2 * to * a.n + m]; g.Oy[f] = a.coords[(2 * to + 1) * a.n + m]; g.kn[f] = a.tper[m];
  }
}
__device__ __forceinline__ void comp(const double* X, const double* Y, double k, const double* Ox, const double* Oy,
                                     const double* kn, double* img)
{
  double s[9];
#pragma unroll
  for (int f = 0; f < 3; ++f) { s[3 * f] = X[f] * Ox[f]; s[3 * f + 1] = Y[f] * Oy[f]; s[3 * f + 2] = k * kn[f]; }
#pragma unroll
  for (int j = 0; j < RB; ++j) img[j] = s[j % 9] + double(j);
}
__global__ void __launch_bounds__(64, 1) elem_major(const Args a)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  long t, t_end, step; sched(a.ntiles, t, t_end, step);
  if (t >= t_end) return;
  OwnE o; GatE g;
  own_e(a, t * 64 + lane, o); gat_e(a, t * 64 + lane, o, g);
  for (;;) {
    const bool more = t + step < t_end; const long tn = more ? t + step : t;
    OwnE on; own_e(a, tn * 64 + lane, on);
    comp(o.X, o.Y, o.k, g.Ox, g.Oy, g.kn, lds + lane * RB);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    GatE gn; gat_e(a, tn * 64 + lane, on, gn);
    store_tile(a, t, lds, lane);
    if (!more) break;
    t = tn; o = on; g = gn;
  }
}

// ---- element-major, tile-blocked (AoSoA): every per-element row of a tile in one contiguous block ----
__device__ __forceinline__ long tb(long e, int row, int rows) { return ((e >> 6) * rows + row) * 64 + (e & 63); }
__device__ __forceinline__ void own_t(const Args& a, long e, OwnE& o)
{
#pragma unroll
  for (int v = 0; v < 3; ++v) { o.X[v] = a.tiled[tb(e, 2 * v, 7)]; o.Y[v] = a.tiled[tb(e, 2 * v + 1, 7)]; }
  o.k = a.tiled[tb(e, 6, 7)];
#pragma unroll
  for (int f = 0; f < 3; ++f) o.nb[f] = a.tiledi[tb(e, f, 4)];
  o.fi = unsigned(a.tiledi[tb(e, 3, 4)]);
}
__device__ __forceinline__ void gat_t(const Args& a, long e, const OwnE& o, GatE& g)
{
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const long m = o.nb[f] >= 0 ? o.nb[f] : e;
    const int to = opp(o.fi, f);
    g.Ox[f] = a.tiled[tb(m, 2 * to, 7)]; g.Oy[f] = a.tiled[tb(m, 2 * to + 1, 7)]; g.kn[f] = a.tiled[tb(m, 6, 7)];
  }
}
__global__ void __launch_bounds__(64, 1) elem_tiled(const Args a)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  long t, t_end, step; sched(a.ntiles, t, t_end, step);
  if (t >= t_end) return;
  OwnE o; GatE g;
  own_t(a, t * 64 + lane, o); gat_t(a, t * 64 + lane, o, g);
  for (;;) {
    const bool more = t + step < t_end; const long tn = more ? t + step : t;
    OwnE on; own_t(a, tn * 64 + lane, on);
    comp(o.X, o.Y, o.k, g.Ox, g.Oy, g.kn, lds + lane * RB);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    GatE gn; gat_t(a, tn * 64 + lane, on, gn);
    store_tile(a, t, lds, lane);
    if (!more) break;
    t = tn; o = on; g = gn;
  }
}

// ---- vertex-indexed ----
struct OwnV { int v[3]; int nb[3]; unsigned fi; double k; };
struct Gat1 { dvec2 P[3]; int ov[3]; double kn[3]; };   // own vertex coords, neighbour opposite vertex id, kappa
struct Gat2 { dvec2 O[3]; };
__device__ __forceinline__ void own_v(const Args& a, long e, OwnV& o)
{
#pragma unroll
  for (int v = 0; v < 3; ++v) o.v[v] = a.vid[v * a.n + e];
#pragma unroll
  for (int f = 0; f < 3; ++f) o.nb[f] = a.nbr[f * a.n + e];
  o.fi = a.finfo[e]; o.k = a.tper[e];
}
__device__ __forceinline__ void gat1(const Args& a, long e, const OwnV& o, Gat1& g)
{
#pragma unroll
  for (int v = 0; v < 3; ++v) g.P[v] = a.xy[o.v[v]];
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const long m = o.nb[f] >= 0 ? o.nb[f] : e;
    g.ov[f] = a.vid[opp(o.fi, f) * a.n + m]; g.kn[f] = a.tper[m];
  }
}
__device__ __forceinline__ void gat2(const Args& a, const Gat1& g1, Gat2& g)
{
#pragma unroll
  for (int f = 0; f < 3; ++f) g.O[f] = a.xy[g1.ov[f]];
}
__global__ void __launch_bounds__(64, 1) vertex_indexed(const Args a)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  long t, t_end, step; sched(a.ntiles, t, t_end, step);
  if (t >= t_end) return;
  OwnV o; Gat1 g1; Gat2 g2;
  own_v(a, t * 64 + lane, o); gat1(a, t * 64 + lane, o, g1); gat2(a, g1, g2);
  for (;;) {
    const bool more = t + step < t_end; const long tn = more ? t + step : t;
    OwnV on; own_v(a, tn * 64 + lane, on);
    double X[3], Y[3], Ox[3], Oy[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) { X[v] = g1.P[v].x; Y[v] = g1.P[v].y; Ox[v] = g2.O[v].x; Oy[v] = g2.O[v].y; }
    comp(X, Y, o.k, Ox, Oy, g1.kn, lds + lane * RB);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    Gat1 g1n; gat1(a, tn * 64 + lane, on, g1n);
    store_tile(a, t, lds, lane);
    Gat2 g2n; gat2(a, g1n, g2n);     // waits for the level-1 gathers (issued before the stores)
    if (!more) break;
    t = tn; o = on; g1 = g1n; g2 = g2n;
  }
}

// ---- vertex-indexed, packed per-element ints (AoS int4): vid + finfo in one 16-B load, nbr in another ----
template <bool NB4>
__device__ __forceinline__ void own_p(const Args& a, long e, OwnV& o)
{
  const ivec4 vf = a.vf4[e];
  o.v[0] = vf.x; o.v[1] = vf.y; o.v[2] = vf.z; o.fi = unsigned(vf.w);
  if constexpr (NB4) {
    const ivec4 nb = a.nb4[e];
    o.nb[0] = nb.x; o.nb[1] = nb.y; o.nb[2] = nb.z;
  } else {
#pragma unroll
    for (int f = 0; f < 3; ++f) o.nb[f] = a.nbr[f * a.n + e];
  }
  o.k = a.tper[e];
}
template <bool NB4>
__global__ void __launch_bounds__(64, 1) vertex_packed(const Args a)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  long t, t_end, step; sched(a.ntiles, t, t_end, step);
  if (t >= t_end) return;
  OwnV o; Gat1 g1; Gat2 g2;
  own_p<NB4>(a, t * 64 + lane, o); gat1(a, t * 64 + lane, o, g1); gat2(a, g1, g2);
  for (;;) {
    const bool more = t + step < t_end; const long tn = more ? t + step : t;
    OwnV on; own_p<NB4>(a, tn * 64 + lane, on);
    double X[3], Y[3], Ox[3], Oy[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) { X[v] = g1.P[v].x; Y[v] = g1.P[v].y; Ox[v] = g2.O[v].x; Oy[v] = g2.O[v].y; }
    comp(X, Y, o.k, Ox, Oy, g1.kn, lds + lane * RB);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    Gat1 g1n; gat1(a, tn * 64 + lane, on, g1n);
    store_tile(a, t, lds, lane);
    Gat2 g2n; gat2(a, g1n, g2n);
    if (!more) break;
    t = tn; o = on; g1 = g1n; g2 = g2n;
  }
}

int main()
{
  const long nx = 3200, ny = 640, n = nx * ny * 2, ntiles = n / 64, nv = (nx + 1) * (ny + 1);
  std::vector<double> coords(6 * n), tper(n);
  std::vector<int> vid(3 * n), nbr(3 * n);
  std::vector<unsigned> fi(n);
  std::vector<dvec2> xy(nv);
  for (long v = 0; v < nv; ++v) xy[v] = dvec2{double(v % (nx + 1)) / nx * 5.0, double(v / (nx + 1)) / ny};
  auto el = [&](long i, long j, int t) -> int { return (i < 0 || j < 0 || i >= nx || j >= ny) ? -1 : int(2 * (j * nx + i) + t); };
  for (long j = 0; j < ny; ++j)
    for (long i = 0; i < nx; ++i)
      for (int t = 0; t < 2; ++t) {
        const long e = 2 * (j * nx + i) + t;
        const long v00 = j * (nx + 1) + i, v10 = v00 + 1, v01 = v00 + nx + 1, v11 = v01 + 1;
        const long vv[3] = {v00, t ? v01 : v10, v11};
        for (int k = 0; k < 3; ++k) {
          vid[k * n + e] = int(vv[k]);
          coords[2 * k * n + e] = xy[vv[k]].x; coords[(2 * k + 1) * n + e] = xy[vv[k]].y;
        }
        if (!t) { nbr[e] = el(i, j - 1, 1); nbr[n + e] = el(i, j, 1); nbr[2 * n + e] = el(i + 1, j, 1); }
        else { nbr[e] = el(i - 1, j, 0); nbr[n + e] = el(i, j, 0); nbr[2 * n + e] = el(i, j + 1, 0); }
        fi[e] = unsigned(e * 2654435761u) & 0x111u;
        tper[e] = 1.0 + 1e-3 * double(e % 977);
      }
  Args a{};
  a.n = n; a.ntiles = ntiles;
  double *dc, *dt, *dout; int *dv, *dn; unsigned* df; dvec2* dxy;
  hipMalloc(&dc, 6 * n * 8); hipMalloc(&dt, n * 8); hipMalloc(&dv, 3 * n * 4); hipMalloc(&dn, 3 * n * 4);
  hipMalloc(&df, n * 4); hipMalloc(&dxy, nv * 16); hipMalloc(&dout, ntiles * IMG * 8);
  hipMemcpy(dc, coords.data(), 6 * n * 8, hipMemcpyHostToDevice); hipMemcpy(dt, tper.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dv, vid.data(), 3 * n * 4, hipMemcpyHostToDevice); hipMemcpy(dn, nbr.data(), 3 * n * 4, hipMemcpyHostToDevice);
  hipMemcpy(df, fi.data(), n * 4, hipMemcpyHostToDevice); hipMemcpy(dxy, xy.data(), nv * 16, hipMemcpyHostToDevice);
  std::vector<double> tiled(size_t(ntiles) * 7 * 64);
  std::vector<int> tiledi(size_t(ntiles) * 4 * 64);
  for (long e = 0; e < n; ++e) {
    const long T = e >> 6, l = e & 63;
    for (int r = 0; r < 6; ++r) tiled[(T * 7 + r) * 64 + l] = coords[r * n + e];
    tiled[(T * 7 + 6) * 64 + l] = tper[e];
    for (int f = 0; f < 3; ++f) tiledi[(T * 4 + f) * 64 + l] = nbr[f * n + e];
    tiledi[(T * 4 + 3) * 64 + l] = int(fi[e]);
  }
  double* dtl; int* dti;
  hipMalloc(&dtl, tiled.size() * 8); hipMalloc(&dti, tiledi.size() * 4);
  hipMemcpy(dtl, tiled.data(), tiled.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dti, tiledi.data(), tiledi.size() * 4, hipMemcpyHostToDevice);
  a.tiled = dtl; a.tiledi = dti;
  std::vector<ivec4> vf4(n), nb4(n);
  for (long e = 0; e < n; ++e) {
    vf4[e] = ivec4{vid[e], vid[n + e], vid[2 * n + e], int(fi[e])};
    nb4[e] = ivec4{nbr[e], nbr[n + e], nbr[2 * n + e], 0};
  }
  ivec4 *dvf4, *dnb4;
  hipMalloc(&dvf4, n * 16); hipMalloc(&dnb4, n * 16);
  hipMemcpy(dvf4, vf4.data(), n * 16, hipMemcpyHostToDevice); hipMemcpy(dnb4, nb4.data(), n * 16, hipMemcpyHostToDevice);
  a.vf4 = dvf4; a.nb4 = dnb4;
  a.coords = dc; a.tper = dt; a.vid = dv; a.nbr = dn; a.finfo = df; a.xy = dxy; a.out = dout;
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto time = [&](const char* name, auto launch) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.4f ms\n", name, ms / 20); fflush(stdout);
  };
  // the three layouts compute the same images: compare the outputs bit for bit
  std::vector<double> o1(ntiles * IMG), o2(ntiles * IMG);
  hipLaunchKernelGGL(elem_major, dim3(cus * 8), dim3(64), 0, 0, a); hipDeviceSynchronize();
  hipMemcpy(o1.data(), dout, o1.size() * 8, hipMemcpyDeviceToHost);
  for (int v = 0; v < 4; ++v) {
    hipMemset(dout, 0, o2.size() * 8);
    if (v == 0) hipLaunchKernelGGL(vertex_indexed, dim3(cus * 8), dim3(64), 0, 0, a);
    else if (v == 1) hipLaunchKernelGGL(elem_tiled, dim3(cus * 8), dim3(64), 0, 0, a);
    else if (v == 2) hipLaunchKernelGGL(vertex_packed<false>, dim3(cus * 8), dim3(64), 0, 0, a);
    else hipLaunchKernelGGL(vertex_packed<true>, dim3(cus * 8), dim3(64), 0, 0, a);
    hipDeviceSynchronize();
    hipMemcpy(o2.data(), dout, o2.size() * 8, hipMemcpyDeviceToHost);
    long diff = 0;
    for (size_t i = 0; i < o1.size(); ++i) diff += o1[i] != o2[i];
    printf("variant %d outputs differing from element-major: %ld of %zu\n", v, diff, o1.size());
  }
  for (int rep = 0; rep < 3; ++rep)
    for (int wg : {4, 8}) {
      char nm[64];
      snprintf(nm, sizeof nm, "element-major wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL(elem_major, dim3(cus * wg), dim3(64), 0, 0, a); });
      snprintf(nm, sizeof nm, "tile-blocked wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL(elem_tiled, dim3(cus * wg), dim3(64), 0, 0, a); });
      snprintf(nm, sizeof nm, "vx packed vid+fi wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL(vertex_packed<false>, dim3(cus * wg), dim3(64), 0, 0, a); });
      snprintf(nm, sizeof nm, "vx packed vid+fi, nb wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL(vertex_packed<true>, dim3(cus * wg), dim3(64), 0, 0, a); });
      snprintf(nm, sizeof nm, "vertex-indexed wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL(vertex_indexed, dim3(cus * wg), dim3(64), 0, 0, a); });
    }
  return 0;
}
